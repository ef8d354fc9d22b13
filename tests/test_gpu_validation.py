"""Argument validation at the Python mirror (the kernels take raw pointers) and the ordering of
host-pointer calls after device-resident calls on one shard."""
import numpy as np
import pytest

from glint_amd import PartialMatrix, PartialVector, RangePartition
from oracle import oracle as O
import glint_amd._native as N

pytestmark = pytest.mark.gpu


def test_device_argument_checks(gpu):
    import torch
    dev = torch.device("cuda", gpu)
    with PartialVector(RangePartition(0, 0, 1000), "double", gpu) as sh:
        k = torch.arange(10, dtype=torch.int64, device=dev)
        with pytest.raises(TypeError):
            sh.update(k, torch.ones(10, dtype=torch.float32, device=dev))      # wrong value type
        with pytest.raises(TypeError):
            sh.update(k.to(torch.int32), torch.ones(10, dtype=torch.float64, device=dev))
        with pytest.raises(ValueError):
            sh.update(k, torch.ones(9, dtype=torch.float64, device=dev))       # short values
        with pytest.raises(ValueError):
            sh.get(k, out=torch.empty(9, dtype=torch.float64, device=dev))     # undersized out
        with pytest.raises(TypeError):
            sh.get(k, out=torch.empty(10, dtype=torch.float32, device=dev))
        with pytest.raises(TypeError):
            sh.update(k, np.ones(10))                                          # host values with device keys
        assert sh.get(k).sum().item() == 0.0
    with PartialMatrix(RangePartition(0, 0, 100), 16, "long", gpu) as sh:
        r = torch.zeros(10, dtype=torch.int64, device=dev)
        c = torch.zeros(10, dtype=torch.int32, device=dev)
        v = torch.ones(10, dtype=torch.int64, device=dev)
        with pytest.raises(ValueError):
            sh.update(r, c[:5], v)                                             # short cols
        with pytest.raises(TypeError):
            sh.update(r, c.to(torch.int64), v)
        with pytest.raises(ValueError):
            sh.getRows(r, out=torch.empty((10, 15), dtype=torch.int64, device=dev))
        sh.update(r, c, v)
        assert sh.get(r[:1], c[:1]).item() == 10


def test_host_argument_checks(gpu):
    with PartialVector(RangePartition(0, 0, 1000), "float", gpu) as sh:
        with pytest.raises(ValueError):
            sh.update([1, 2, 3], [1.0, 2.0])
        with pytest.raises(ValueError):
            sh.get([1, 2, 3], out=np.empty(3, np.float64))                     # wrong out dtype
        with pytest.raises(ValueError):
            sh.get([1, 2, 3], out=np.empty(2, np.float32))                     # undersized out
        out = np.empty(3, np.float32)
        assert sh.get([1, 2, 3], out=out) is out
    with PartialMatrix(RangePartition(0, 0, 10), 4, "int", gpu) as sh:
        with pytest.raises(ValueError):
            sh.get([1, 2], [0])
        with pytest.raises(ValueError):
            sh.getRows([1, 2], out=np.empty((2, 3), np.int32))


def test_host_calls_order_after_device_calls(gpu):
    """update(tensor, sync=False) then host-pointer pushes and pulls on the same shard: the host
    calls (private stream) wait for the device call (caller's stream) -- no lost updates, and the
    pull sees every push."""
    import torch
    dev = torch.device("cuda", gpu)
    n = 1 << 22
    ref = O.OracleVector(O.part_range(0, n), O.O_I64)
    rng = np.random.default_rng(1)
    with PartialVector(RangePartition(0, 0, n), "long", gpu) as sh:
        for it in range(4):
            kd = rng.integers(0, n, n).astype(np.int64)  # large unordered device push (slow path)
            vd = rng.integers(-9, 9, n).astype(np.int64)
            sh.update(torch.from_numpy(kd).to(dev), torch.from_numpy(vd).to(dev), sync=False)
            kh = rng.integers(0, n, 5000).astype(np.int64)
            vh = rng.integers(-9, 9, kh.size).astype(np.int64)
            sh.update(kh, vh)                                   # host push right behind it
            ref.update(kd, vd)
            ref.update(kh, vh)
            q = rng.integers(0, n, 3000).astype(np.int64)
            np.testing.assert_array_equal(sh.get(q), ref.get(q)[0])
        sh.sync(torch.cuda.current_stream(dev).cuda_stream)
        np.testing.assert_array_equal(sh.to_numpy(), ref.data)


# ---- the library's environment knobs: each non-default branch (DESIGN.md §8 lists them) ----------------
def test_host_prof_knob(gpu, monkeypatch, capfd):
    """GLINT_HOST_PROF=1: a shard counts its lock waits, launches, retire waits and copies, and prints
    them as one `glint_host_prof {...}` JSON line on stderr when it is destroyed (the loopback harness's
    --cpu-stats rows read it). Without it nothing is printed."""
    import json
    from glint_amd import PartialVector, RangePartition
    part = RangePartition(0, 0, 4096)
    keys = np.arange(1000, dtype=np.int64)
    for on in (True, False):
        if on:
            monkeypatch.setenv("GLINT_HOST_PROF", "1")
        else:
            monkeypatch.delenv("GLINT_HOST_PROF", raising=False)
        N.reload_env()
        with PartialVector(part, "long", gpu) as sh:
            t = sh.push_async(keys, np.ones(keys.size, np.int64))
            sh.wait(t)
            assert (sh.get(keys) == 1).all()
        err = capfd.readouterr().err
        lines = [ln for ln in err.splitlines() if ln.startswith("glint_host_prof ")]
        if on:
            assert len(lines) == 1, err
            d = json.loads(lines[0][len("glint_host_prof "):])
            assert d["device"] == gpu and d["locks"] >= 2 and d["launches"] >= 1 and d["tickets"] >= 1
        else:
            assert not lines


@pytest.mark.parametrize("stage_max", ["0", "64"])
def test_pinned_stage_max_knob(gpu, monkeypatch, stage_max):
    """GLINT_PINNED_STAGE_MAX (bytes): host arrays up to it are staged through the shard's pinned buffer
    (one DMA per call), larger ones go straight from pageable memory. At 0 / 64 B every call of this test
    takes the pageable path that only messages above the 2 MiB default take; results are the oracle's."""
    from glint_amd import PartialMatrix, PartialVector, RangePartition
    from oracle import oracle as O
    monkeypatch.setenv("GLINT_PINNED_STAGE_MAX", stage_max)
    N.reload_env()
    rng = np.random.default_rng(3)
    size = 50_000
    ref = O.OracleVector(O.part_range(100, 100 + size), O.CODE["long"])
    with PartialVector(RangePartition(0, 100, 100 + size), "long", gpu) as sh:
        for n in (1, 1000, 70_000):
            k = rng.integers(100, 100 + size, n).astype(np.int64)
            v = rng.integers(-99, 99, n).astype(np.int64)
            sh.update(k, v)
            assert ref.update(k, v) == -1
        q = rng.integers(100, 100 + size, 5000).astype(np.int64)
        np.testing.assert_array_equal(sh.get(q), ref.get(q)[0])
    mref = O.OracleMatrix(O.part_range(0, 64), 33, O.CODE["double"])
    with PartialMatrix(RangePartition(0, 0, 64), 33, "double", gpu) as sh:
        r = rng.integers(0, 64, 3000).astype(np.int64)
        c = rng.integers(0, 33, 3000).astype(np.int32)
        v = rng.uniform(-1, 1, 3000)
        sh.update(r, c, v, deterministic=True)
        assert mref.update(r, c, v) == -1
        np.testing.assert_array_equal(sh.getRows(np.arange(64)), mref.data)
