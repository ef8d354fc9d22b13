"""Argument validation at the Python mirror (the kernels take raw pointers) and the ordering of
host-pointer calls after device-resident calls on one shard."""
import numpy as np
import pytest

from glint_amd import PartialMatrix, PartialVector, RangePartition
from oracle import oracle as O

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
