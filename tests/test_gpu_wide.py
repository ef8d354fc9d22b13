"""Pushes at the north star's own scale, past the 4 GiB line of the binned pipeline's buffers.

A binned push of n records keeps a u32 address and an LDS-width value per record in its partition
buffers; from n * sizeof(value) >= 2^32 (Double / Long / Float from 2^29 records, Int from 2^30) the
partition kernels store through 64-bit addresses (WideOut, glint_amd/csrc/glint_bin.hip) instead of
one 32-bit buffer window. These tests drive that path through every way a push reaches it -- the
UNORDERED hint, the adaptive switch's whole-push bin, and a validating gated push -- and a matrix
shard of 2^32 elements, which the binned path's u32 element addresses exclude (it takes check +
apply + the LDS-hash scatter, 64-bit addressed).

Expected values come from torch's own index_add_ on the GPU (PartialVector.scala:35-43 /
PartialMatrix.scala:74-83 restated as one scatter-add over the same records): Long and Int are
bit-exact (wrapping sums are associative); Double and Float are within 1e-9 of each element's sum of
magnitudes (sum |v| over its records, the accuracy every summation order has -- a lost or doubled
record, an error of a whole |v|, cannot pass). The C oracle would take minutes per push at this size;
the same kernels are pinned against it at cfg3's full size (tests/test_gpu_fullsize.py).
"""
import numpy as np
import pytest

from glint_amd import PartialMatrix, PartialVector, RangePartition
import glint_amd._native as N

pytestmark = pytest.mark.gpu

SHARD = 1 << 30          # the north star's 2^30-key vector
NREC = (1 << 29) + (1 << 20)  # past 2^29 records: 8-byte partial sums exceed 2^32 bytes


def _keys(torch, d, n, seed):
    """Uniform keys over the shard plus a Zipf-like hot head (the dedup / hot front ends see duplicates)."""
    g = torch.Generator(device=d)
    g.manual_seed(seed)
    k = torch.randint(0, SHARD, (n,), dtype=torch.int64, device=d, generator=g)
    hot = torch.randint(0, 4096, (n // 8,), dtype=torch.int64, device=d, generator=g) * 7919
    k[: hot.numel()] = hot
    perm = torch.randperm(n, device=d, generator=g)
    return k[perm], g


def _vals(torch, d, dtype, n, g):
    if dtype in ("long", "int"):
        tdt = torch.int64 if dtype == "long" else torch.int32
        lim = 1 << 40 if dtype == "long" else 1 << 20
        return torch.randint(-lim, lim, (n,), dtype=tdt, device=d, generator=g)
    tdt = torch.float64 if dtype == "double" else torch.float32
    return (torch.rand(n, dtype=torch.float64, device=d, generator=g) * 2 - 1).to(tdt)


def _launches(sh, kid):
    import ctypes as C
    ms, cnt = C.c_double(), C.c_int64()
    N.load().glint_prof_read(sh.handle, kid, C.byref(ms), C.byref(cnt))
    return cnt.value


def _check(torch, got, ref, mag, exact):
    if exact:
        assert torch.equal(got, ref), f"{int((got != ref).sum())} elements differ"
    else:
        err = (got.double() - ref.double()).abs()
        bad = err > 1e-9 * mag
        assert not bool(bad.any()), f"{int(bad.sum())} elements off by more than 1e-9 of sum |v|"


@pytest.mark.parametrize("dtype,front", [("long", None), ("double", None), ("double", "hot"), ("float", None),
                                         ("int", None)])
def test_wide_binned_push(gpu, monkeypatch, dtype, front):
    """2^29 + 2^20 records (Int: 2^30 + 2^20) into a 2^30-key shard, pushed three ways: with the
    UNORDERED hint (first push: the dedup probe), by the adaptive switch (the checked path's scatter,
    then a whole-push bin from the latched tail), and again with the hint (the front end the probe
    chose, or the hot-split front end forced)."""
    import torch
    if front is not None:
        monkeypatch.setenv("GLINT_BIN_FRONT", front)
    monkeypatch.delenv("GLINT_BINNED", raising=False)
    N.reload_env()
    d = torch.device("cuda", gpu)
    n = NREC if dtype != "int" else (1 << 30) + (1 << 20)
    keys, g = _keys(torch, d, n, 7)
    vals = _vals(torch, d, dtype, n, g)
    exact = dtype in ("long", "int")
    acc = torch.int64 if dtype == "long" else torch.int32 if dtype == "int" else torch.float64
    ref = torch.zeros(SHARD, dtype=acc, device=d)
    ref.index_add_(0, keys, vals.to(acc))
    mag = None
    if not exact:
        mag = torch.zeros(SHARD, dtype=torch.float64, device=d)
        mag.index_add_(0, keys, vals.double().abs())
    # Float: the binned pushes only (the checked path's atomic scatter rounds a hot element's float sum
    # once per 2048-record chunk; a binned push once per apply unit / hot-table flush)
    hints = (True, True) if dtype == "float" else (True, False, False, True)
    with PartialVector(RangePartition(0, 0, SHARD), dtype, gpu) as sh:
        N.load().glint_prof_enable(sh.handle, 1)
        for unordered in hints:  # (False twice: check + apply + scatter with no history, then the
            sh.update(keys, vals, unordered=unordered)  # latched tail's whole-push bin)
        # every push but the one with no history went through the binned pipeline (its wide stores)
        assert _launches(sh, N.GLINT_K_PUSH_BINNED) == (3 if False in hints else 2)
        got = sh.get(torch.arange(SHARD, dtype=torch.int64, device=d))
    ref *= len(hints)
    if mag is not None:
        mag *= len(hints)
    if dtype == "float":  # float adds round at every flush: a few hundred roundings per element at most
        err = (got.double() - ref).abs()
        bad = err > 2e-5 * mag
        assert not bool(bad.any()), f"{int(bad.sum())} elements off"
    else:
        _check(torch, got, ref.to(got.dtype) if exact else ref, mag, exact)


def test_wide_validating_gated_push(gpu, monkeypatch):
    """A validating gated push past 4 GiB: the count pass validates the binned tail; a batch with one
    key outside the shard applies nothing, a clean one is the plain push."""
    import torch
    monkeypatch.delenv("GLINT_BINNED", raising=False)
    N.reload_env()
    d = torch.device("cuda", gpu)
    keys, g = _keys(torch, d, NREC, 11)
    vals = torch.randint(-(1 << 30), 1 << 30, (NREC,), dtype=torch.int64, device=d, generator=g)
    bad = keys.clone()
    first = NREC - 12345
    bad[first] = SHARD + 3
    ref = torch.zeros(SHARD, dtype=torch.int64, device=d)
    gate = torch.full((1,), 777, dtype=torch.int64, device=d)
    with PartialVector(RangePartition(0, 0, SHARD), "long", gpu) as sh:
        N.load().glint_prof_enable(sh.handle, 1)
        for i, (batch, ok) in enumerate(((keys, True), (keys, True), (bad, False), (keys, True))):
            sh.update(batch, vals, gate=gate, validate=True)
            w = int(gate.cpu()[0])
            if ok:
                assert w == 0
                ref.index_add_(0, keys, vals)
            else:
                assert ~w == first, (w, first)
            # the first push (no history) checks, applies and scatters; the rest are whole-push bins
            # whose count pass validates every record
            assert _launches(sh, N.GLINT_K_PUSH_BINNED) == i
        got = sh.get(torch.arange(SHARD, dtype=torch.int64, device=d))
    assert torch.equal(got, ref)


@pytest.mark.parametrize("unordered", [True, False])
def test_matrix_shard_past_2p32_elements(gpu, unordered):
    """A (2^23 + 2^12) x 512 Double matrix shard (2^32 + 2^21 elements, 32 GiB): element addresses pass
    32 bits, so the push takes the 64-bit addressed scatter (and check + apply before it without the
    hint). Rows Zipf-like over the whole shard, so records land on both sides of element 2^32."""
    import torch
    d = torch.device("cuda", gpu)
    rows_n, cols_n, n = (1 << 23) + (1 << 12), 512, 1 << 26
    g = torch.Generator(device=d)
    g.manual_seed(5)
    u = torch.rand(n, dtype=torch.float64, device=d, generator=g)
    r = (torch.floor(torch.pow(float(rows_n), u)).to(torch.int64) - 1).clamp_(0, rows_n - 1)
    r = (r * 2654435761) % rows_n  # scatter the hot rows over the shard
    c = torch.randint(0, cols_n, (n,), dtype=torch.int32, device=d, generator=g)
    v = torch.rand(n, dtype=torch.float64, device=d, generator=g) * 2 - 1
    start = 3 * rows_n  # partition 3 of RangePartitioner(8, 8 * rows_n)
    flat = r * cols_n + c.to(torch.int64)
    assert int(flat.max()) >= 1 << 32 and int(flat.min()) < 1 << 31
    with PartialMatrix(RangePartition(3, start, start + rows_n), cols_n, "double", gpu) as sh:
        for _ in range(2):
            sh.update(r + start, c, v, unordered=unordered)
        ref = torch.zeros(rows_n * cols_n, dtype=torch.float64, device=d)
        ref.index_add_(0, flat, v)
        ref *= 2
        mag = torch.zeros(rows_n * cols_n, dtype=torch.float64, device=d)
        mag.index_add_(0, flat, v.abs())
        mag *= 2
        step = 1 << 19  # compare in row blocks of 2 GiB (the pulled rows beside the reference)
        for r0 in range(0, rows_n, step):
            r1 = min(rows_n, r0 + step)
            got = sh.getRows(torch.arange(start + r0, start + r1, dtype=torch.int64, device=d)).reshape(-1)
            sl = slice(r0 * cols_n, r1 * cols_n)
            _check(torch, got, ref[sl], mag[sl], False)
