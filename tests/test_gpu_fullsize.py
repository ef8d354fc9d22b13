"""Oracle parity at BASELINE.json's full sizes (the configs the bench lines are quoted on).

* cfg3: 2^26 Zipf(1.1) records into a 2^28-key shard, pushed device-resident three times -- the
  first push takes the LDS-hash scatter (no history), the second the binned path by the adaptive
  switch, the third with the UNORDERED hint -- then compared element by element with the C
  oracle's sequential loop (PartialVector.scala:35-43) over the same three pushes.
* cfg5 per GPU: 2^23 Zipf(1.0)-row x uniform-col triplets into a 2^17 x 512 shard
  (PartialMatrix.scala:74-83), same scheme.

Long is bit-exact; Double in the default mode is within 1e-9 of each element's sum of magnitudes
(sum |v| over its records: the scale every summation order is accurate to -- n terms in any order are
within ~n eps sum |v|, ~1e-10 here -- so it is far inside the north star's 1e-6 relative, yet a lost or
duplicated record, an error of a whole |v|, cannot pass; it demands exact zeros where nothing was
pushed); Double with GLINT_PUSH_DETERMINISTIC is bit-exact.
Zipf ranks are scattered over the shard by an odd-multiplier bijection of [0, 2^k) (the bench uses
a seeded permutation; the mapping does not matter for parity).
"""
import numpy as np
import pytest

from glint_amd import PartialMatrix, PartialVector, RangePartition
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _scatter(ranks, log2):
    return ((ranks.astype(np.uint64) * np.uint64(0x9E3779B1)) & np.uint64((1 << log2) - 1)).astype(np.int64)


@pytest.fixture(scope="module")
def cfg3():
    rng = np.random.default_rng(42)
    nrec, log2 = 1 << 26, 28
    r = rng.zipf(1.1, size=int(nrec * 1.3))
    r = r[r <= (1 << log2)][:nrec] - 1
    return _scatter(r, log2), rng


@pytest.fixture(scope="module")
def cfg5():
    rng = np.random.default_rng(43)
    nrec, rows = 1 << 23, 1 << 17
    ranks = np.minimum(np.floor(np.power(float(rows), rng.random(nrec))).astype(np.int64) - 1, rows - 1)
    return _scatter(ranks, 17), rng.integers(0, 512, nrec).astype(np.int32), rng


def assert_close_mag(got, want, mag):
    """|got - want| <= 1e-9 * sum |v| per element (see the module docstring)."""
    err = np.abs(got.astype(np.float64) - want.astype(np.float64))
    bad = err > 1e-9 * mag
    assert not bad.any(), f"{int(bad.sum())} elements off by more than 1e-9 of sum |v|"


def _push3(sh, torch, dev, *arrays, deterministic=False):
    t = [torch.from_numpy(a).to(dev) for a in arrays]
    if deterministic:
        sh.update(*t, deterministic=True)
        return 1
    sh.update(*t)                 # no history: the LDS-hash scatter
    sh.update(*t)                 # previous tail was large: the binned path (adaptive switch)
    sh.update(*t, unordered=True)  # the hint
    return 3


@pytest.mark.parametrize("mode", ["long", "double", "double_det"])
def test_cfg3_full_size(gpu, cfg3, mode):
    import torch
    dev = torch.device("cuda", gpu)
    keys, rng = cfg3
    dtype = "long" if mode == "long" else "double"
    if dtype == "long":
        vals = rng.integers(-(1 << 40), 1 << 40, keys.size)
    else:
        vals = rng.uniform(-1, 1, keys.size)
    start = 3 << 28  # the shard of partition 3 of RangePartitioner(8, 2^31)
    part = RangePartition(3, start, start + (1 << 28))
    ref = O.OracleVector(O.part_range(start, start + (1 << 28)), O.CODE[dtype])
    with PartialVector(part, dtype, gpu) as sh:
        reps = _push3(sh, torch, dev, keys + start, vals, deterministic=mode == "double_det")
        got = sh.to_numpy()
    for _ in range(reps):
        assert ref.update(keys + start, vals) == -1
    if mode == "double":
        mag = reps * np.bincount(keys, np.abs(vals), minlength=1 << 28)
        assert_close_mag(got, ref.data, mag)
    else:
        np.testing.assert_array_equal(got, ref.data)


@pytest.mark.parametrize("mode", ["long", "double", "double_det"])
def test_cfg5_slice_full_size(gpu, cfg5, mode):
    import torch
    dev = torch.device("cuda", gpu)
    rows, cols, rng = cfg5
    dtype = "long" if mode == "long" else "double"
    if dtype == "long":
        vals = rng.integers(-(1 << 40), 1 << 40, rows.size)
    else:
        vals = rng.uniform(-1, 1, rows.size)
    start = 5 << 17  # partition 5 of RangePartitioner(8, 2^20) rows
    part = RangePartition(5, start, start + (1 << 17))
    ref = O.OracleMatrix(O.part_range(start, start + (1 << 17)), 512, O.CODE[dtype])
    with PartialMatrix(part, 512, dtype, gpu) as sh:
        reps = _push3(sh, torch, dev, rows + start, cols, vals, deterministic=mode == "double_det")
        got = sh.to_numpy()
    for _ in range(reps):
        assert ref.update(rows + start, cols, vals) == -1
    if mode == "double":
        mag = reps * np.bincount(rows * 512 + cols, np.abs(vals), minlength=(1 << 17) * 512).reshape(1 << 17, 512)
        assert_close_mag(got, ref.data, mag)
    else:
        np.testing.assert_array_equal(got, ref.data)
