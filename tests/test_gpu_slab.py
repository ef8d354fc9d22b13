"""Slabs (glint_shard_create_in): the partitions one server hosts, as views of one allocation.

A view is a shard like any other -- its own RangePartition, key check, stream and error state --
whose elements are rows of the slab. These tests pin the C ABI's contract (include/glint_gpu.h): the
views and the slab see one memory; a slab with views takes device-resident calls only, each ordered
after the views' host-pointer work; views are destroyed first; offsets are checked. The world-1
exchange on top of it (one push on the slab for all partitions) is dist_workers' slab cases. Last, the
other way to push a server's partitions at once: glint_vec_push_dev_shards (one launch sequence over
several separately allocated shards; dist_workers' set case drives it through DistributedBigVector)."""
import numpy as np
import pytest
import torch

from glint_amd.errors import ArrayIndexOutOfBoundsException
from glint_amd.partitioning import RangePartition
from glint_amd.shard import PartialMatrix, PartialVector

pytestmark = pytest.mark.gpu


def _vec_slab(gpu, dtype="long", start=100, rows=1024, nviews=3):
    slab = PartialVector(RangePartition(0, start, start + rows * nviews), dtype, gpu)
    views = [PartialVector.view(slab, RangePartition(j, start + rows * j, start + rows * (j + 1)), rows * j)
             for j in range(nviews)]
    return slab, views


def test_views_and_slab_share_elements(gpu):
    dev = torch.device("cuda", gpu)
    slab, views = _vec_slab(gpu)
    one = lambda n, x: torch.full((n,), x, dtype=torch.int64, device=dev)  # noqa: E731
    views[1].update(torch.arange(1124, 2148, device=dev), one(1024, 1))         # device push on a view
    views[2].update(np.arange(2148, 3172), np.full(1024, 2, np.int64))          # host push on another
    t = views[0].push_async(np.arange(100, 1124), np.full(1024, 5, np.int64))   # enqueued, not waited for
    slab.update(torch.arange(100, 3172, device=dev), one(3072, 10))             # one push on the slab
    views[0].wait(t)
    want = 10 + np.repeat(np.array([5, 1, 2], np.int64), 1024)
    np.testing.assert_array_equal(slab.get(torch.arange(100, 3172, device=dev)).cpu().numpy(), want)
    for j, v in enumerate(views):
        lo = 100 + 1024 * j
        np.testing.assert_array_equal(v.get(np.arange(lo, lo + 1024)), want[1024 * j:1024 * (j + 1)])
    # a view checks its own partition
    with pytest.raises(ArrayIndexOutOfBoundsException):
        views[0].update(np.array([1124]), np.array([1], np.int64))
    for v in views:
        v.destroy()
    slab.destroy()


def test_slab_takes_device_calls_only_while_it_has_views(gpu):
    dev = torch.device("cuda", gpu)
    slab, views = _vec_slab(gpu, nviews=2)
    with pytest.raises(ValueError):
        slab.update(np.array([100]), np.array([1], np.int64))
    with pytest.raises(ValueError):
        slab.get(np.array([100]))
    with pytest.raises(ValueError):
        slab.push_async(np.array([100]), np.array([1], np.int64))
    with pytest.raises(ValueError):
        slab.zero()
    with pytest.raises(ValueError):  # its views read and write its memory
        slab.destroy()
    slab.update(torch.tensor([100], device=dev), torch.tensor([3], dtype=torch.int64, device=dev))
    views[1].destroy()
    with pytest.raises(ValueError):
        slab.destroy()
    views[0].destroy()
    # no views left: a shard like any other again
    slab.update(np.array([100]), np.array([1], np.int64))
    assert slab.get(np.array([100]))[0] == 4
    slab.destroy()


def test_view_offsets_are_checked(gpu):
    slab = PartialVector(RangePartition(0, 0, 4096), "double", gpu)
    with pytest.raises(ValueError):  # 8 bytes into the slab: not 256-byte aligned
        PartialVector.view(slab, RangePartition(0, 0, 10), 1)
    with pytest.raises(ValueError):  # past the slab's end
        PartialVector.view(slab, RangePartition(0, 0, 64), 4096 - 32)
    v = PartialVector.view(slab, RangePartition(0, 0, 64), 32)
    with pytest.raises(ValueError):  # a view of a view
        PartialVector.view(v, RangePartition(0, 0, 32), 0)
    v.destroy()
    slab.destroy()


@pytest.mark.parametrize("unordered", [False, True])
def test_odd_view_writes_stay_inside(gpu, unordered):
    """A 1023-element view followed by a gap element and the next view: dense and unordered pushes
    into the odd-sized view (the slab-wide pair paths) leave the gap and the neighbour untouched."""
    dev = torch.device("cuda", gpu)
    slab = PartialVector(RangePartition(0, 0, 2048), "double", gpu)
    a = PartialVector.view(slab, RangePartition(0, 0, 1023), 0)
    b = PartialVector.view(slab, RangePartition(1, 1024, 2048), 1024)
    k = torch.arange(0, 1023, device=dev)
    if unordered:
        k = k[torch.randperm(1023, device=dev)]
    for _ in range(3):
        a.update(k, torch.ones(1023, dtype=torch.float64, device=dev), unordered=unordered)
    b.update(torch.arange(1024, 2048, device=dev), torch.full((1024,), 7.0, dtype=torch.float64, device=dev))
    for v in (a, b):
        v.destroy()
    got = slab.get(torch.arange(0, 2048, device=dev)).cpu().numpy()
    np.testing.assert_array_equal(got[:1023], np.full(1023, 3.0))
    assert got[1023] == 0.0
    np.testing.assert_array_equal(got[1024:], np.full(1024, 7.0))
    slab.destroy()


def test_matrix_views(gpu):
    """Rows of a 17-column Double slab (row pitch 18 elements = 144 B: views start every 16 rows)."""
    dev = torch.device("cuda", gpu)
    slab = PartialMatrix(RangePartition(0, 0, 64), 17, "double", gpu)
    views = [PartialMatrix.view(slab, RangePartition(j, 16 * j, 16 * (j + 1)), 16 * j) for j in range(4)]
    with pytest.raises(ValueError):  # 8 rows in: 1152 B, not 256-byte aligned
        PartialMatrix.view(slab, RangePartition(9, 8, 16), 8)
    rng = np.random.default_rng(5)
    want = np.zeros((64, 17))
    for j, v in enumerate(views):
        r = rng.integers(16 * j, 16 * (j + 1), 500).astype(np.int64)
        c = rng.integers(0, 17, 500).astype(np.int32)
        x = rng.integers(-50, 50, 500).astype(np.float64)  # small integers: exact in any order
        v.update(torch.from_numpy(r).to(dev), torch.from_numpy(c).to(dev), torch.from_numpy(x).to(dev))
        np.add.at(want, (r, c), x)
    got = slab.getRows(torch.arange(0, 64, device=dev)).cpu().numpy()
    np.testing.assert_array_equal(got, want)
    with pytest.raises(ArrayIndexOutOfBoundsException):  # a view's own column check
        views[2].update(np.array([33]), np.array([17], np.int32), np.array([1.0]))
    for v in views:
        v.destroy()
    slab.destroy()


# ---- several shards in one push (glint_vec_push_dev_shards) --------------------------------------------
def _set_push(shards, keys, vals, gate):
    import ctypes as C
    from glint_amd import _native as N
    hs = (C.c_void_p * len(shards))(*[s.handle for s in shards])
    st = torch.cuda.current_stream(keys.device).cuda_stream
    return N.load().glint_vec_push_dev_shards(hs, len(shards), keys.data_ptr(), vals.data_ptr(), keys.numel(),
                                              gate.data_ptr(), st)


@pytest.mark.parametrize("dtype", ["long", "double"])
def test_set_push_routes_each_record_to_its_shard(gpu, dtype):
    """Three range shards given out of order, with a gap between two ranges: each record lands in the
    shard that holds its key (duplicates summed); a key in the gap or outside applies nothing and the
    gate holds ~(first such record). Long: bit-exact; Double: small integers, exact in any order."""
    dev = torch.device("cuda", gpu)
    ranges = [(5000, 9000), (0, 3000), (3000, 4500)]  # (4500, 5000) belongs to no shard
    shards = [PartialVector(RangePartition(i, a, b), dtype, gpu) for i, (a, b) in enumerate(ranges)]
    tdt = torch.int64 if dtype == "long" else torch.float64
    rng = np.random.default_rng(11)
    k = np.concatenate([rng.integers(0, 4500, 30_000), rng.integers(5000, 9000, 30_000)]).astype(np.int64)
    rng.shuffle(k)
    v = rng.integers(-20, 20, k.size)
    gate = torch.full((1,), 7, dtype=torch.int64, device=dev)
    kt, vt = torch.from_numpy(k).to(dev), torch.from_numpy(v).to(dev).to(tdt)
    for _ in range(2):
        assert _set_push(shards, kt, vt, gate) == 0
    assert _set_push(shards, kt[1:], vt[1:], gate) == 0  # keys 8 B off a 16-B boundary, odd count
    shards[0].sync(torch.cuda.current_stream(dev).cuda_stream)
    assert int(gate.item()) == 0
    want = np.zeros(9000, np.int64)
    np.add.at(want, k, 2 * v)
    np.add.at(want, k[1:], v[1:])
    for sh, (a, b) in zip(shards, ranges):
        got = sh.get(torch.arange(a, b, device=dev)).cpu().numpy()
        np.testing.assert_array_equal(got.astype(np.int64), want[a:b])
    # a key in the gap (record 2) and one past the end (record 4): nothing applied
    bad = torch.tensor([10, 20, 4700, 30, 9000], dtype=torch.int64, device=dev)
    assert _set_push(shards, bad[3:], torch.ones(2, dtype=tdt, device=dev), gate) == 0  # unaligned, bad last
    shards[0].sync(torch.cuda.current_stream(dev).cuda_stream)
    assert int(gate.item()) == ~1
    assert _set_push(shards, bad, torch.ones(5, dtype=tdt, device=dev), gate) == 0
    shards[0].sync(torch.cuda.current_stream(dev).cuda_stream)
    assert int(gate.item()) == ~2
    for sh, (a, b) in zip(shards, ranges):
        np.testing.assert_array_equal(sh.get(torch.arange(a, b, device=dev)).cpu().numpy().astype(np.int64), want[a:b])
    # an empty batch: verdict 0
    gate.fill_(5)
    assert _set_push(shards, torch.zeros(0, dtype=torch.int64, device=dev), torch.zeros(0, dtype=tdt, device=dev),
                     gate) == 0
    torch.cuda.synchronize(dev)
    assert int(gate.item()) == 0
    for sh in shards:
        sh.destroy()


def test_set_push_rejects_bad_sets(gpu):
    from glint_amd import _native as N
    dev = torch.device("cuda", gpu)
    a = PartialVector(RangePartition(0, 0, 100), "double", gpu)
    b = PartialVector(RangePartition(1, 50, 150), "double", gpu)   # overlaps a
    c = PartialVector(RangePartition(2, 200, 300), "float", gpu)   # another type
    m = PartialMatrix(RangePartition(3, 400, 500), 4, "double", gpu)
    d = PartialVector(RangePartition(4, 100, 200), "double", gpu)
    k = torch.tensor([1], dtype=torch.int64, device=dev)
    x = torch.ones(1, dtype=torch.float64, device=dev)
    g = torch.zeros(1, dtype=torch.int64, device=dev)
    for bad in ([a, b], [a, c], [a, m], [a, a], []):  # overlap, mixed types, a matrix, twice, none
        assert _set_push(bad, k, x, g) == N.GLINT_EINVAL
    assert _set_push([d, a], k, x, g) == 0
    slab = PartialVector(RangePartition(5, 1000, 1064), "double", gpu)
    view = PartialVector.view(slab, RangePartition(6, 600, 632), 32)
    assert _set_push([slab, a], k, x, g) == N.GLINT_EINVAL  # a slab with views
    assert _set_push([view, a], k, x, g) == 0                # its view is a shard like any other
    torch.cuda.synchronize(dev)
    view.destroy()
    slab.destroy()
    for s in (a, b, c, m, d):
        s.destroy()


def test_set_push_on_two_streams_keeps_each_verdict(gpu):
    """Two pushes over the same shard set on two streams, enqueued back to back so their kernels may
    overlap: each call's verdict lives in a word of its own stream (the set's first shard keeps one per
    caller stream), so the clean batch is applied and reports 0 while the batch with a bad key reports
    it and applies nothing. (With one shared word, one call's zeroing could clear the other's verdict
    and its scatter would then apply a rejected batch.) Repeated, alternating which stream goes first."""
    dev = torch.device("cuda", gpu)
    ranges = [(0, 1 << 20), (1 << 20, 3 << 19)]
    shards = [PartialVector(RangePartition(i, a, b), "long", gpu) for i, (a, b) in enumerate(ranges)]
    rng = np.random.default_rng(17)
    k = torch.from_numpy(rng.integers(0, 3 << 19, 1 << 20).astype(np.int64)).to(dev)
    v = torch.from_numpy(rng.integers(-9, 9, k.numel()).astype(np.int64)).to(dev)
    kb = k.clone()
    kb[-1] = 3 << 19  # past the last shard
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    g1 = torch.full((1,), 3, dtype=torch.int64, device=dev)
    g2 = torch.full((1,), 3, dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)
    want = np.zeros(3 << 19, np.int64)
    for rep in range(4):
        order = [(s1, kb, g1), (s2, k, g2)] if rep % 2 else [(s2, k, g2), (s1, kb, g1)]
        for st, keys, gate in order:
            with torch.cuda.stream(st):
                assert _set_push(shards, keys, v, gate) == 0
        torch.cuda.synchronize(dev)
        assert int(g1.item()) == ~(k.numel() - 1) and int(g2.item()) == 0, rep
        np.add.at(want, k.cpu().numpy(), v.cpu().numpy())
    for sh, (a, b) in zip(shards, ranges):
        sh.sync(torch.cuda.current_stream(dev).cuda_stream)
        np.testing.assert_array_equal(sh.get(torch.arange(a, b, device=dev)).cpu().numpy(), want[a:b])
    for sh in shards:
        sh.destroy()
