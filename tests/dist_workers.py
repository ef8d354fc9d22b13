"""Worker bodies for the multi-process tests (test_dist_cpu.py, test_gpu_parity.py::test_dist_*).

Each rank pushes / pulls its own seeded batch through glint_amd.dist; every rank regenerates all
ranks' batches and checks its answers against one sequential oracle replay of the whole job:
shards apply records in source-rank order, each source's records in its caller's order, so the
replay -- rank 0's batch, then rank 1's, ... -- is bit-exact also for Double sums.
"""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from glint_amd.errors import ArrayIndexOutOfBoundsException, IndexOutOfBoundsException  # noqa: E402
from glint_amd.partitioning import CyclicPartitioner, RangePartition, RangePartitioner  # noqa: E402
from glint_amd.shard import resolve_dtype  # noqa: E402
from oracle import oracle as O  # noqa: E402


class OracleShard:
    """Test double with the PartialVector / PartialMatrix call surface over the CPU oracle, so the
    routing and exchange layers can be exercised on CPU-only ranks (gloo)."""

    def __init__(self, kind, partition, cols, dtype, device):
        self.code, self.np_dtype = resolve_dtype(dtype)
        if isinstance(partition, RangePartition):
            part = O.part_range(partition.start, partition.end)
        else:
            part = O.part_cyclic(partition.index, partition.numberOfPartitions, partition.numberOfKeys)
        self.o = O.OracleVector(part, self.code) if kind == "vector" else O.OracleMatrix(part, cols, self.code)

    def update(self, *args, deterministic=False):
        bad = self.o.update(*[a.cpu().numpy() for a in args])
        if bad != -1:  # as the HBM shard reports it (glint_amd/shard.py)
            raise ArrayIndexOutOfBoundsException(f"record {bad} is outside the partition", bad)

    def get(self, *args):
        out, bad = self.o.get(*[a.cpu().numpy() for a in args])
        assert bad == -1
        return torch.from_numpy(out)

    def getRows(self, rows):
        out, bad = self.o.get_rows(rows.cpu().numpy())
        assert bad == -1
        return torch.from_numpy(out)

    def destroy(self):
        pass


def _oracle_factory(kind, partition, cols, dtype, device):
    return OracleShard(kind, partition, cols, dtype, device)


def _batch(seed, n, nkeys, np_dtype):
    rng = np.random.default_rng(seed)
    k = rng.integers(0, nkeys, n).astype(np.int64)
    k[: n // 4] = k[n // 2: n // 2 + n // 4]  # duplicates inside the batch
    if np.dtype(np_dtype).kind == "f":
        v = rng.uniform(-1, 1, n).astype(np_dtype)
    else:
        v = rng.integers(-1000, 1000, n).astype(np_dtype)
    return k, v


def _init(rank, world, port, backend):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group(backend, rank=rank, world_size=world)


def run_case(rank, world, port, backend, case, use_gpu):
    _init(rank, world, port, backend)
    try:
        if use_gpu:
            torch.cuda.set_device(0)
            dev = torch.device("cuda", 0)
            from glint_amd.dist import DistributedClient
            client = DistributedClient(device=dev)
        else:
            dev = torch.device("cpu")
            from glint_amd.dist import DistributedClient
            client = DistributedClient(device=dev, shard_factory=_oracle_factory)
        (CASES.get(case) or GPU_CASES[case])(client, rank, world, dev)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _vector_case(nkeys, mps, partitioner, dtype, n=3000):
    def body(client, rank, world, dev):
        _, np_dtype = resolve_dtype(dtype)
        vec = client.vector(nkeys, dtype, modelsPerServer=mps, createPartitioner=partitioner)
        for step in range(2):
            k, v = _batch(1000 * step + rank, n + 37 * rank, nkeys, np_dtype)
            vec.push(torch.from_numpy(k).to(dev), torch.from_numpy(v).to(dev), deterministic=True)
        # oracle replay: all ranks' batches in rank order, step by step
        ref = O.OracleVector(O.part_range(0, nkeys), resolve_dtype(dtype)[0])
        for step in range(2):
            for r in range(world):
                k, v = _batch(1000 * step + r, n + 37 * r, nkeys, np_dtype)
                assert ref.update(k, v) == -1
        q = np.random.default_rng(77 + rank).integers(0, nkeys, 1500 + rank).astype(np.int64)
        got = vec.pull(torch.from_numpy(q).to(dev)).cpu().numpy()
        want, _ = ref.get(q)
        np.testing.assert_array_equal(got, want)
        # out-of-range key: raised on every rank before any exchange, the model is untouched
        bad = np.array([0, nkeys], dtype=np.int64)
        try:
            vec.push(torch.from_numpy(bad).to(dev), torch.from_numpy(np.zeros(2, np_dtype)).to(dev))
            raise AssertionError("out-of-range key accepted")
        except IndexOutOfBoundsException:
            pass
        got2 = vec.pull(torch.from_numpy(q).to(dev)).cpu().numpy()
        np.testing.assert_array_equal(got2, want)
        # keys 2^32 away from an in-range key: (key - start).toInt would alias them onto elements, but
        # RangePartitioner.partition rejects them (RangePartitioner.scala:30), on every path
        for wrap in ([nkeys + 2**32], [-(2**32) + 1], [1, nkeys - 1 + 2**32]):
            kw = np.array(wrap, dtype=np.int64)
            try:
                vec.push(torch.from_numpy(kw).to(dev), torch.from_numpy(np.ones(kw.size, np_dtype)).to(dev))
                raise AssertionError(f"wrapped key {wrap} accepted")
            except IndexOutOfBoundsException:
                pass
        np.testing.assert_array_equal(vec.pull(torch.from_numpy(q).to(dev)).cpu().numpy(), want)
        # only rank 0's batch is bad: it raises after the collectives, the other ranks' pushes land
        k1 = np.array([3], np.int64) if rank else np.array([1, nkeys + 5], np.int64)
        try:
            vec.push(torch.from_numpy(k1).to(dev), torch.from_numpy(np.ones(k1.size, np_dtype)).to(dev))
            assert rank != 0, "out-of-range key accepted"
        except IndexOutOfBoundsException:
            assert rank == 0
        for _ in range(world - 1):
            assert ref.update(np.array([3], np.int64), np.ones(1, np_dtype)) == -1
        want, _ = ref.get(q)
        np.testing.assert_array_equal(vec.pull(torch.from_numpy(q).to(dev)).cpu().numpy(), want)
        # a bad pull on rank 0 only: the others are answered
        qb = q.copy()
        if rank == 0:
            qb[3] = -1
        try:
            got3 = vec.pull(torch.from_numpy(qb).to(dev)).cpu().numpy()
            assert rank != 0, "out-of-range pull accepted"
            np.testing.assert_array_equal(got3, want)
        except IndexOutOfBoundsException:
            assert rank == 0
        # an empty batch still takes part in the exchange
        vec.push(torch.zeros(0, dtype=torch.int64, device=dev), torch.zeros(0, dtype=torch.float64, device=dev))
        assert vec.pull(torch.zeros(0, dtype=torch.int64, device=dev)).numel() == 0
        vec.destroy()
    return body


def _matrix_case(nrows, ncols, mps, dtype="double", n=2500):
    def body(client, rank, world, dev):
        _, np_dtype = resolve_dtype(dtype)
        mat = client.matrix(nrows, ncols, dtype, modelsPerServer=mps)
        ref = O.OracleMatrix(O.part_range(0, nrows), ncols, resolve_dtype(dtype)[0])
        for r in range(world):
            rng = np.random.default_rng(500 + r)
            rows = rng.integers(0, nrows, n).astype(np.int64)
            cols = rng.integers(0, ncols, n).astype(np.int32)
            vals = rng.uniform(-1, 1, n).astype(np_dtype)
            if r == rank:
                mat.push(torch.from_numpy(rows).to(dev), torch.from_numpy(cols).to(dev),
                         torch.from_numpy(vals).to(dev), deterministic=True)
            assert ref.update(rows, cols, vals) == -1
        rng = np.random.default_rng(900 + rank)
        qr = rng.integers(0, nrows, 700).astype(np.int64)
        qc = rng.integers(0, ncols, 700).astype(np.int32)
        got = mat.pull(torch.from_numpy(qr).to(dev), torch.from_numpy(qc).to(dev)).cpu().numpy()
        np.testing.assert_array_equal(got, ref.get(qr, qc)[0])
        rows_got = mat.pull(torch.from_numpy(qr[:50]).to(dev)).cpu().numpy()
        np.testing.assert_array_equal(rows_got, ref.get_rows(qr[:50])[0])
        # rows 2^32 away from an in-range row are rejected as keys; at world 1 (one rank hosts every
        # shard) a bad column is the shard's ArrayIndexOutOfBoundsException on every path
        one = torch.ones(2, dtype=mat.dtype, device=dev)
        for wrap in ([nrows + 2**32, 0], [-(2**32) + 1, 0]):
            try:
                mat.push(torch.tensor(wrap, dtype=torch.int64, device=dev),
                         torch.zeros(2, dtype=torch.int32, device=dev), one)
                raise AssertionError(f"wrapped row {wrap} accepted")
            except IndexOutOfBoundsException:
                pass
        if world == 1:
            for badc in (ncols, -1):
                try:
                    mat.push(torch.tensor([1], dtype=torch.int64, device=dev),
                             torch.tensor([badc], dtype=torch.int32, device=dev), one[:1])
                    raise AssertionError("bad column accepted")
                except ArrayIndexOutOfBoundsException as e:
                    assert e.record == 0, e.record
        np.testing.assert_array_equal(mat.pull(torch.from_numpy(qr).to(dev), torch.from_numpy(qc).to(dev)).cpu().numpy(),
                                      ref.get(qr, qc)[0])
        mat.destroy()
    return body


def _slab_case(nkeys, mps, dtype, keyed, n=60_000):
    """The rank's partitions in one slab (dist.slab_shards). World 1, partitions side by side and
    aligned (keyed): an unordered device push is ONE validating push on the slab (_push_gated);
    otherwise (unaligned partitions, or world > 1 where rank r hosts r, r + W, ...) the route
    rebases keys into every rank's slab and each rank pushes what it receives as one call
    (_push_slab). Interleaved with deterministic pushes (the views, through the route) and, at
    world 1, with the views' own host-pointer pushes left in flight -- against the oracle's replay
    (every rank pushes the same batches). Long: bit-exact; Double: within 1e-12 of each element's
    sum of magnitudes (unordered sums)."""
    def body(client, rank, world, dev):
        _, np_dtype = resolve_dtype(dtype)
        vec = client.vector(nkeys, dtype, modelsPerServer=mps)
        assert vec.slab is not None and all(sh.slab is vec.slab for sh in vec.shards)
        assert vec._delta is not None and vec._slab_keyed == (keyed and world == 1), (vec._slab_keyed, keyed)
        ref = O.OracleVector(O.part_range(0, nkeys), resolve_dtype(dtype)[0])
        mag = np.zeros(nkeys, np.float64)
        tickets = []
        for step, how in enumerate(["device", "host", "device", "deterministic", "device"]):
            k, v = _batch(3000 + step, n, nkeys, np_dtype)
            if how == "host" and world == 1:
                # each view's records through its host-pointer path, enqueued and NOT waited for: the
                # slab's next push must order itself after them (dev_order_after_host over its views)
                for sh in vec.shards:
                    m = (k >= sh.partition.start) & (k < sh.partition.end)
                    tickets.append((sh, sh.push_async(k[m], v[m])))
            else:
                vec.push(torch.from_numpy(k).to(dev), torch.from_numpy(v).to(dev), deterministic=how == "deterministic")
            for _ in range(1 if how == "host" and world == 1 else world):
                assert ref.update(k, v) == -1
                np.add.at(mag, k, np.abs(v.astype(np.float64)))
            if step == 2:
                for sh, t in tickets:
                    sh.wait(t)
        allk = np.arange(nkeys, dtype=np.int64)
        want, _ = ref.get(allk)
        got = vec.pull(torch.from_numpy(allk).to(dev)).cpu().numpy()
        if np.dtype(np_dtype).kind == "f":
            assert np.all(np.abs(got - want) <= 1e-12 * mag), np.max(np.abs(got - want) - 1e-12 * mag)
        else:
            np.testing.assert_array_equal(got, want)
        # each local view holds its partition's elements (the slab's rows at its place)
        for sh in vec.shards:
            p = sh.partition
            np.testing.assert_array_equal(sh.get(torch.arange(p.start, p.end, device=dev)).cpu().numpy(),
                                          got[p.start:p.end])
        # a bad key on rank 0: it sends nothing and raises (after the collectives); the others land
        bad = np.array([5, nkeys, 7], dtype=np.int64) if rank == 0 else np.array([5, 7], dtype=np.int64)
        try:
            vec.push(torch.from_numpy(bad).to(dev), torch.from_numpy(np.ones(bad.size, np_dtype)).to(dev))
            assert rank != 0, "out-of-range key accepted"
        except IndexOutOfBoundsException:
            assert rank == 0
        for _ in range(world - 1):
            assert ref.update(np.array([5, 7], np.int64), np.ones(2, np_dtype)) == -1
        want, _ = ref.get(allk)
        got = vec.pull(torch.from_numpy(allk).to(dev)).cpu().numpy()
        if np.dtype(np_dtype).kind != "f":
            np.testing.assert_array_equal(got, want)
        # pulls of keys 2^32 away from real ones (a keyed slab's gather would alias them): the route's
        # check rejects them on every path
        for wrap in ([2**32 + 5], [3, -(2**32) + 1], [nkeys]):
            try:
                vec.pull(torch.tensor(wrap, dtype=torch.int64, device=dev))
                raise AssertionError(f"pull of {wrap} accepted")
            except IndexOutOfBoundsException as e:
                assert f"(record {len(wrap) - 1})" in str(e), str(e)
        q = torch.from_numpy(np.random.default_rng(5).integers(0, nkeys, 999)).to(dev)
        np.testing.assert_array_equal(vec.pull(q).cpu().numpy(), got[q.cpu().numpy()])
        vec.destroy()
    return body


def _set_case(nkeys, mps, dtype, n=20_000):
    """Sparse unordered device pushes (fewer records than a rank's keys / 8): one push for all local
    shards (glint_vec_push_dev_shards, DistributedBigVector._set_push) -- at world 1 in place of the
    route (_push_set), at world > 1 (slabs off) for everything a rank receives -- against the oracle's
    replay (every rank pushes the same batches); a bad key applies nothing and raises the route's
    exception."""
    def body(client, rank, world, dev):
        _, np_dtype = resolve_dtype(dtype)
        if world > 1:
            client.slabs = False  # (the slab's rebased route would take these pushes)
        try:
            vec = client.vector(nkeys, dtype, modelsPerServer=mps)
        finally:
            client.slabs = True
        assert not vec._slab_keyed and n * 8 * world < nkeys
        calls = []
        orig = vec._set_push
        vec._set_push = lambda k, v: calls.append(1) or orig(k, v)
        ref = O.OracleVector(O.part_range(0, nkeys), resolve_dtype(dtype)[0])
        for step in range(3):
            k, v = _batch(7000 + step, n, nkeys, np_dtype)
            vec.push(torch.from_numpy(k).to(dev), torch.from_numpy(v).to(dev))
            for _ in range(world):
                assert ref.update(k, v) == -1
        allk = np.arange(nkeys, dtype=np.int64)
        want, _ = ref.get(allk)
        got = vec.pull(torch.from_numpy(allk).to(dev)).cpu().numpy()
        np.testing.assert_array_equal(got, want)
        for bad in ([3, nkeys, 9], [-1, 4], [nkeys + 2**32]):
            b = np.array(bad, dtype=np.int64)
            try:
                vec.push(torch.from_numpy(b).to(dev), torch.from_numpy(np.ones(b.size, np_dtype)).to(dev))
                raise AssertionError(f"bad key {bad} accepted")
            except IndexOutOfBoundsException as e:
                assert f"record {[i for i, x in enumerate(bad) if not 0 <= x < nkeys][0]})" in str(e), str(e)
        np.testing.assert_array_equal(vec.pull(torch.from_numpy(allk).to(dev)).cpu().numpy(), want)
        # world 1: three good and three bad batches through the set push; world > 1: the bad batches
        # send nothing (every rank's is bad), so only the good ones arrive
        assert len(calls) == (6 if world == 1 else 3), len(calls)
        vec.destroy()
    return body


# HBM shards only (test_gpu_parity.test_dist_exchange_on_gpu): world 1 with the partitions in one slab
GPU_CASES = {
    "vec_slab_long_mps8": _slab_case(8 * 4096, 8, "long", keyed=True),
    "vec_slab_double_mps4": _slab_case(4 * 8192, 4, "double", keyed=True),
    "vec_slab_long_mps3_unaligned": _slab_case(3 * 1000 + 1, 3, "long", keyed=False),  # (rebased route)
    "vec_range_mps4_aligned": _vector_case(4 * 4096, 4, RangePartitioner.apply, "double"),
    "mat_range_mps4_aligned": _matrix_case(1_024, 17, 4),
    "vec_set_long_mps8": _set_case(8 * 50_000 + 5, 8, "long"),
}

CASES = {
    "vec_range": _vector_case(10_007, 1, RangePartitioner.apply, "double"),
    "vec_range_mps3": _vector_case(10_007, 3, RangePartitioner.apply, "double"),
    "vec_cyclic_mps2": _vector_case(9_001, 2, CyclicPartitioner.apply, "double"),
    "vec_long_few_keys": _vector_case(5, 2, RangePartitioner.apply, "long", n=200),
    "mat_range": _matrix_case(1_003, 17, 1),
    "mat_range_mps2": _matrix_case(1_003, 17, 2),
}


def _check_close(got, ref, mag, what):
    """Default-mode Double sums of repeated keys are summed in no particular order. The bound is 1e-9
    of each element's sum of magnitudes (sum |v|) -- the scale every ordering of a floating-point sum
    is accurate to (n terms: ~n eps sum |v|) and far inside the north star's 1e-6 relative, while a
    lost or duplicated record cannot pass; it demands exact zeros where nothing was pushed."""
    err = (got - ref).abs()
    bad = err > 1e-9 * mag
    assert not bool(bad.any()), f"{what}: {int(bad.sum())} elements off by more than 1e-9 of sum |v|"


def run_cfg4(rank, world, port, backend, nbatch, log2_batch, dtype="long"):
    """BASELINE.json configs[3] at its own key space on one GPU: RangePartitioner(8, 2^31) -- eight
    2^28-key shards (modelsPerServer = 8 on one server) behind DistributedClient -- fed `nbatch`
    client batches of 2^log2_batch uniform keys (the 64 loopback clients of cfg4), each routed to the
    8 shards by glint_route_gather_dev (AsyncBigVector.scala:96-121). Long sums are exact in any
    order, so every shard must equal a torch.index_add_ int64 reference bit for bit; Double shards
    must be within 1e-6 of fp64 segment sums (relative to the sum of magnitudes, _check_close). Two
    sampled key ranges are replayed through the oracle's sequential update loop as well."""
    _init(rank, world, port, backend)
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        from glint_amd.dist import DistributedClient
        nkeys = 1 << 31
        fp = dtype == "double"
        tdt = torch.float64 if fp else torch.int64
        client = DistributedClient(device=dev)
        vec = client.vector(nkeys, dtype, modelsPerServer=8)
        parts = vec.partitioner.all()
        assert vec.nrOfPartitions == 8 and all(p.size == 1 << 28 for p in parts)
        ref = torch.zeros(nkeys, dtype=tdt, device=dev)
        mag = torch.zeros(nkeys, dtype=tdt, device=dev) if fp else None
        # oracle replay windows: 2^20 keys inside partitions 2 and 7 (the last key of the space included)
        windows = [(parts[2].start + 12_345, parts[2].start + 12_345 + (1 << 20)), (nkeys - (1 << 20), nkeys)]
        orc = [O.OracleVector(O.part_range(a, b), O.O_F64 if fp else O.O_I64) for a, b in windows]
        n = 1 << log2_batch
        for c in range(nbatch):
            g = torch.Generator(device=dev)
            g.manual_seed(4000 + c)
            k = torch.randint(0, nkeys, (n,), dtype=torch.int64, device=dev, generator=g)
            if fp:
                v = torch.rand(n, dtype=torch.float64, device=dev, generator=g) * 2 - 1
            else:
                v = torch.randint(-(1 << 40), 1 << 40, (n,), dtype=torch.int64, device=dev, generator=g)
            assert vec.push(k, v)
            ref.index_add_(0, k, v)
            if fp:
                mag.index_add_(0, k, v.abs())
            for (a, b), o in zip(windows, orc):
                m = (k >= a) & (k < b)
                assert o.update(k[m].cpu().numpy(), v[m].cpu().numpy()) == -1
        torch.cuda.synchronize(dev)
        for p, sh in zip(parts, vec.shards):
            got = sh.get(torch.arange(p.start, p.end, dtype=torch.int64, device=dev))
            if fp:
                _check_close(got, ref[p.start:p.end], mag[p.start:p.end], f"partition {p.index}")
            else:
                assert torch.equal(got, ref[p.start:p.end]), f"partition {p.index} differs from index_add_"
            del got
        for (a, b), o in zip(windows, orc):
            got = vec.pull(torch.arange(a, b, dtype=torch.int64, device=dev))
            if fp:
                _check_close(got.cpu(), torch.from_numpy(o.data), mag[a:b].cpu(), "oracle window")
            else:
                np.testing.assert_array_equal(got.cpu().numpy(), o.data)
        # pulls of random keys over all 8 shards come back in the caller's order, bit-equal to the shards
        q = torch.randint(0, nkeys, (1 << 20,), dtype=torch.int64, device=dev)
        got = vec.pull(q)
        own = torch.empty_like(got)
        for p, sh in zip(parts, vec.shards):
            m = (q >= p.start) & (q < p.end)
            own[m] = sh.get(q[m].contiguous())
        assert torch.equal(got, own)
        if not fp:
            assert torch.equal(got, ref[q])
        vec.destroy()
        dist.barrier()
    finally:
        dist.destroy_process_group()


def zipf_rows(g, n, rows, dev):
    """Zipf(1.0)-distributed row indices (P(rank r) ~ 1/r: floor(rows^u) for uniform u is log-uniform)
    scattered over [0, rows) by an odd-multiplier bijection (rows a power of two)."""
    u = torch.rand(n, dtype=torch.float64, device=dev, generator=g)
    ranks = torch.clamp(torch.floor(torch.pow(float(rows), u)).to(torch.int64) - 1, 0, rows - 1)
    return (ranks * 0x9E3779B1) & (rows - 1)


def run_cfg5(rank, world, port, backend, dtype, log2_rows=20, ncols=512, nbatch=8, log2_batch=23, log2_pull=16):
    """BASELINE.json configs[4] at its own shape on one GPU: a 2^20 x 512 matrix (4 GiB of Double) over
    RangePartitioner(8, 2^20) -- modelsPerServer = 8 on one server, eight 2^17-row shards -- behind
    DistributedClient / DistributedBigMatrix. 2^26 triplets (Zipf(1.0) rows x uniform cols) arrive as
    8 client batches of 2^23, each routed to the 8 shards (AsyncBigMatrix.scala:141-156); then 2^16
    Zipf rows are pulled back whole (AsyncBigMatrix.scala:53-86). Long: every shard and every pulled
    row equal a torch.index_add_ int64 reference bit for bit; Double: within 1e-6 of fp64 segment sums
    (_check_close), and the pulled rows bit-equal to the shards. Two row windows are replayed through
    the oracle's PartialMatrix.update loop."""
    _init(rank, world, port, backend)
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        from glint_amd.dist import DistributedClient
        nrows = 1 << log2_rows
        fp = dtype == "double"
        tdt = torch.float64 if fp else torch.int64
        client = DistributedClient(device=dev)
        mat = client.matrix(nrows, ncols, dtype, modelsPerServer=8)
        parts = mat.partitioner.all()
        assert mat.nrOfPartitions == 8 and all(p.size == nrows // 8 for p in parts)
        ref = torch.zeros(nrows * ncols, dtype=tdt, device=dev)
        mag = torch.zeros(nrows * ncols, dtype=tdt, device=dev) if fp else None
        wins = [(parts[2].start + 777, parts[2].start + 777 + 64), (nrows - 64, nrows)]
        orc = [O.OracleMatrix(O.part_range(a, b), ncols, O.O_F64 if fp else O.O_I64) for a, b in wins]
        n = 1 << log2_batch
        for c in range(nbatch):
            g = torch.Generator(device=dev)
            g.manual_seed(5000 + c)
            r = zipf_rows(g, n, nrows, dev)
            cl = torch.randint(0, ncols, (n,), dtype=torch.int32, device=dev, generator=g)
            if fp:
                v = torch.rand(n, dtype=torch.float64, device=dev, generator=g) * 2 - 1
            else:
                v = torch.randint(-(1 << 40), 1 << 40, (n,), dtype=torch.int64, device=dev, generator=g)
            assert mat.push(r, cl, v)
            flat = r * ncols + cl.to(torch.int64)
            ref.index_add_(0, flat, v)
            if fp:
                mag.index_add_(0, flat, v.abs())
            for (a, b), o in zip(wins, orc):
                m = (r >= a) & (r < b)
                assert o.update(r[m].cpu().numpy(), cl[m].cpu().numpy(), v[m].cpu().numpy()) == -1
        torch.cuda.synchronize(dev)
        ref = ref.view(nrows, ncols)
        mag = mag.view(nrows, ncols) if fp else None
        full = torch.empty((nrows, ncols), dtype=tdt, device=dev)
        for p, sh in zip(parts, mat.shards):
            sh.getRows(torch.arange(p.start, p.end, dtype=torch.int64, device=dev), out=full[p.start:p.end])
            if fp:
                _check_close(full[p.start:p.end], ref[p.start:p.end], mag[p.start:p.end], f"partition {p.index}")
            else:
                assert torch.equal(full[p.start:p.end], ref[p.start:p.end]), f"partition {p.index} differs"
        for (a, b), o in zip(wins, orc):
            want = torch.from_numpy(o.data.reshape(b - a, ncols))
            if fp:
                _check_close(full[a:b].cpu(), want, mag[a:b].cpu(), "oracle window")
            else:
                assert torch.equal(full[a:b].cpu(), want)
        # the row pull: 2^16 Zipf rows through DistributedBigMatrix.pull(rows)
        g = torch.Generator(device=dev)
        g.manual_seed(6000)
        q = zipf_rows(g, 1 << log2_pull, nrows, dev)
        got = mat.pull(q)
        assert got.shape == (q.numel(), ncols)
        assert torch.equal(got, full[q])
        if not fp:
            assert torch.equal(got, ref[q])
        # element pulls of the same rows at random cols, through DistributedBigMatrix.pull(rows, cols)
        qc = torch.randint(0, ncols, (q.numel(),), dtype=torch.int32, device=dev, generator=g)
        assert torch.equal(mat.pull(q, qc), full[q, qc.to(torch.int64)])
        mat.destroy()
        dist.barrier()
    finally:
        dist.destroy_process_group()
