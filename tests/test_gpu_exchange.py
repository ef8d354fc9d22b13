"""The exchange step on the device: glint_route_gather_dev (client bucketing + send-buffer gather in
one pass, AsyncBigVector.scala:96-116 / AsyncBigMatrix.scala:141-156) against the oracle's stable
bucketing, and the self-launching multi-rank bench (one process per rank, gloo rehearsal on one GPU).
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

from glint_amd import _native as N
from oracle import oracle as O

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


def route_gather(keys, nparts, nkeys, slot_of=None, cols=None, vals=None, dev=0):
    import torch
    d = torch.device("cuda", dev)
    lib = N.load()
    k = torch.from_numpy(keys).to(d)
    c = None if cols is None else torch.from_numpy(cols).to(d)
    v = None if vals is None else torch.from_numpy(vals).to(d)
    so = None if slot_of is None else torch.from_numpy(np.asarray(slot_of, np.int32)).to(d)
    n = keys.size
    counts = torch.full((nparts,), -7, dtype=torch.int64, device=d)
    order = torch.full((max(n, 1),), -7, dtype=torch.int64, device=d)
    ok = torch.full((max(n, 1),), -7, dtype=torch.int64, device=d)
    oc = torch.full((max(n, 1),), -7, dtype=torch.int32, device=d)
    ov = torch.full((max(n, 1),), -7, dtype=v.dtype if v is not None else torch.float64, device=d)
    bad = torch.full((1,), -7, dtype=torch.int64, device=d)
    p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    rc = lib.glint_route_gather_dev(k.data_ptr(), p(c), p(v), v.element_size() if v is not None else 0, n,
                                    N.GLINT_ROUTE_RANGE, nparts, nkeys, p(so), counts.data_ptr(), order.data_ptr(),
                                    ok.data_ptr(), p(oc) if c is not None else None,
                                    p(ov) if v is not None else None, bad.data_ptr(),
                                    torch.cuda.current_stream(d).cuda_stream)
    torch.cuda.synchronize(d)
    return rc, counts.cpu().numpy(), order.cpu().numpy()[:n], ok.cpu().numpy()[:n], oc.cpu().numpy()[:n], \
        ov.cpu().numpy()[:n], int(bad.item())


@pytest.mark.parametrize("nparts", [1, 3, 8, 64, 1000])
@pytest.mark.parametrize("n", [0, 1, 4097, 300_001])
def test_route_gather_matches_oracle(gpu, nparts, n):
    nkeys = 1_000_003
    rng = np.random.default_rng(nparts * 7 + n)
    keys = rng.integers(0, nkeys, n).astype(np.int64)
    cols = rng.integers(0, 512, n).astype(np.int32)
    vals = rng.uniform(-1, 1, n)
    c_ref, off, o_ref = O.bucket_range(keys, nparts, nkeys)
    rc, counts, order, ok, oc, ov, bad = route_gather(keys, nparts, nkeys, cols=cols, vals=vals, dev=gpu)
    assert rc == N.GLINT_OK and bad == 0
    np.testing.assert_array_equal(counts, c_ref)
    np.testing.assert_array_equal(order, o_ref)         # stable: the oracle's exact permutation
    np.testing.assert_array_equal(ok, keys[o_ref])       # send buffers in send order
    np.testing.assert_array_equal(oc, cols[o_ref])
    np.testing.assert_array_equal(ov, vals[o_ref])


def test_route_gather_slot_order_and_float_values(gpu):
    """Partitions ordered by hosting rank (rank r hosts r, r + W, ...: Client.scala:75-84), 4-byte values."""
    nparts, world, nkeys = 6, 4, 50_000
    perm = [p for r in range(world) for p in range(r, nparts, world)]
    slot_of = np.empty(nparts, np.int32)
    slot_of[perm] = np.arange(nparts)
    rng = np.random.default_rng(1)
    keys = rng.integers(0, nkeys, 77_777).astype(np.int64)
    vals = rng.uniform(-1, 1, keys.size).astype(np.float32)
    c_ref, off, o_ref = O.bucket_range(keys, nparts, nkeys)
    want = np.concatenate([o_ref[off[p]:off[p + 1]] for p in perm])
    rc, counts, order, ok, _, ov, bad = route_gather(keys, nparts, nkeys, slot_of=slot_of, vals=vals, dev=gpu)
    assert rc == N.GLINT_OK and bad == 0
    np.testing.assert_array_equal(counts, c_ref[perm])
    np.testing.assert_array_equal(order, want)
    np.testing.assert_array_equal(ok, keys[want])
    np.testing.assert_array_equal(ov, vals[want])


def test_route_gather_bad_key_word(gpu):
    keys = np.arange(10_000, dtype=np.int64)
    keys[7_777] = 10_000
    keys[9_000] = -5
    rc, counts, *_, bad = route_gather(keys, 4, 10_000, dev=gpu)
    assert rc == N.GLINT_OK  # no synchronisation: the status stays on the device
    assert bad != 0 and ~bad == 7_777
    assert counts.sum() == keys.size - 2  # bad records are in no group


def test_route_int_edge_partitioner(gpu):
    """largePartitionSize wraps to Int.MinValue at q = 2^31 - 1 (RangePartitioner.scala:18): the
    route kernel picks the JVM's partition (the hand-worked KATs of test_oracle_kat) and rejects the
    keys whose wrapped index falls outside the partition array."""
    from test_oracle_kat import INT_EDGE_CASES
    for P, N_, cases in INT_EDGE_CASES:
        keys = np.array([k for k, _ in cases], np.int64)
        rc, counts, order, ok, *_, bad = route_gather(keys, P, N_, dev=gpu)
        assert rc == N.GLINT_OK
        first_bad = next((i for i, (_, w) in enumerate(cases) if w < 0), None)
        assert (bad == 0) if first_bad is None else (~bad == first_bad)
        want = np.bincount([w for _, w in cases if w >= 0], minlength=P)
        np.testing.assert_array_equal(counts, want)


def _bench(args, **env):
    e = dict(os.environ, **env)
    e.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, capture_output=True, text=True,
                       timeout=300, env=e, cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 alone prints
    return json.loads(lines[0])


@pytest.mark.parametrize("args", [["--pattern", "dense"], ["--pattern", "dense", "--scaling", "strong"],
                                  ["--pattern", "exchange"]])
def test_bench_self_launches_ranks(gpu, args):
    """`python bench.py --gpus 2` with no launcher: two rank processes (here both on this GPU over
    gloo -- the rehearsal hooks), one JSON line with n_gpus 2 whose check is every rank's (the ranks
    agree on it with an all-reduce before rank 0 prints): what an 8-GPU SCALE run executes, at N = 2."""
    d = _bench(["--gpus", "2", "--steps", "3", "--warmup", "1", "--log2-keys", "22", "--no-cpu-baseline"] + args,
               GLINT_BENCH_DEVICE=str(gpu), GLINT_BENCH_BACKEND="gloo")
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["check"] is True
    assert d["scaling"] == ("strong" if "strong" in args else "weak")
    # the line names the GPU every rank ran on: here both on this one, flagged as a rehearsal
    dv = d["devices"]
    assert d["world_size"] == 2 and [r["rank"] for r in dv["ranks"]] == [0, 1]
    assert all(r["device"] == gpu for r in dv["ranks"]) and dv["distinct_gpus"] == 1
    assert dv["rehearsal"] is True and dv["backend"] == "gloo"


@pytest.mark.parametrize("args", [["--pattern", "zipf", "--log2-keys", "22"], ["--pattern", "matrix"],
                                  ["--pattern", "exchange", "--log2-keys", "22"],
                                  ["--pattern", "dense", "--log2-keys", "22"]])
def test_bench_rotated_batches(gpu, args):
    """--batches K: K different batches of one distribution rotated per step; the post-run check
    replays all of them (a batch pushed t times counts t times)."""
    d = _bench(args + ["--steps", "5", "--warmup", "2", "--batches", "3", "--no-cpu-baseline"])
    assert d["check"] is True and d["value"] > 0 and d["batches"]["k"] == 3


@pytest.mark.parametrize("args", [["--pattern", "pull"], ["--pattern", "rowpull"],
                                  ["--scaling", "strong", "--log2-keys", "24"]])
def test_bench_patterns(gpu, args):
    d = _bench(args + ["--steps", "3", "--warmup", "1", "--no-cpu-baseline"])
    assert d["check"] is True and d["value"] > 0 and d["roofline"]["achieved"] > 0


def test_bench_default_line_is_the_north_star(gpu):
    """With no --log2-keys the driver's line is BASELINE.json north_star's configuration (a 2^30-key
    Double vector, dense push at 1 GPU), with cfg2 (2^28) as the extra key; both are checked."""
    d = _bench(["--steps", "2", "--warmup", "1", "--no-cpu-baseline"])
    assert "2^30" in d["config"]["workload"] and d["config"]["keys_per_gpu"] == 1 << 30 and d["check"] is True
    assert d["cfg2_2p28"]["check"] is True and "2^28" in d["cfg2_2p28"]["workload"]


@pytest.mark.parametrize("n", [1, 7, 100_001, 1 << 20])
def test_route_one_partition_validates_only(gpu, n):
    """One partition and no outputs: the batch is its own send buffer; the pass checks the keys
    (the first bad record as ~index) and reports the count."""
    import torch
    d = torch.device("cuda", gpu)
    lib = N.load()
    nkeys = 1 << 22
    rng = np.random.default_rng(n)
    keys = rng.integers(0, nkeys, n).astype(np.int64)
    for bad_at in ([], [n - 1], [n // 3, n // 2] if n > 2 else []):
        k = keys.copy()
        for j, b in enumerate(bad_at):
            k[b] = nkeys + j if j == 0 else -3
        kt = torch.from_numpy(k).to(d)
        counts = torch.full((1,), -7, dtype=torch.int64, device=d)
        bad = torch.full((1,), -7, dtype=torch.int64, device=d)
        rc = lib.glint_route_gather_dev(kt.data_ptr(), None, None, 0, n, N.GLINT_ROUTE_RANGE, 1, nkeys, None,
                                        counts.data_ptr(), None, None, None, None, bad.data_ptr(),
                                        torch.cuda.current_stream(d).cuda_stream)
        torch.cuda.synchronize(d)
        assert rc == N.GLINT_OK
        if bad_at:
            assert int(bad.item()) != 0 and ~int(bad.item()) == min(bad_at)
        else:
            assert int(bad.item()) == 0 and int(counts.item()) == n


def test_routes_on_two_streams_at_once(gpu):
    """Two routes on two streams of one device run concurrently: each keeps its own scratch
    (histogram, offsets), so both equal the oracle's bucketing."""
    import torch
    d = torch.device("cuda", gpu)
    lib = N.load()
    nkeys, n = 1 << 30, 1 << 23
    cases = []
    for j, nparts in enumerate((8, 1000)):
        rng = np.random.default_rng(500 + j)
        keys = rng.integers(0, nkeys, n).astype(np.int64)
        cases.append((nparts, keys, torch.from_numpy(keys).to(d)))
    torch.cuda.synchronize(d)
    streams = [torch.cuda.Stream(d), torch.cuda.Stream(d)]
    outs = []
    for (nparts, _, kt), st in zip(cases, streams):
        with torch.cuda.stream(st):
            counts = torch.full((nparts,), -7, dtype=torch.int64, device=d)
            order = torch.full((n,), -7, dtype=torch.int64, device=d)
            bad = torch.full((1,), -7, dtype=torch.int64, device=d)
            rc = lib.glint_route_gather_dev(kt.data_ptr(), None, None, 0, n, N.GLINT_ROUTE_RANGE, nparts, nkeys,
                                            None, counts.data_ptr(), order.data_ptr(), None, None, None,
                                            bad.data_ptr(), st.cuda_stream)
            assert rc == N.GLINT_OK
            outs.append((counts, order, bad))
    torch.cuda.synchronize(d)
    for (nparts, keys, _), (counts, order, bad) in zip(cases, outs):
        c_ref, _, o_ref = O.bucket_range(keys, nparts, nkeys)
        assert int(bad.item()) == 0
        np.testing.assert_array_equal(counts.cpu().numpy(), c_ref)
        np.testing.assert_array_equal(order.cpu().numpy(), o_ref)


@pytest.mark.parametrize("row_elems,dtype", [(1, "float64"), (1, "float32"), (1, "int64"), (512, "float64"),
                                             (3, "float32"), (300, "float64"), (7, "int32")])
@pytest.mark.parametrize("n", [0, 1, 4097, 100_003])
def test_scatter_rows_matches_index_copy(gpu, row_elems, dtype, n):
    """glint_scatter_rows_dev: the pull answer's way back to the caller's order
    (AsyncBigVector.scala:61-79), out[order[i]] = src[i] for elements and whole rows, against
    torch's index_copy_; a sub-range of order (a partition's range) lands only its rows."""
    import torch
    from glint_amd.dist import scatter_rows
    d = torch.device("cuda", gpu)
    g = torch.Generator(device=d)
    g.manual_seed(n * 31 + row_elems)
    dt = getattr(torch, dtype)
    shape = (n,) if row_elems == 1 else (n, row_elems)
    src = torch.randint(-1000, 1000, shape, generator=g, device=d).to(dt)
    order = torch.randperm(n, generator=g, device=d)
    out = torch.full(shape, -7, dtype=dt, device=d)
    scatter_rows(src, order, out)
    want = torch.full(shape, -7, dtype=dt, device=d)
    want.index_copy_(0, order, src)
    assert torch.equal(out, want)
    if n > 10:  # a partition's sub-range of order
        a, c = n // 3, n // 4
        out2 = torch.full(shape, -7, dtype=dt, device=d)
        scatter_rows(src[a:a + c], order[a:a + c], out2)
        want2 = torch.full(shape, -7, dtype=dt, device=d)
        want2.index_copy_(0, order[a:a + c], src[a:a + c])
        assert torch.equal(out2, want2)


@pytest.mark.parametrize("row_elems,dtype", [(1, "float64"), (1, "int32"), (512, "float64"), (3, "float32")])
def test_copy_segments_gathers_and_puts_ranges(gpu, row_elems, dtype):
    """glint_copy_segments_dev: a local partition's records from several source ranks gathered into
    one buffer in one launch (the exchange's take), and its answers put back (put); more segments than
    one launch carries (64) are split over launches."""
    import torch
    from glint_amd.dist import copy_ranges
    d = torch.device("cuda", gpu)
    g = torch.Generator()
    g.manual_seed(row_elems)
    dt = getattr(torch, dtype)
    for nseg in (1, 3, 8, 150):
        lens = torch.randint(0, 900, (nseg,), generator=g).tolist()
        total = sum(lens) + 5000
        shape = (total,) if row_elems == 1 else (total, row_elems)
        src = torch.randint(-1000, 1000, shape, generator=g).to(dt).to(d)
        starts = sorted(torch.randint(0, total - 900, (nseg,), generator=g).tolist())
        ranges, o = [], 0
        for a, c in zip(starts, lens):
            ranges.append((a, o, c))
            o += c
        out = torch.full((o,) + tuple(shape[1:]), -7, dtype=dt, device=d)
        copy_ranges(src, out, ranges)
        want = torch.cat([src[a:a + c] for a, _, c in ranges]) if o else out
        assert torch.equal(out, want)
        back = torch.full(shape, -7, dtype=dt, device=d)
        copy_ranges(out, back, [(b, a, c) for a, b, c in ranges])
        for a, _, c in ranges:
            assert torch.equal(back[a:a + c], src[a:a + c])


def test_send_matrix_from_route_counts(gpu):
    """glint_send_matrix_dev: the split exchange's (rank, local partition) count matrix from the route's
    per-partition counts, and all zero when the route's status word reports a bad key."""
    import torch
    from glint_amd.dist import Router
    from glint_amd.partitioning import RangePartitioner
    d = torch.device("cuda", gpu)
    lib = N.load()
    router = Router(RangePartitioner.apply(7, 70_000), 3)  # 7 partitions over 3 ranks: maxp 3
    _, cell = router._device_tables(d)
    counts = torch.arange(11, 18, dtype=torch.int64, device=d)
    for badv, want_zero in ((0, False), (~5 & 0xFFFFFFFFFFFFFFFF, True)):
        bad = torch.tensor([badv - (1 << 64) if badv >= (1 << 63) else badv], dtype=torch.int64, device=d)
        send = torch.full((3 * router.maxp,), -1, dtype=torch.int64, device=d)
        assert lib.glint_send_matrix_dev(counts.data_ptr(), cell.data_ptr(), 7, 3 * router.maxp, bad.data_ptr(),
                                         send.data_ptr(), torch.cuda.current_stream(d).cuda_stream) == N.GLINT_OK
        want = torch.zeros(3 * router.maxp, dtype=torch.int64, device=d)
        if not want_zero:
            want[cell] = counts
        assert torch.equal(send, want)
