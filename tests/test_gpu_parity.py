"""GPU parity: the HIP push/pull path against the oracle, through the C ABI.

Bar: bit-exact for Int/Long everywhere and for Float/Double whenever a push touches each element
at most once or runs with GLINT_PUSH_DETERMINISTIC; <= 1e-6 relative (north star) for Double sums of
repeated keys in the default (atomic) mode. Run on the MI355X box: pytest -m gpu.
"""
import zlib
from pathlib import Path

import numpy as np
import pytest

import glint_amd
from glint_amd import _native as N
from glint_amd import ArrayIndexOutOfBoundsException, Client, CyclicPartition, PartialMatrix, PartialVector, \
    RangePartition
from oracle import oracle as O

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden"
DT = ["double", "float", "long", "int"]


def rand_vals(rng, dtype, n):
    npd = glint_amd.shard.resolve_dtype(dtype)[1]
    if np.issubdtype(npd, np.floating):
        return rng.uniform(-1, 1, n).astype(npd)
    info = np.iinfo(npd)
    return rng.integers(info.min, info.max, n, dtype=npd, endpoint=True)


def oracle_vec(part, dtype):
    code = O.CODE[dtype]
    if isinstance(part, RangePartition):
        return O.OracleVector(O.part_range(part.start, part.end), code)
    return O.OracleVector(O.part_cyclic(part.index, part.numberOfPartitions, part.numberOfKeys), code)


# ---- the reference's known-answer scenarios, through the GPU client -----------------------------------
def test_reference_scenarios_on_gpu(kat, gpu):
    from test_oracle_kat import expected_array
    for sc in kat["scenarios"]:
        client = Client([gpu] * sc["servers"])  # `servers` parameter servers, all on this GPU
        if sc["model"] == "vector":
            m = client.vector(sc["keys"], sc["dtype"], sc["modelsPerServer"])
        else:
            m = client.matrix(sc["rows"], sc["cols"], sc["dtype"], sc["modelsPerServer"])
        assert m.nrOfPartitions == min(sc.get("keys", sc.get("rows")), sc["modelsPerServer"] * sc["servers"])
        code = O.CODE[sc["dtype"]]
        for op in sc["ops"]:
            if op["op"] == "push":
                if sc["model"] == "vector":
                    m.push(op["keys"], op["values"])
                else:
                    m.push(op["rows"], op["cols"], op["values"])
            else:
                if op["op"] == "pull_rows":
                    got = m.pull(op["rows"])
                elif sc["model"] == "vector":
                    got = m.pull(op["keys"])
                else:
                    got = m.pull(op["rows"], op["cols"])
                np.testing.assert_array_equal(got, expected_array(op, code, sc.get("cols")), err_msg=sc["spec"])
        m.destroy()


def test_granular_big_vector_on_gpu(kat, gpu):
    """GranularBigVectorSpec.scala:14-35 through the GPU shards (2 servers, messages of 1000)."""
    spec = kat["large"][0]
    n = spec["keys"]
    values = O.JavaRandom(42).nextDoubles(n)
    keys = np.arange(n, dtype=np.int64)
    m = Client([gpu, gpu]).vector(n, "double")
    for i in range(0, n, 100_000):  # message chunking does not change the result; fewer calls
        m.push(keys[i:i + 100_000], values[i:i + 100_000])
    np.testing.assert_array_equal(m.pull(keys), values)
    m.destroy()


@pytest.mark.parametrize("which", [1, 2])
def test_granular_big_matrix_on_gpu(kat, gpu, which):
    spec = kat["large"][which]
    i = np.arange(1_000_000, dtype=np.int64)
    rows, cols, vals = i % 1000, (i // 1000).astype(np.int32), i.astype(np.float64) * 3.14
    m = Client([gpu] * spec["servers"]).matrix(1000, 1000, "double")
    for s0 in range(0, rows.size, spec["maximumMessageSize"] * 10):
        s1 = s0 + spec["maximumMessageSize"] * 10
        m.push(rows[s0:s1], cols[s0:s1], vals[s0:s1])
    if spec["pull"] == "elements":
        np.testing.assert_array_equal(m.pull(rows, cols), vals)
    else:
        full = m.pull(np.arange(1000, dtype=np.int64))
        np.testing.assert_array_equal(full[rows, cols], vals)
    m.destroy()


# ---- vector push/pull vs oracle --------------------------------------------------------------------
@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("pattern", ["dense", "dense_odd", "sorted_sparse", "permutation", "duplicates",
                                     "dense_then_repeat", "single", "empty"])
def test_vector_push_pull(gpu, dtype, pattern):
    rng = np.random.default_rng(zlib.crc32(f"{dtype}/{pattern}".encode()))
    start, size = 1_000_003, 300_001
    part = RangePartition(2, start, start + size)
    if pattern == "dense":
        keys = np.arange(start, start + size, dtype=np.int64)
    elif pattern == "dense_odd":
        keys = np.arange(start + 1, start + size, dtype=np.int64)[:123_457]
    elif pattern == "sorted_sparse":
        keys = np.sort(rng.choice(size, 50_000, replace=False)).astype(np.int64) + start
    elif pattern == "permutation":
        keys = rng.permutation(size).astype(np.int64) + start
    elif pattern == "duplicates":
        keys = rng.integers(0, 1000, 200_000).astype(np.int64) + start
    elif pattern == "dense_then_repeat":  # increasing for many tiles, then the whole range again
        k = np.arange(start, start + size, dtype=np.int64)
        keys = np.concatenate([k, k[:100_000]])
    elif pattern == "single":
        keys = np.array([start + 17], np.int64)
    else:
        keys = np.zeros(0, np.int64)
    vals = rand_vals(rng, dtype, keys.size)
    ref = oracle_vec(part, dtype)
    with PartialVector(part, dtype, gpu) as sh:
        for _ in range(2):  # push twice: accumulation onto non-zero state
            assert sh.update(keys, vals)
            assert ref.update(keys, vals) == -1
        got = sh.to_numpy()
        exact = dtype in ("long", "int") or pattern not in ("duplicates", "dense_then_repeat")
        if exact:
            np.testing.assert_array_equal(got, ref.data)
        else:
            # atomic (unordered) sums of ~400 values per key: <= 1e-6 relative for Double (north star);
            # the absolute floor covers sums that cancel to ~0
            np.testing.assert_allclose(got, ref.data, rtol=1e-6 if dtype == "double" else 1e-4,
                                       atol=1e-9 if dtype == "double" else 2e-3)
        # pull == the shard's own state at those keys (bit-exact), and == the oracle where exact
        q = keys if keys.size else np.zeros(0, np.int64)
        np.testing.assert_array_equal(sh.get(q), got[q - start])
        if exact and q.size:
            np.testing.assert_array_equal(sh.get(q), ref.get(q)[0])


@pytest.mark.parametrize("dtype", ["double", "float"])
def test_deterministic_push_is_bit_exact(gpu, dtype):
    """GLINT_PUSH_DETERMINISTIC reproduces the sequential order bit for bit, duplicates included."""
    z = np.load(GOLD / "zipf_push.npz")
    start, size = int(z["start"]), int(z["size"])
    part = RangePartition(0, start, start + size)
    keys = z["keys"]
    vals = z["values_f64"].astype(glint_amd.shard.resolve_dtype(dtype)[1])
    ref = oracle_vec(part, dtype)
    assert ref.update(keys, vals) == -1
    if dtype == "double":
        np.testing.assert_array_equal(ref.data, z["expect_f64"])
    with PartialVector(part, dtype, gpu) as sh:
        sh.update(keys, vals, deterministic=True)
        np.testing.assert_array_equal(sh.to_numpy(), ref.data)
        # a sorted head followed by an unsorted tail: the tail continues from the head's sums
        k2 = np.concatenate([np.arange(start, start + size, dtype=np.int64), keys])
        v2 = np.concatenate([np.full(size, 0.1, vals.dtype), vals])
        sh.update(k2, v2, deterministic=True)
        assert ref.update(k2, v2) == -1
        np.testing.assert_array_equal(sh.to_numpy(), ref.data)


@pytest.mark.parametrize("dtype", ["double", "float"])
@pytest.mark.parametrize("layout", ["range", "cyclic"])
@pytest.mark.parametrize("head", [False, True])
def test_deterministic_hot_chain_split(gpu, dtype, layout, head):
    """The deterministic tail's hot-chain split (glint_sort.hip: det_hot_pick / det_hot_count /
    det_hot_scatter and det_fold_hot on the second stream, joined by an event) engages for tails of
    >= 2^19 records with elements of >= 2^16 estimated records. 2^21 records, three keys taking 40 %,
    20 % and 10 % of them in push order, the rest over the partition: the result must be the
    sequential loop's (PartialVector.scala:35-43) bit for bit, with and without a sorted head in front
    (the tail then continues from the head's sums)."""
    rng = np.random.default_rng(zlib.crc32(f"hotchain/{dtype}/{layout}/{head}".encode()))
    n, size = 1 << 21, 1 << 20
    if layout == "range":
        start = 3 << 20
        part = RangePartition(3, start, start + size)
        owned = np.arange(start, start + size, dtype=np.int64)
    else:
        P, idx = 5, 2
        part = CyclicPartition(idx, P, P * size)
        owned = np.arange(idx, P * size, P, dtype=np.int64)
    hot = owned[rng.choice(size, 3, replace=False)]
    which = rng.random(n)
    keys = owned[rng.integers(0, size, n)]
    keys[which < 0.4] = hot[0]
    keys[(which >= 0.4) & (which < 0.6)] = hot[1]
    keys[(which >= 0.6) & (which < 0.7)] = hot[2]
    vals = rand_vals(rng, dtype, n)
    if head:  # strictly increasing head (plain-RMW prefix), then the unordered tail
        keys = np.concatenate([owned, keys])
        vals = np.concatenate([rand_vals(rng, dtype, size), vals])
    ref = oracle_vec(part, dtype)
    assert ref.update(keys, vals) == -1
    import torch
    d = torch.device("cuda", gpu)
    with PartialVector(part, dtype, gpu) as sh:
        sh.update(torch.from_numpy(keys).to(d), torch.from_numpy(vals).to(d), deterministic=True)
        np.testing.assert_array_equal(sh.to_numpy(), ref.data)


@pytest.mark.parametrize("n", [(1 << 26) + 1, (2 << 26) + 1])
def test_windowed_sweep_odd_record_once(gpu, n):
    """A dense push is applied in windows of 2^26 records; with n = k * 2^26 + 1 the window before the
    last also ends at pair n >> 1, and the odd last record must still be added once (it was added by
    both windows before the fix)."""
    import torch
    d = torch.device("cuda", gpu)
    for dtype in ("long", "double"):
        part = RangePartition(0, 0, n + 5)
        with PartialVector(part, dtype, gpu) as sh:
            keys = torch.arange(n, dtype=torch.int64, device=d)
            if dtype == "long":
                vals = torch.arange(1, n + 1, dtype=torch.int64, device=d)
            else:
                vals = torch.arange(1, n + 1, dtype=torch.float64, device=d) * 0.5
            sh.update(keys, vals)
            sh.update(keys, vals)
            got = sh.get(torch.arange(n + 5, dtype=torch.int64, device=d))
            want = torch.zeros(n + 5, dtype=vals.dtype, device=d)
            want[:n] = 2 * vals
            assert torch.equal(got, want), f"{dtype} n={n}"


@pytest.mark.parametrize("pattern", ["dense", "zipf_binned", "small", "matrix"])
def test_gated_push(gpu, pattern):
    """glint_*_push_dev_gated: with the gate word set the push applies nothing and reports nothing;
    with it clear the push is the plain device push; a cancelled push leaves no trace on the pushes
    after it (the LaunchCtl slots alternate and each check clears the next one's cancel word)."""
    import torch
    d = torch.device("cuda", gpu)
    rng = np.random.default_rng(17)
    size = 1 << 22
    if pattern == "matrix":
        part = RangePartition(0, 0, 1 << 12)
        sh = PartialMatrix(part, 512, "long", gpu)
        r = torch.from_numpy(rng.integers(0, 1 << 12, 1 << 21).astype(np.int64)).to(d)
        c = torch.from_numpy(rng.integers(0, 512, 1 << 21).astype(np.int32)).to(d)
        v = torch.from_numpy(rng.integers(-9, 9, 1 << 21).astype(np.int64)).to(d)
        args = (r, c, v)
        flat = r * 512 + c.to(torch.int64)
        ref = torch.zeros((1 << 12) * 512, dtype=torch.int64, device=d)
    else:
        part = RangePartition(0, 0, size)
        sh = PartialVector(part, "long", gpu)
        if pattern == "dense":
            k = torch.arange(size, dtype=torch.int64, device=d)
        elif pattern == "small":
            k = torch.from_numpy(rng.integers(0, size, 1000).astype(np.int64)).to(d)
        else:
            k = torch.from_numpy(np.minimum(rng.zipf(1.1, 1 << 21) - 1, size - 1).astype(np.int64)).to(d)
        v = torch.from_numpy(rng.integers(-9, 9, k.numel()).astype(np.int64)).to(d)
        args = (k, v)
        flat = k
        ref = torch.zeros(size, dtype=torch.int64, device=d)
    on = torch.ones(1, dtype=torch.int64, device=d)
    off = torch.zeros(1, dtype=torch.int64, device=d)
    with sh:
        def state():
            if pattern == "matrix":
                return sh.getRows(torch.arange(1 << 12, dtype=torch.int64, device=d)).reshape(-1)
            return sh.get(torch.arange(size, dtype=torch.int64, device=d))
        for gate, applied in ((off, True), (on, False), (off, True), (on, False), (on, False), (None, True),
                              (off, True)):
            sh.update(*args, gate=gate)  # sync=True: a cancelled push reports no error either
            if applied:
                ref.index_add_(0, flat, args[-1])
            assert torch.equal(state(), ref)


@pytest.mark.parametrize("pattern", ["dense", "zipf", "small", "matrix", "sorted_bad", "empty", "wrap", "zipf_wrap",
                                     "head_bad"])
@pytest.mark.parametrize("word", ["device", "host"])
def test_validating_gated_push(gpu, pattern, word):
    """GLINT_PUSH_VALIDATE: the gated push checks its own records and writes the verdict -- 0, or
    ~(first out-of-range record) -- to the gate word; a batch with a bad record applies NOTHING (not
    its dense head, not its tail), as mapPartitions throws before sending (AsyncBigVector.scala:96-98);
    a clean batch is the plain device push. Pushes after a cancelled one are unaffected. Once the
    pushes' unordered tails are large (zipf*, head_bad), the tail is binned and the check is split: the
    count pass validates the tail and push_check the sorted head before it (zipf_wrap: keys 2^32 away
    from in-range ones in the tail; head_bad: the bad key inside a 2^20-record sorted head)."""
    import torch
    d = torch.device("cuda", gpu)
    rng = np.random.default_rng(23)
    size = 1 << 22
    if pattern == "matrix":
        part = RangePartition(0, 0, 1 << 12)
        sh = PartialMatrix(part, 512, "long", gpu)
        r = torch.from_numpy(rng.integers(0, 1 << 12, 1 << 21).astype(np.int64)).to(d)
        c = torch.from_numpy(rng.integers(0, 512, 1 << 21).astype(np.int32)).to(d)
        v = torch.from_numpy(rng.integers(-9, 9, 1 << 21).astype(np.int64)).to(d)
        good = (r, c, v)
        c_bad = c.clone()
        c_bad[777_777] = 512  # a column outside the matrix
        c_bad[1_500_000] = -1
        bad, first = (r, c_bad, v), 777_777
        flat = r * 512 + c.to(torch.int64)
        ref = torch.zeros((1 << 12) * 512, dtype=torch.int64, device=d)
    else:
        part = RangePartition(0, 0, size)
        sh = PartialVector(part, "long", gpu)
        if pattern in ("dense", "sorted_bad", "wrap"):
            k = torch.arange(size, dtype=torch.int64, device=d)
        elif pattern == "small":
            k = torch.from_numpy(rng.integers(0, size, 1000).astype(np.int64)).to(d)
        elif pattern == "empty":
            k = torch.empty(0, dtype=torch.int64, device=d)
        elif pattern == "head_bad":
            tail = np.minimum(rng.zipf(1.1, 1 << 20) - 1, size - 1)
            k = torch.from_numpy(np.concatenate([np.arange(1 << 20), tail]).astype(np.int64)).to(d)
        else:
            k = torch.from_numpy(np.minimum(rng.zipf(1.1, 1 << 21) - 1, size - 1).astype(np.int64)).to(d)
        v = torch.from_numpy(rng.integers(-9, 9, k.numel()).astype(np.int64)).to(d)
        good = (k, v)
        kb = k.clone()
        first = -1
        if k.numel():
            # sorted_bad: a dense increasing head, then the bad key (and a break after it)
            first = k.numel() // 2 if pattern == "sorted_bad" else min(k.numel() - 1, 123_457)
            if pattern == "head_bad":
                first = 1000
                kb[first] = -5  # inside the sorted head
                kb[-1] = size + 9  # and one in the tail
            elif pattern in ("wrap", "zipf_wrap"):  # 2^32 away from in-range keys: (key - start).toInt aliases them
                kb[first] = int(k[first]) + 2**32
                kb[-1] = -(2**32) + 1
            else:
                kb[first] = size + 5
                kb[-1] = -3 if k.numel() - 1 != first else kb[-1]
        bad = (kb, v)
        flat = k
        ref = torch.zeros(size, dtype=torch.int64, device=d)
    from glint_amd.shard import HostBuffer
    hb = HostBuffer(64) if word == "host" else None  # the verdict read from pinned host memory
    if hb is not None:
        hw = hb.array(np.int64, 1)
        hw[0] = 12345
    dw = torch.full((1,), 12345, dtype=torch.int64, device=d)  # overwritten by every push
    gate = hb.ptr if hb is not None else dw

    def verdict():
        return int(hw[0]) if hb is not None else int(dw.cpu()[0])
    with sh:
        def state():
            if pattern == "matrix":
                return sh.getRows(torch.arange(1 << 12, dtype=torch.int64, device=d)).reshape(-1)
            return sh.get(torch.arange(size, dtype=torch.int64, device=d))
        for batch, ok in ((good, True), (bad, False), (good, True), (bad, False), (bad, False), (good, True)):
            if batch is bad and first < 0:
                continue
            sh.update(*batch, gate=gate, validate=True)
            w = verdict()
            if ok:
                assert w == 0
                ref.index_add_(0, flat, batch[-1])
            else:
                assert w != 0 and ~w == first, (w, first)
            assert torch.equal(state(), ref)
    if hb is not None:
        hb.free()


def test_zipf_fixture_default_mode(gpu):
    z = np.load(GOLD / "zipf_push.npz")
    start, size = int(z["start"]), int(z["size"])
    part = RangePartition(0, start, start + size)
    with PartialVector(part, "long", gpu) as sh:
        sh.update(z["keys"], z["values_i64"])
        np.testing.assert_array_equal(sh.to_numpy(), z["expect_i64"])
    with PartialVector(part, "double", gpu) as sh:
        sh.update(z["keys"], z["values_f64"])
        np.testing.assert_allclose(sh.to_numpy(), z["expect_f64"], rtol=1e-6, atol=1e-9)


def test_int_wraparound(gpu):
    """Int/Long adds wrap (two's complement), as on the JVM."""
    part = RangePartition(0, 0, 4)
    with PartialVector(part, "int", gpu) as sh:
        sh.update([0, 0, 1, 1], np.array([2**31 - 1, 5, -2**31, -1], np.int32))
        np.testing.assert_array_equal(sh.get([0, 1]), np.array([-2**31 + 4, 2**31 - 1], np.int32))
    with PartialVector(part, "long", gpu) as sh:
        sh.update([2, 2], np.array([2**63 - 1, 1], np.int64))
        assert sh.get([2])[0] == -2**63


def test_cyclic_partition_shard(gpu):
    P, Nk = 7, 100_003
    rng = np.random.default_rng(5)
    for idx in (0, 3, 6):
        part = CyclicPartition(idx, P, Nk)
        owned = np.arange(idx, Nk, P, dtype=np.int64)
        keys = rng.choice(owned, 40_000)
        vals = rng.uniform(-1, 1, keys.size)
        ref = oracle_vec(part, "double")
        with PartialVector(part, "double", gpu) as sh:
            assert sh.size == ref.size
            sh.update(np.sort(owned), np.ones(owned.size))
            ref.update(np.sort(owned), np.ones(owned.size))
            sh.update(keys, vals, deterministic=True)
            ref.update(keys, vals)
            np.testing.assert_array_equal(sh.to_numpy(), ref.data)


def test_out_of_range_raises(gpu):
    part = RangePartition(1, 100, 200)
    with PartialVector(part, "long", gpu) as sh:
        with pytest.raises(ArrayIndexOutOfBoundsException) as ei:
            sh.update([100, 150, 200, 120], [1, 1, 1, 1])
        assert ei.value.record == 2
        with pytest.raises(ArrayIndexOutOfBoundsException):
            sh.get([99])
        sh.zero()  # Akka restart semantics
        assert sh.get([100, 150]).tolist() == [0, 0]
        # the reference's (key - start).toInt aliasing is reproduced, not rejected
        sh.update([100 + (1 << 32) + 7], [5])
        assert sh.get([107])[0] == 5


# ---- small pushes: the one-launch path (<= 4096 records, the Akka message sizes) ------------------
@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("n,pattern", [(1000, "dense"), (1000, "duplicates"), (4096, "permutation"),
                                       (4097, "permutation"), (4096, "duplicates"), (3, "single_bad")])
def test_small_push(gpu, dtype, n, pattern):
    """Akka-sized messages (GranularBigVectorSpec.scala:21 slices 1000 records per push), replayed
    many times onto one shard as a server sees them; 4096/4097 straddle the single-launch bound."""
    rng = np.random.default_rng(zlib.crc32(f"small/{dtype}/{n}/{pattern}".encode()))
    start, size = 77, 10_000
    part = RangePartition(0, start, start + size)
    ref = oracle_vec(part, dtype)
    with PartialVector(part, dtype, gpu) as sh:
        if pattern == "single_bad":  # record 1 is out of range: the others are applied, as in the reference
            with pytest.raises(ArrayIndexOutOfBoundsException) as ei:
                sh.update([start, start + size, start + 5], rand_vals(rng, dtype, 3))
            assert ei.value.record == 1
            return
        for m in range(20):
            if pattern == "dense":
                keys = (np.arange(n, dtype=np.int64) + m * n // 4) % size + start
            elif pattern == "permutation":
                keys = rng.permutation(size)[:n].astype(np.int64) + start
            else:
                keys = rng.integers(0, 64, n).astype(np.int64) + start
            vals = rand_vals(rng, dtype, n)
            assert sh.update(keys, vals)
            assert ref.update(keys, vals) == -1
        got = sh.to_numpy()
        if dtype in ("long", "int") or pattern != "duplicates":
            np.testing.assert_array_equal(got, ref.data)
        else:
            np.testing.assert_allclose(got, ref.data, rtol=1e-6 if dtype == "double" else 1e-4,
                                       atol=1e-9 if dtype == "double" else 2e-3)
        np.testing.assert_array_equal(sh.get(keys), got[keys - start])


# ---- matrix ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("cols", [512, 300, 7, 1])
def test_matrix_push_pull(gpu, dtype, cols):
    rng = np.random.default_rng(cols * 31 + len(dtype))
    start, nrows = 4096, 2000
    part = RangePartition(1, start, start + nrows)
    ref = O.OracleMatrix(O.part_range(start, start + nrows), cols, O.CODE[dtype])
    n = 150_000
    rows = rng.integers(0, nrows, n).astype(np.int64) + start
    cl = rng.integers(0, cols, n).astype(np.int32)
    vals = rand_vals(rng, dtype, n)
    # dense row-major sweep (unique, increasing addresses) then random triplets with duplicates
    dr = np.repeat(np.arange(start, start + nrows, dtype=np.int64), cols)
    dc = np.tile(np.arange(cols, dtype=np.int32), nrows)
    dv = rand_vals(rng, dtype, dr.size)
    with PartialMatrix(part, cols, dtype, gpu) as sh:
        sh.update(dr, dc, dv)
        ref.update(dr, dc, dv)
        np.testing.assert_array_equal(sh.to_numpy(), ref.data)
        sh.update(rows, cl, vals, deterministic=True)
        ref.update(rows, cl, vals)
        np.testing.assert_array_equal(sh.to_numpy(), ref.data)
        np.testing.assert_array_equal(sh.get(rows[:5000], cl[:5000]), ref.get(rows[:5000], cl[:5000])[0])
        q = rng.integers(0, nrows, 777).astype(np.int64) + start
        np.testing.assert_array_equal(sh.getRows(q), ref.get_rows(q)[0])
        with pytest.raises(ArrayIndexOutOfBoundsException):
            sh.update([start], [cols], np.ones(1, dtype=sh.np_dtype))
        with pytest.raises(ArrayIndexOutOfBoundsException):
            sh.getRows([start + nrows])


# ---- wire ingest --------------------------------------------------------------------------------
def test_wire_push_pull_vector(gpu):
    rng = np.random.default_rng(9)
    part = RangePartition(0, 0, 10_000)
    keys = rng.integers(0, 10_000, 5001).astype(np.int64)
    vals = rng.uniform(-1, 1, keys.size)
    ref = oracle_vec(part, "double")
    ref.update(keys, vals)
    with PartialVector(part, "double", gpu) as sh:
        mid = sh.push_wire(O.encode_push_vector(O.O_F64, 77, keys, vals), deterministic=True)
        assert mid == 77
        resp = sh.pull_wire(O.encode_pull_vector(keys))
        d = O.decode_response(resp)
        assert resp[0] == 0x10
        np.testing.assert_array_equal(d["values"], ref.get(keys)[0])
        with pytest.raises(ValueError):
            sh.push_wire(O.encode_push_vector(O.O_F32, 1, keys, vals))  # wrong value type


def test_wire_push_pull_matrix(gpu):
    rng = np.random.default_rng(10)
    part = RangePartition(0, 50, 150)
    ref = O.OracleMatrix(O.part_range(50, 150), 64, O.O_I32)
    rows = rng.integers(50, 150, 3000).astype(np.int64)
    cols = rng.integers(0, 64, 3000).astype(np.int32)
    vals = rng.integers(-1000, 1000, 3000).astype(np.int32)
    ref.update(rows, cols, vals)
    with PartialMatrix(part, 64, "int", gpu) as sh:
        assert sh.push_wire(O.encode_push_matrix(O.O_I32, 5, rows, cols, vals)) == 5
        d = O.decode_response(sh.pull_wire(O.encode_pull_matrix(rows[:100], cols[:100])))
        np.testing.assert_array_equal(d["values"], ref.get(rows[:100], cols[:100])[0])
        q = np.array([50, 149, 77], np.int64)
        resp = sh.pull_wire(O.encode_pull_matrix_rows(q))
        assert resp == O.encode_response_rows(O.O_I32, ref.get_rows(q)[0])


# ---- device-resident path (torch tensors in HBM) -----------------------------------------------------
def test_device_resident_push_pull(gpu):
    import torch
    dev = torch.device("cuda", gpu)
    n = 1 << 20
    part = RangePartition(0, 0, n)
    with PartialVector(part, "double", gpu) as sh:
        keys = torch.arange(n, dtype=torch.int64, device=dev)
        vals = torch.rand(n, dtype=torch.float64, device=dev)
        sh.update(keys, vals)
        sh.update(keys, vals)
        out = sh.get(keys)
        torch.testing.assert_close(out, vals + vals, rtol=0, atol=0)
        # misaligned (odd offset) device pointers take the scalar path
        sh.update(keys[1:], vals[1:])
        out = sh.get(keys[1:])
        torch.testing.assert_close(out, 3 * vals[1:], rtol=0, atol=0)
        with pytest.raises(ArrayIndexOutOfBoundsException):
            sh.update(torch.tensor([n], dtype=torch.int64, device=dev),
                      torch.ones(1, dtype=torch.float64, device=dev))


@pytest.mark.slow
def test_large_dense_push_property(gpu):
    """BASELINE cfg2 size (2^28 keys): push the same dense stream twice, every element == 2 v."""
    import torch
    dev = torch.device("cuda", gpu)
    n = 1 << 28
    part = RangePartition(0, 0, n)
    with PartialVector(part, "double", gpu) as sh:
        keys = torch.arange(n, dtype=torch.int64, device=dev)
        vals = torch.rand(n, dtype=torch.float64, device=dev)
        sh.update(keys, vals)
        sh.update(keys, vals)
        out = sh.get(keys)
        assert torch.equal(out, vals * 2)


# ---- client routing on the device (glint_route_dev) against the oracle's bucketing -------------------
def route_dev(keys_np, kind, nparts, nkeys, dev=0):
    import ctypes as C
    import torch
    lib = N.load()
    keys = torch.from_numpy(keys_np).to(torch.device("cuda", dev))
    counts = torch.full((nparts,), -7, dtype=torch.int64, device=keys.device)
    order = torch.full((max(keys.numel(), 1),), -7, dtype=torch.int64, device=keys.device)
    bad = C.c_int64(-2)
    rc = lib.glint_route_dev(keys.data_ptr(), keys.numel(), kind, nparts, nkeys, counts.data_ptr(),
                             order.data_ptr(), C.byref(bad), torch.cuda.current_stream(keys.device).cuda_stream)
    return rc, bad.value, counts.cpu().numpy(), order[:keys.numel()].cpu().numpy()


@pytest.mark.parametrize("nparts", [1, 2, 7, 64, 1000, 8192])
@pytest.mark.parametrize("n", [0, 1, 4095, 4096, 4097, 100_003, 1 << 22])
def test_route_range_matches_oracle(gpu, nparts, n):
    nkeys = 1_000_003
    if nparts > nkeys:
        pytest.skip("more partitions than keys")
    rng = np.random.default_rng(n + nparts)
    keys = rng.integers(0, nkeys, n).astype(np.int64)
    if n > 100:
        keys[: n // 3] = np.sort(keys[: n // 3])  # ordered runs next to random ones
    rc, bad, counts, order = route_dev(keys, N.GLINT_ROUTE_RANGE, nparts, nkeys, gpu)
    assert rc == N.GLINT_OK and bad == -1
    c_ref, _, o_ref = O.bucket_range(keys, nparts, nkeys)
    np.testing.assert_array_equal(counts, c_ref)
    np.testing.assert_array_equal(order, o_ref)  # stable: identical permutation


@pytest.mark.parametrize("nparts", [1, 3, 8, 4096])
def test_route_cyclic_matches_host(gpu, nparts):
    from glint_amd.partitioning import CyclicPartitioner
    nkeys = (1 << 31) + 11  # keys beyond Int range: Long modulo, as CyclicPartitioner.partition
    rng = np.random.default_rng(nparts)
    keys = rng.integers(0, nkeys, 300_001).astype(np.int64)
    rc, bad, counts, order = route_dev(keys, N.GLINT_ROUTE_CYCLIC, nparts, nkeys, gpu)
    assert rc == N.GLINT_OK and bad == -1
    owner = CyclicPartitioner.apply(nparts, nkeys).partition_indices(keys)
    np.testing.assert_array_equal(counts, np.bincount(owner, minlength=nparts))
    np.testing.assert_array_equal(order, np.argsort(owner, kind="stable"))


def test_route_range_odd_partitioner_sizes(gpu):
    """Large and small partitions (RangePartitioner.apply with N % P != 0) and P > N/2."""
    for nparts, nkeys in [(7, 100), (60, 100), (100, 100), (3, 1 << 32)]:
        rng = np.random.default_rng(nkeys)
        keys = rng.integers(0, nkeys, 50_000).astype(np.int64)
        keys[:nparts] = np.arange(nparts) * (nkeys // nparts)
        rc, bad, counts, order = route_dev(keys, N.GLINT_ROUTE_RANGE, nparts, nkeys, gpu)
        assert rc == N.GLINT_OK
        c_ref, _, o_ref = O.bucket_range(keys, nparts, nkeys)
        np.testing.assert_array_equal(counts, c_ref)
        np.testing.assert_array_equal(order, o_ref)


def test_route_out_of_range_reports_first_bad(gpu):
    keys = np.arange(20_000, dtype=np.int64)
    keys[12_345] = 20_000
    keys[15_000] = -1
    rc, bad, _, _ = route_dev(keys, N.GLINT_ROUTE_RANGE, 4, 20_000, gpu)
    assert rc == N.GLINT_EOUTOFRANGE and bad == 12_345
    rc, bad, _, _ = route_dev(keys, N.GLINT_ROUTE_CYCLIC, 4, 20_000, gpu)
    assert rc == N.GLINT_EOUTOFRANGE and bad == 12_345
    assert route_dev(keys, N.GLINT_ROUTE_RANGE, 8193, 20_000, gpu)[0] == N.GLINT_EINVAL


# ---- the exchange layer with HBM shards: gloo world 2 (both ranks on this GPU), nccl world 1 --------
@pytest.mark.parametrize("backend,world,case", [
    ("gloo", 2, "vec_range"), ("gloo", 2, "vec_range_mps3"), ("gloo", 2, "vec_cyclic_mps2"),
    ("gloo", 2, "vec_long_few_keys"), ("gloo", 2, "mat_range_mps2"),
    ("nccl", 1, "vec_range_mps3"), ("nccl", 1, "vec_range"), ("nccl", 1, "mat_range"),
    # the partitions of a rank in one slab (dist.slab_shards)
    ("nccl", 1, "vec_slab_long_mps8"), ("nccl", 1, "vec_slab_double_mps4"), ("nccl", 1, "vec_slab_long_mps3_unaligned"),
    ("nccl", 1, "vec_range_mps4_aligned"), ("nccl", 1, "mat_range_mps4_aligned"), ("nccl", 1, "vec_set_long_mps8"),
    # world 2: every rank's slab, keys rebased by the route (rank r hosts r, r + 2, ...)
    ("gloo", 2, "vec_slab_long_mps8"), ("gloo", 2, "vec_slab_long_mps3_unaligned"), ("gloo", 2, "vec_range_mps4_aligned"),
    ("gloo", 2, "vec_set_long_mps8")])
def test_dist_exchange_on_gpu(gpu, backend, world, case):
    import socket
    import torch.multiprocessing as mp
    import dist_workers
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(dist_workers.run_case, args=(world, port, backend, case, True), nprocs=world, join=True)


# ---- binned unordered push (GLINT_PUSH_UNORDERED, and the adaptive switch) ----------------------------
@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("pattern", ["permutation", "uniform", "zipf", "hot_slab", "with_prefix"])
def test_binned_push(gpu, dtype, pattern):
    rng = np.random.default_rng(zlib.crc32(f"binned/{dtype}/{pattern}".encode()))
    start, size = 5_000_000, 1_000_003  # 123 slabs, the last one partial (odd element count)
    part = RangePartition(1, start, start + size)
    if pattern == "permutation":
        keys = rng.permutation(size).astype(np.int64)
    elif pattern == "uniform":
        keys = rng.integers(0, size, 700_000).astype(np.int64)
    elif pattern == "zipf":
        keys = np.minimum(rng.zipf(1.2, 600_000) - 1, size - 1).astype(np.int64)
        keys = rng.permutation(size)[keys].astype(np.int64)
    elif pattern == "hot_slab":  # one slab with > kBinItem records: split items flush with atomics
        keys = np.concatenate([rng.integers(0, 8192, 100_000), rng.integers(0, size, 50_000)]).astype(np.int64)
        keys = rng.permutation(keys)
    else:  # an increasing prefix then an unordered tail (adaptive path masks the prefix on the device)
        keys = np.concatenate([np.arange(0, size, 3), rng.integers(0, size, 300_000)]).astype(np.int64)
    keys += start
    keys[-1] = size - 1 + start  # the shard's last element (odd-count edge)
    vals = rand_vals(rng, dtype, keys.size)
    ref = oracle_vec(part, dtype)
    with PartialVector(part, dtype, gpu) as sh:
        lib = N.load()
        lib.glint_prof_enable(sh.handle, 1)
        for _ in range(2):
            sh.update(keys, vals, unordered=True)
            assert ref.update(keys, vals) == -1
        import ctypes as C
        ms, cnt = C.c_double(), C.c_int64()
        lib.glint_prof_read(sh.handle, N.GLINT_K_PUSH_BINNED, C.byref(ms), C.byref(cnt))
        assert cnt.value == 2, "the unordered hint must take the binned path"
        got = sh.to_numpy()
        if dtype in ("long", "int") or pattern == "permutation":
            np.testing.assert_array_equal(got, ref.data)  # unique keys: 0 + v is exact, then one add
        else:
            np.testing.assert_allclose(got, ref.data, rtol=1e-6 if dtype == "double" else 1e-4,
                                       atol=1e-9 if dtype == "double" else 2e-3)


def test_binned_adaptive_switch_and_errors(gpu, monkeypatch):
    import ctypes as C
    lib = N.load()
    start, size = 0, 1 << 22
    part = RangePartition(0, start, start + size)
    rng = np.random.default_rng(5)
    keys = rng.integers(0, size, 1 << 21).astype(np.int64)
    vals = rng.integers(-5, 5, keys.size).astype(np.int64)
    ref = oracle_vec(part, "long")
    monkeypatch.delenv("GLINT_BINNED", raising=False)
    N.reload_env()
    with PartialVector(part, "long", gpu) as sh:
        lib.glint_prof_enable(sh.handle, 1)
        counts = []
        for _ in range(3):
            sh.update(keys, vals)
            assert ref.update(keys, vals) == -1
            ms, cnt = C.c_double(), C.c_int64()
            lib.glint_prof_read(sh.handle, N.GLINT_K_PUSH_BINNED, C.byref(ms), C.byref(cnt))
            counts.append(cnt.value)
        # push 1: no history -> LDS-hash scatter; pushes 2, 3: the previous tail was large -> binned
        assert counts == [0, 1, 2]
        np.testing.assert_array_equal(sh.to_numpy(), ref.data)
        # a sorted dense push afterwards is still exact (the prefix is masked on the device)
        dense = np.arange(size, dtype=np.int64)
        sh.update(dense, np.ones(size, np.int64))
        assert ref.update(dense, np.ones(size, np.int64)) == -1
        np.testing.assert_array_equal(sh.to_numpy(), ref.data)
        # an out-of-range record in a binned push is reported; the other records are not corrupted
        bad = keys.copy()
        bad[1234] = size + 7
        with pytest.raises(ArrayIndexOutOfBoundsException) as ei:
            sh.update(bad, vals, unordered=True)
        assert ei.value.record == 1234
    monkeypatch.setenv("GLINT_BINNED", "0")  # never bin
    N.reload_env()
    with PartialVector(part, "long", gpu) as sh:
        lib.glint_prof_enable(sh.handle, 1)
        for _ in range(2):
            sh.update(keys, vals)
        ms, cnt = C.c_double(), C.c_int64()
        lib.glint_prof_read(sh.handle, N.GLINT_K_PUSH_BINNED, C.byref(ms), C.byref(cnt))
        assert cnt.value == 0
    monkeypatch.setenv("GLINT_BINNED", "1")  # bin every large push, the first one (no history) too
    N.reload_env()
    ref = oracle_vec(part, "long")
    with PartialVector(part, "long", gpu) as sh:
        lib.glint_prof_enable(sh.handle, 1)
        for i in range(2):
            sh.update(keys, vals)
            assert ref.update(keys, vals) == -1
            ms, cnt = C.c_double(), C.c_int64()
            lib.glint_prof_read(sh.handle, N.GLINT_K_PUSH_BINNED, C.byref(ms), C.byref(cnt))
            assert cnt.value == i + 1
        np.testing.assert_array_equal(sh.to_numpy(), ref.data)


def test_binned_switch_density_floor(gpu, monkeypatch):
    """The adaptive switch bins a large unordered tail only from GLINT_BIN_DENSITY (default 512)
    records per 4096-element slab of the shard on: below it the atomic scatter is faster at every
    size measured (tools/tail_ab.py). 2^20 records into a 2^24-element shard (256 per slab) stay on the
    scatter; 2^22 (1024 per slab) are binned; with the floor at 0 the sparse push is binned too."""
    import ctypes as C
    lib = N.load()
    size = 1 << 24
    part = RangePartition(0, 0, size)
    rng = np.random.default_rng(41)
    monkeypatch.delenv("GLINT_BINNED", raising=False)
    monkeypatch.delenv("GLINT_BIN_DENSITY", raising=False)
    N.reload_env()

    def binned(sh):
        ms, cnt = C.c_double(), C.c_int64()
        lib.glint_prof_read(sh.handle, N.GLINT_K_PUSH_BINNED, C.byref(ms), C.byref(cnt))
        return cnt.value
    ref = np.zeros(size, np.int64)
    with PartialVector(part, "long", gpu) as sh:
        lib.glint_prof_enable(sh.handle, 1)
        # (the switch decides from the previous push's tail: binned pushes counted cumulatively)
        for lg, want in ((20, 0), (20, 0), (22, 0), (22, 1), (20, 2), (20, 2)):
            k = rng.integers(0, size, 1 << lg).astype(np.int64)
            v = rng.integers(-9, 9, k.size).astype(np.int64)
            sh.update(k, v)  # a host call ends at a sync point: its tail is the next push's history
            np.add.at(ref, k, v)
            assert binned(sh) == want, (lg, want)
        np.testing.assert_array_equal(sh.to_numpy(), ref)
    monkeypatch.setenv("GLINT_BIN_DENSITY", "0")
    N.reload_env()
    with PartialVector(part, "long", gpu) as sh:
        lib.glint_prof_enable(sh.handle, 1)
        k = rng.integers(0, size, 1 << 20).astype(np.int64)
        for _ in range(2):
            sh.update(k, np.ones(k.size, np.int64))
        assert binned(sh) == 1


@pytest.mark.parametrize("whole", ["1", "0"])
def test_whole_push_bin(gpu, monkeypatch, whole):
    """Once a push broke order in its first tile, the next binned push takes every record from 0 with
    no push_check (a whole-push bin); one whose records all arrive in order sends the push after it
    back to the checked path (its ordered sweep). GLINT_BIN_WHOLE=0 checks every push. Sums exact
    (Long) whichever path each push took."""
    import ctypes as C
    lib = N.load()
    size = 1 << 22
    part = RangePartition(0, 0, size)
    rng = np.random.default_rng(43)
    monkeypatch.delenv("GLINT_BINNED", raising=False)
    monkeypatch.delenv("GLINT_BIN_DENSITY", raising=False)
    monkeypatch.setenv("GLINT_BIN_WHOLE", whole)
    N.reload_env()

    def count(sh, k):
        ms, cnt = C.c_double(), C.c_int64()
        lib.glint_prof_read(sh.handle, k, C.byref(ms), C.byref(cnt))
        return cnt.value
    ref = np.zeros(size, np.int64)
    # (pattern, push_check launches and binned pushes so far)
    if whole == "1":
        seq = (("rand", 1, 0), ("rand", 1, 1), ("rand", 1, 2), ("dense", 1, 3), ("dense", 2, 3), ("rand", 3, 3),
               ("rand", 3, 4))
    else:
        seq = (("rand", 1, 0), ("rand", 2, 1), ("rand", 3, 2), ("dense", 4, 3), ("dense", 5, 3), ("rand", 6, 3),
               ("rand", 7, 4))
    with PartialVector(part, "long", gpu) as sh:
        lib.glint_prof_enable(sh.handle, 1)
        for pat, checks, bins in seq:
            k = rng.integers(0, size, 1 << 21).astype(np.int64) if pat == "rand" else np.arange(size, dtype=np.int64)
            v = rng.integers(-9, 9, k.size).astype(np.int64)
            sh.update(k, v)
            np.add.at(ref, k, v)
            assert (count(sh, N.GLINT_K_PUSH_CHECK), count(sh, N.GLINT_K_PUSH_BINNED)) == (checks, bins), pat
            np.testing.assert_array_equal(sh.to_numpy(), ref)
        bad = rng.integers(0, size, 1 << 21).astype(np.int64)
        bad[4321] = size + 3  # an out-of-range record in a whole-push bin is reported
        with pytest.raises(ArrayIndexOutOfBoundsException) as ei:
            sh.update(bad, np.ones(bad.size, np.int64))
        assert ei.value.record == 4321
    monkeypatch.delenv("GLINT_BIN_WHOLE", raising=False)
    N.reload_env()


def test_adaptive_switch_decides_at_sync_points(gpu, monkeypatch):
    """The binned/scatter choice of a device-resident push comes from the previous pushes' tails as
    of the shard's last sync point, never from a word the device may or may not have written yet:
    unsynchronised pushes keep the path they started with, and the same sequence of pushes and
    syncs takes the same paths on every run."""
    import ctypes as C
    import torch
    lib = N.load()
    d = torch.device("cuda", gpu)
    size = 1 << 22
    part = RangePartition(0, 0, size)
    rng = np.random.default_rng(31)
    keys = torch.from_numpy(rng.integers(0, size, 1 << 21).astype(np.int64)).to(d)
    vals = torch.from_numpy(rng.integers(-5, 5, 1 << 21).astype(np.int64)).to(d)
    monkeypatch.delenv("GLINT_BINNED", raising=False)
    N.reload_env()

    def binned_launches(sh):
        ms, cnt = C.c_double(), C.c_int64()
        lib.glint_prof_read(sh.handle, N.GLINT_K_PUSH_BINNED, C.byref(ms), C.byref(cnt))
        return cnt.value

    runs = []
    for _ in range(2):
        with PartialVector(part, "long", gpu) as sh:
            lib.glint_prof_enable(sh.handle, 1)
            seq = []
            for _ in range(3):  # no sync in between: no history is taken up, the scatter every time
                sh.update(keys, vals, sync=False)
                seq.append(binned_launches(sh))
            sh.sync()
            for _ in range(2):  # after the sync point: the large unordered tail is known -> binned
                sh.update(keys, vals, sync=False)
                seq.append(binned_launches(sh))
            sh.sync()
            np.testing.assert_array_equal(sh.to_numpy(), 5 * np.bincount(keys.cpu().numpy(), vals.cpu().numpy(),
                                                                              minlength=size).astype(np.int64))
            runs.append(seq)
    assert runs[0] == [0, 0, 0, 1, 2] and runs[1] == runs[0]


@pytest.mark.parametrize("dtype", ["double", "int"])
def test_binned_matrix_push(gpu, dtype):
    rng = np.random.default_rng(11)
    rows_n, cols_n = 20_011, 301  # pitch 302 (double) / 304 (int): the row padding stays untouched
    part = RangePartition(0, 0, rows_n)
    r = rng.integers(0, rows_n, 800_000).astype(np.int64)
    c = rng.integers(0, cols_n, r.size).astype(np.int32)
    v = rand_vals(rng, dtype, r.size)
    code = O.CODE[dtype]
    ref = O.OracleMatrix(O.part_range(0, rows_n), cols_n, code)
    assert ref.update(r, c, v) == -1
    with PartialMatrix(part, cols_n, dtype, gpu) as sh:
        sh.update(r, c, v, unordered=True)
        got = sh.to_numpy()
        if dtype == "int":
            np.testing.assert_array_equal(got, ref.data)
        else:
            np.testing.assert_allclose(got, ref.data, rtol=1e-6, atol=1e-9)


def test_binned_dedup_policy(gpu):
    """Duplicate-heavy unordered pushes are summed per chunk in LDS before binning; unique-key
    pushes stop paying for that after one probe. Both stay correct across the switch."""
    rng = np.random.default_rng(3)
    size = 1 << 20
    part = RangePartition(0, 0, size)
    hot = rng.integers(0, 5000, 1 << 20).astype(np.int64)            # ~0.5 % distinct per chunk
    uniq = rng.permutation(size).astype(np.int64)                     # 100 % distinct
    ref = oracle_vec(part, "long")
    with PartialVector(part, "long", gpu) as sh:
        for keys in (hot, uniq, uniq, hot, uniq, hot):
            vals = rng.integers(-9, 9, keys.size).astype(np.int64)
            sh.update(keys, vals, unordered=True)
            assert ref.update(keys, vals) == -1
            np.testing.assert_array_equal(sh.to_numpy(), ref.data)


@pytest.mark.parametrize("front", ["dedup", "hot", "prep"])
@pytest.mark.parametrize("dtype", ["double", "float", "long"])
@pytest.mark.parametrize("pattern", ["zipf", "hot_slab", "uniform", "with_prefix", "one_key", "unique"])
def test_binned_fronts(gpu, monkeypatch, front, dtype, pattern):
    """Every front end of the binned tail (GLINT_BIN_FRONT: per-chunk LDS dedup, plain with the
    hot-element split, plain address prepare) against the oracle, on skewed and flat tails; Long is bit-exact, and so is Float when
    every key occurs once per push (its LDS partial sums are double, LdsAcc in glint_device.h).
    Float sums over duplicates are checked against the exact (float64) sum within 1e-6 of the sum
    of magnitudes per element -- the reference's sequential float order is one rounding of many."""
    monkeypatch.setenv("GLINT_BIN_FRONT", front)
    N.reload_env()
    rng = np.random.default_rng(zlib.crc32(f"fronts/{front}/{dtype}/{pattern}".encode()))
    start, size = 1 << 33, 2_000_003
    part = RangePartition(2, start, start + size)
    n = 1_500_000
    if pattern == "zipf":
        keys = rng.permutation(size)[np.minimum(rng.zipf(1.1, n) - 1, size - 1)]
    elif pattern == "hot_slab":  # a few hundred hot elements inside one slab, plus a uniform tail
        keys = np.concatenate([rng.integers(4096, 4096 + 300, n // 2), rng.integers(0, size, n - n // 2)])
        keys = rng.permutation(keys)
    elif pattern == "uniform":
        keys = rng.integers(0, size, n)
    elif pattern == "with_prefix":  # ordered prefix (plain path), then a skewed unordered tail
        keys = np.concatenate([np.arange(0, size, 2), rng.permutation(size)[np.minimum(rng.zipf(1.3, n) - 1,
                                                                                       size - 1)]])
    elif pattern == "unique":  # every key at most once per push, in random order
        keys = rng.permutation(size)[:n]
    else:  # every record on one element: the whole tail is one hot key
        keys = np.full(n, size - 1)
    keys = keys.astype(np.int64) + start
    if dtype == "long":
        vals = rng.integers(-1 << 40, 1 << 40, keys.size)
    else:
        vals = rand_vals(rng, dtype, keys.size)
    ref = oracle_vec(part, dtype)
    with PartialVector(part, dtype, gpu) as sh:
        for _ in range(2):
            sh.update(keys, vals, unordered=(pattern != "with_prefix"))
            assert ref.update(keys, vals) == -1
        got = sh.to_numpy()
        if dtype == "long" or (dtype == "float" and pattern == "unique"):
            np.testing.assert_array_equal(got, ref.data)
        elif dtype == "double":
            np.testing.assert_allclose(got, ref.data, rtol=1e-6, atol=1e-9)
        else:
            exact = np.zeros(size)
            mag = np.zeros(size)
            np.add.at(exact, keys - start, 2 * vals.astype(np.float64))
            np.add.at(mag, keys - start, 2 * np.abs(vals.astype(np.float64)))
            assert np.all(np.abs(got.astype(np.float64) - exact) <= 1e-6 * mag + 1e-30)
        # an out-of-range record is reported (first bad index) and nothing else is corrupted
        bad = keys.copy()
        bad[777] = start + size + 5
        with pytest.raises(ArrayIndexOutOfBoundsException) as ei:
            sh.update(bad, vals, unordered=True)
        assert ei.value.record == 777


@pytest.mark.parametrize("front", ["dedup", "hot", "prep"])
def test_binned_fronts_matrix(gpu, monkeypatch, front):
    monkeypatch.setenv("GLINT_BIN_FRONT", front)
    N.reload_env()
    rng = np.random.default_rng(23)
    rows_n, cols_n = 30_011, 129  # pitch 130: row padding stays untouched
    part = RangePartition(0, 0, rows_n)
    r = np.minimum(rng.zipf(1.05, 1_200_000) - 1, rows_n - 1).astype(np.int64)
    c = rng.integers(0, cols_n, r.size).astype(np.int32)
    c[::3] = 7  # hot columns of hot rows
    v = rng.integers(-1000, 1000, r.size).astype(np.int64)
    ref = O.OracleMatrix(O.part_range(0, rows_n), cols_n, O.CODE["long"])
    assert ref.update(r, c, v) == -1
    with PartialMatrix(part, cols_n, "long", gpu) as sh:
        sh.update(r, c, v, unordered=True)
        np.testing.assert_array_equal(sh.to_numpy(), ref.data)


@pytest.mark.parametrize("kind,lg", [("matrix", 21), ("vector", 21), ("matrix", 24), ("vector", 24)])
def test_binned_fine_stage_shapes(gpu, kind, lg):
    """The fine stage in each of its shapes, bit-exact (Long) against the oracle: a small push (2^21
    records: <= ~4 fine items per CU) plans its buckets inside bin_fsort, a large one (2^24) launches
    bin_plan; a vector shard groups its sparse neighbour slabs into one unit, a matrix shard does not.
    Zipf keys with hot elements (units split across a slab, flushed by atomics) and cold sparse slabs."""
    rng = np.random.default_rng(29)
    nrec = 1 << lg
    if kind == "matrix":
        rows_n, cols_n = 1 << 13, 512
        part = RangePartition(0, 0, rows_n)
        r = np.minimum(np.floor(np.power(float(rows_n), rng.random(nrec))).astype(np.int64) - 1, rows_n - 1)
        r = rng.permutation(rows_n)[r].astype(np.int64)
        c = rng.integers(0, cols_n, r.size).astype(np.int32)
        v = rng.integers(-1000, 1000, r.size).astype(np.int64)
        ref = O.OracleMatrix(O.part_range(0, rows_n), cols_n, O.CODE["long"])
        sh, args = PartialMatrix(part, cols_n, "long", gpu), (r, c, v)
    else:
        size = 1 << 24
        part = RangePartition(0, 0, size)
        k = np.minimum(np.floor(np.power(float(size), rng.random(nrec))).astype(np.int64) - 1, size - 1)
        k = ((k.astype(np.uint64) * np.uint64(0x9E3779B1)) & np.uint64(size - 1)).astype(np.int64)
        v = rng.integers(-1000, 1000, k.size).astype(np.int64)
        ref = O.OracleVector(O.part_range(0, size), O.CODE["long"])
        sh, args = PartialVector(part, "long", gpu), (k, v)
    with sh:
        for _ in range(2):
            sh.update(*args, unordered=True)
            assert ref.update(*args) == -1
        np.testing.assert_array_equal(sh.to_numpy(), ref.data)


@pytest.mark.parametrize("dtype", ["long", "double"])
def test_binned_stream_of_batches(gpu, dtype):
    """A server sees a stream of different batches (AsyncBigVector.scala:107-121: every push is a new
    message), while the binned push keeps state across pushes: the wide hot table, resampled every 8th
    push, the front-end choice and the whole-push hints, all latched from earlier pushes. Twelve Zipf
    batches from distinct seeds -- with the hot set drifting between them -- pushed with the hint and
    through the adaptive switch, against the oracle's sequential loop over the same stream (Long
    bit-exact, Double within 1e-9 of each element's sum of magnitudes)."""
    size = 1 << 24
    part = RangePartition(0, 0, size)
    ref = O.OracleVector(O.part_range(0, size), O.CODE[dtype])
    mag = np.zeros(size)
    with PartialVector(part, dtype, gpu) as sh:
        for b in range(12):
            rng = np.random.default_rng(1000 + b)
            z = np.minimum(rng.zipf(1.1, 1 << 22) - 1, size - 1)
            shift = (b // 4) * 977  # the hot elements move every fourth batch
            k = (((z + shift).astype(np.uint64) * np.uint64(0x9E3779B1)) & np.uint64(size - 1)).astype(np.int64)
            v = rand_vals(rng, dtype, k.size)
            sh.update(k, v, unordered=b % 3 != 2)
            assert ref.update(k, v) == -1
            mag += np.bincount(k, np.abs(v.astype(np.float64)), minlength=size)
        got = sh.to_numpy()
    if dtype == "long":
        np.testing.assert_array_equal(got, ref.data)
    else:
        assert not (np.abs(got - ref.data) > 1e-9 * mag).any()


def test_loopback_harness_gpu_backend(gpu):
    """configs[0] over loopback TCP with HBM shards fed the raw wire images (glint_push_wire /
    glint_pull_wire): pulled values equal the pushed ones bit for bit."""
    import json
    import subprocess
    from glint_amd.build import LIB, LOOPBACK_BIN
    r = subprocess.run([str(LOOPBACK_BIN), "--backend", "gpu", "--lib", str(LIB), "--device", str(gpu)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout)
    assert d["check"] is True and d["push_messages"] == 1000


@pytest.mark.parametrize("args", [
    ["--clients", "64", "--servers", "8", "--keys", str(1 << 22), "--msg", "1000"],
    ["--clients", "64", "--servers", "8", "--keys", str(1 << 22), "--pattern", "uniform", "--records", "32768",
     "--dtype", "long"],
    ["--clients", "16", "--servers", "4", "--keys", str(1 << 20), "--pattern", "uniform", "--records", "65536"],
])
@pytest.mark.parametrize("server,replies,answers", [("threads", "async", "copy"), ("threads", "burst", "direct"),
                                                    ("threads", "burst", "copy"), ("actor", "burst", "direct"),
                                                    ("actor", "burst", "copy")])
def test_loopback_concurrent_clients_gpu_backend(gpu, args, server, replies, answers):
    """configs[3]'s shape (64 concurrent loopback clients, 8 range-sharded servers -- here all on one
    GPU) with HBM shards: pushes enqueued through the pinned ring and acknowledged once applied, the
    replies written by each connection's reply thread (async) or after one wait per drained burst, by
    the connection's thread or by the server's one actor thread; pull answers written by the GPU
    straight into pinned arenas (direct) or copied out of the ring (copy). Long sums bit-exact, dense
    ranges bit-exact."""
    import json
    import subprocess
    from glint_amd.build import LIB, LOOPBACK_BIN
    r = subprocess.run([str(LOOPBACK_BIN), "--backend", "gpu", "--lib", str(LIB), "--device", str(gpu),
                        "--replies", replies, "--server", server, "--answers", answers] + args,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout)
    assert d["check"] is True and d["resends"] == 0 and d["server"] == server and d["answers"] == answers
    if server == "threads":
        assert d["replies"] == replies


def test_loopback_client_bucketing_offloaded(gpu):
    """the clients' mapPartitions step (AsyncBigVector.scala:96-98) once per batch,
    either as the reference's groupBy restated on the host or offloaded to the GPU (glint_route_dev,
    one stable route of the whole batch). Both send the same messages; with Long values the shards end
    bit-identical (each run's pulled values equal the exact sums), and each run reports its bucketing
    time per client. `auto` routes a batch on the device while fewer than 4 clients are, else on the
    host (the same messages either way)."""
    import json
    import subprocess
    from glint_amd.build import LIB, LOOPBACK_BIN
    out = {}
    for mode in ("groupby", "device", "auto"):
        r = subprocess.run([str(LOOPBACK_BIN), "--backend", "gpu", "--lib", str(LIB), "--device", str(gpu),
                            "--clients", "64", "--servers", "8", "--keys", str(1 << 22), "--pattern", "uniform",
                            "--records", "32768", "--dtype", "long", "--bucket", mode],
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        d = json.loads(r.stdout)
        assert d["check"] is True and d["resends"] == 0 and d["bucket"] == mode
        assert all(x > 0 for x in d["bucket_s_per_client"])
        out[mode] = d
    for mode in ("device", "auto"):
        assert out["groupby"]["push_messages"] == out[mode]["push_messages"]
        assert out["groupby"]["pull_messages"] == out[mode]["pull_messages"]
    assert out["device"]["device_batches"] == 2 * 64 and 0 < out["auto"]["device_batches"] <= 2 * 64


@pytest.mark.parametrize("dtype", ["long", "double", "float", "int"])
def test_large_pull_shapes(gpu, dtype):
    """Large aligned pulls (>= 2^20 records, the windowed gather of record pairs) in the shapes a dense
    stream and its edges take, against the oracle's get: an even and an odd first element (16-B element
    pairs or two 8-B loads), an odd record count (the last record alone), a run broken in the middle and
    at its end, a key out of range (raises with its record, the rest answered), repeated pulls, and a
    cyclic layout whose keys are one dense run of elements."""
    import torch
    from glint_amd import CyclicPartition
    d = torch.device("cuda", gpu)
    rng = np.random.default_rng(61)
    size = (1 << 21) + 77
    part = RangePartition(2, 1000, 1000 + size)
    vals = rand_vals(rng, dtype, size)
    ref = oracle_vec(part, dtype)
    allk = np.arange(1000, 1000 + size, dtype=np.int64)
    assert ref.update(allk, vals) == -1
    with PartialVector(part, dtype, gpu) as sh:
        sh.update(allk, vals)
        cases = [allk[:1 << 20], allk[1:(1 << 20) + 2], allk[3:(1 << 21) + 3], allk[5:]]
        broken = allk[:1 << 21].copy()
        broken[777_777] = broken[5]
        cases.append(broken)
        end = allk[:(1 << 20) + 1].copy()
        end[-1] = allk[0]
        cases.append(end)
        for k in cases + cases[:2]:
            got = sh.get(torch.from_numpy(k).to(d)).cpu().numpy()
            want, bad = ref.get(k)
            assert bad == -1
            np.testing.assert_array_equal(got, want)
        out_of_range = allk[:1 << 20].copy()
        out_of_range[123_456] = 1000 + size + 3
        with pytest.raises(ArrayIndexOutOfBoundsException) as ei:
            sh.get(torch.from_numpy(out_of_range).to(d))
        assert ei.value.record == 123_456
        got = sh.get(torch.from_numpy(allk[:1 << 20]).to(d)).cpu().numpy()  # the shard and the flags unharmed
        np.testing.assert_array_equal(got, ref.get(allk[:1 << 20])[0])
    cpart = CyclicPartition(1, 3, 3 * (1 << 20))  # keys 1, 4, 7, ...: one dense run of elements
    cref = oracle_vec(cpart, dtype)
    ck = np.arange(1, 3 * (1 << 20), 3, dtype=np.int64)
    cv = rand_vals(rng, dtype, ck.size)
    assert cref.update(ck, cv) == -1
    with PartialVector(cpart, dtype, gpu) as sh:
        sh.update(ck, cv)
        np.testing.assert_array_equal(sh.get(torch.from_numpy(ck).to(d)).cpu().numpy(), cref.get(ck)[0])
