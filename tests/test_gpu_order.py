"""Summation order: the actor's update() path must reproduce the JVM's strictly sequential
`data(k) += v` (PartialVector.scala:35-43, PartialMatrix.scala:74-83) bit for bit.

The reference's only Double-order known answer (BufferedBigMatrixSpec.scala:119, 7.02) gives the
same bits under both associations, so it cannot tell a sequential fold from a pre-summed one. The
vectors here are built so that the two orders round differently:
  ((d + a) + b) + c  !=  d + ((a + b) + c)
The sequential value is computed twice -- by Python's own IEEE-754 double arithmetic (the same
round-to-nearest-even `+` the JVM uses for Double) and by the C oracle -- and both must agree before
the GPU is compared with them. Float vectors use numpy float32 scalars the same way.
"""
import zlib

import numpy as np
import pytest

import glint_amd
from glint_amd import Client, PartialMatrix, PartialVector, RangePartition
from oracle import oracle as O

# (initial shard value, values pushed onto ONE key in message order)
ORDER_VECTORS_F64 = [
    (0.0, [1e16, 1.0, 1.0]),             # sequential: each +1 rounds away; pre-summed: +2 survives
    (0.0, [0.1, 0.2, 0.3]),              # 0.6000000000000001 vs 0.6 (summed right to left)
    (1.0, [1e-16, 1e-16, 1e-16, 1e-16]), # sequential stays 1.0; pre-summed moves by one ulp
    (0.54, [1.5, 0.3, 0.54, 1.5, 0.3]),  # BufferedBigMatrixSpec.scala:85-121's values, another start
]
ORDER_VECTORS_F32 = [
    (0.0, [16777216.0, 1.0, 1.0]),       # 2^24: float's integer limit
    (0.0, [0.1, 0.2, 0.3]),
]


def sequential(d0, vals, dt):
    acc = dt(d0)
    for v in vals:
        acc = dt(acc + dt(v))
    return acc


def presummed(d0, vals, dt):
    s = dt(0)
    for v in reversed(vals):
        s = dt(s + dt(v))
    return dt(dt(d0) + s)


def order_push(dtype):
    """One message with every vector on its own key, interleaved (records of different keys
    alternate, as a real message would hold them). Returns (keys, vals, init, expect)."""
    dt = np.float64 if dtype == "double" else np.float32
    vecs = ORDER_VECTORS_F64 if dtype == "double" else ORDER_VECTORS_F32
    keys, vals = [], []
    longest = max(len(v) for _, v in vecs)
    for i in range(longest):
        for k, (_, v) in enumerate(vecs):
            if i < len(v):
                keys.append(k)
                vals.append(v[i])
    init = np.array([d for d, _ in vecs], dt)
    expect = np.array([sequential(d, v, dt) for d, v in vecs], dt)
    return np.array(keys, np.int64), np.array(vals, dt), init, expect


@pytest.mark.parametrize("dtype", ["double", "float"])
def test_order_vectors_pin_the_oracle(dtype):
    """CPU: the vectors distinguish the orders, and the oracle's loop is the sequential one."""
    dt = np.float64 if dtype == "double" else np.float32
    vecs = ORDER_VECTORS_F64 if dtype == "double" else ORDER_VECTORS_F32
    assert any(sequential(d, v, dt) != presummed(d, v, dt) for d, v in vecs)
    keys, vals, init, expect = order_push(dtype)
    ref = O.OracleVector(O.part_range(0, init.size), O.CODE[dtype])
    ref.data[:] = init
    assert ref.update(keys, vals) == -1
    np.testing.assert_array_equal(ref.data, expect)


def _seeded_shard(sh, init):
    """Shard state = init exactly: pushes of one value onto zero are exact."""
    sh.update(np.arange(init.size, dtype=np.int64), init)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["double", "float"])
@pytest.mark.parametrize("path", ["host", "host_det", "wire", "dev_det"])
def test_order_vectors_on_gpu(gpu, dtype, path):
    keys, vals, init, expect = order_push(dtype)
    with PartialVector(RangePartition(0, 0, init.size), dtype, gpu) as sh:
        _seeded_shard(sh, init)
        if path == "host":
            sh.update(keys, vals)
        elif path == "host_det":
            sh.update(keys, vals, deterministic=True)
        elif path == "wire":
            code = O.O_F64 if dtype == "double" else O.O_F32
            assert sh.push_wire(O.encode_push_vector(code, 3, keys, vals)) == 3
        else:
            import torch
            dev = torch.device("cuda", gpu)
            sh.update(torch.from_numpy(keys).to(dev), torch.from_numpy(vals).to(dev), deterministic=True)
        np.testing.assert_array_equal(sh.to_numpy(), expect)


@pytest.mark.gpu
def test_order_vectors_matrix_on_gpu(gpu):
    keys, vals, init, expect = order_push("double")
    cols = 5
    rows = keys // 2
    cl = (keys % 2 * 3).astype(np.int32)  # two cells per row
    with PartialMatrix(RangePartition(0, 0, init.size), cols, "double", gpu) as sh:
        r0 = np.arange(init.size, dtype=np.int64) // 2
        c0 = (np.arange(init.size) % 2 * 3).astype(np.int32)
        sh.update(r0, c0, init)
        sh.update(rows, cl, vals)
        np.testing.assert_array_equal(sh.get(r0, c0), expect)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["double", "float"])
@pytest.mark.parametrize("n", [1000, 4096, 8192, 79_999])
@pytest.mark.parametrize("path", ["host", "dev_det"])
def test_distinct_fast_path_beside_repeats(gpu, dtype, n, path):
    """The fold's flushes add the records of an all-distinct list directly and sort only a list with
    a repeated address. One push mixes both: distinct keys everywhere, plus the order-distinguishing
    vectors on a few keys (their owners' lists take the sorted path). Bit-exact with the oracle."""
    rng = np.random.default_rng(zlib.crc32(f"fast/{dtype}/{n}/{path}".encode()))
    npd = np.float64 if dtype == "double" else np.float32
    vecs = ORDER_VECTORS_F64 if dtype == "double" else ORDER_VECTORS_F32
    size = 1 << 20
    ks = rng.permutation(size)[:n + len(vecs)].astype(np.int64)
    hot, keys = ks[:len(vecs)], list(ks[len(vecs):n])
    vals = list(rng.uniform(-1, 1, len(keys)).astype(npd))
    for (_, v), k in zip(vecs, hot):  # each vector's records at random positions, in its order
        pos = np.sort(rng.choice(len(keys) + len(v), len(v), replace=False))
        for p, x in zip(pos, v):
            keys.insert(int(p), int(k))
            vals.insert(int(p), npd(x))
    keys, vals = np.array(keys, np.int64), np.array(vals, npd)
    init = rng.uniform(-1, 1, size).astype(npd)
    init[hot] = [d for d, _ in vecs]
    ref = O.OracleVector(O.part_range(0, size), O.CODE[dtype])
    ref.data[:] = init
    assert ref.update(keys, vals) == -1
    with PartialVector(RangePartition(0, 0, size), dtype, gpu) as sh:
        _seeded_shard(sh, init)
        if path == "host":
            sh.update(keys, vals)
        else:
            import torch
            dev = torch.device("cuda", gpu)
            sh.update(torch.from_numpy(keys).to(dev), torch.from_numpy(vals).to(dev), deterministic=True)
        got = sh.to_numpy()
    np.testing.assert_array_equal(got[hot], [sequential(d, v, npd) for d, v in vecs])
    np.testing.assert_array_equal(got, ref.data)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["double", "float"])
@pytest.mark.parametrize("n", [1, 1000, 4096, 4097, 79_999, 131_072])
def test_message_sized_pushes_are_sequential(gpu, dtype, n):
    """Akka-sized messages with heavy duplication, replayed onto one shard: the host-pointer path is
    bit-exact with the oracle's sequential loop at every size up to the one-launch bound."""
    rng = np.random.default_rng(zlib.crc32(f"seq/{dtype}/{n}".encode()))
    start, size = 1 << 33, 50_000
    part = RangePartition(0, start, start + size)
    ref = O.OracleVector(O.part_range(start, start + size), O.CODE[dtype])
    npd = np.float64 if dtype == "double" else np.float32
    with PartialVector(part, dtype, gpu) as sh:
        for m in range(4):
            hot = np.minimum(rng.zipf(1.3, n) - 1, size - 1)          # a few very hot keys
            keys = (rng.permutation(size)[hot] + start).astype(np.int64)
            vals = (rng.uniform(-1, 1, n) * 10.0 ** rng.integers(-8, 8, n)).astype(npd)  # mixed magnitudes
            sh.update(keys, vals)
            assert ref.update(keys, vals) == -1
        np.testing.assert_array_equal(sh.to_numpy(), ref.data)


@pytest.mark.gpu
def test_message_sized_matrix_pushes_are_sequential(gpu):
    rng = np.random.default_rng(77)
    rows_n, cols_n = 3000, 300
    part = RangePartition(1, 10_000, 10_000 + rows_n)
    ref = O.OracleMatrix(O.part_range(10_000, 10_000 + rows_n), cols_n, O.O_F64)
    with PartialMatrix(part, cols_n, "double", gpu) as sh:
        for n in (1000, 79_999):
            r = (np.minimum(rng.zipf(1.2, n) - 1, rows_n - 1) + 10_000).astype(np.int64)
            c = np.minimum(rng.zipf(1.5, n) - 1, cols_n - 1).astype(np.int32)
            v = rng.uniform(-1, 1, n) * 10.0 ** rng.integers(-6, 6, n)
            sh.update(r, c, v)
            assert ref.update(r, c, v) == -1
        np.testing.assert_array_equal(sh.to_numpy(), ref.data)


@pytest.mark.gpu
def test_unordered_opt_out_still_correct(gpu):
    """GLINT_PUSH_UNORDERED on a host push takes the unordered scatter: within the north-star
    tolerance, and exact for unique keys."""
    rng = np.random.default_rng(3)
    size = 10_000
    ref = O.OracleVector(O.part_range(0, size), O.O_F64)
    with PartialVector(RangePartition(0, 0, size), "double", gpu) as sh:
        keys = rng.integers(0, 64, 4000).astype(np.int64)
        vals = rng.uniform(-1, 1, keys.size)
        sh.update(keys, vals, unordered=True)
        ref.update(keys, vals)
        np.testing.assert_allclose(sh.to_numpy(), ref.data, rtol=1e-6, atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("deterministic", [False, True])
def test_reference_scenarios_both_modes(kat, gpu, deterministic):
    """Every reference_kat.json scenario in both push modes, bit-exact (the host path keeps the
    message order by default; deterministic=True forces it)."""
    from test_oracle_kat import expected_array
    for sc in kat["scenarios"]:
        client = Client([gpu] * sc["servers"])
        if sc["model"] == "vector":
            m = client.vector(sc["keys"], sc["dtype"], sc["modelsPerServer"])
        else:
            m = client.matrix(sc["rows"], sc["cols"], sc["dtype"], sc["modelsPerServer"])
        code = O.CODE[sc["dtype"]]
        for op in sc["ops"]:
            if op["op"] == "push":
                if sc["model"] == "vector":
                    m.push(op["keys"], op["values"], deterministic=deterministic)
                else:
                    m.push(op["rows"], op["cols"], op["values"], deterministic=deterministic)
            else:
                if op["op"] == "pull_rows":
                    got = m.pull(op["rows"])
                elif sc["model"] == "vector":
                    got = m.pull(op["keys"])
                else:
                    got = m.pull(op["rows"], op["cols"])
                np.testing.assert_array_equal(got, expected_array(op, code, sc.get("cols")), err_msg=sc["spec"])
        m.destroy()
