"""Pins the oracle (oracle/glint_oracle.c + oracle/oracle.py) to the reference's own known answers.

Each scenario of tests/golden/reference_kat.json is a transcribed spec of the reference's test suite;
it is replayed through the oracle the way the reference's client drives the servers:
Client.create's partitioning (Client.scala:71-72), AsyncBigVector/AsyncBigMatrix bucketing
(AsyncBigVector.scala:96-121), one PartialVector/PartialMatrix loop per partition.
CPU only.
"""
import numpy as np
import pytest

from oracle import oracle as O


class OracleModel:
    """A Glint model made of oracle shards: P = min(keys, modelsPerServer * servers) range partitions."""

    def __init__(self, sc):
        self.sc = sc
        self.code = O.CODE[sc["dtype"]]
        self.N = sc["keys"] if sc["model"] == "vector" else sc["rows"]
        self.P = int(min(self.N, sc["modelsPerServer"] * sc["servers"]))
        starts, ends, _, _ = O.range_partitioner(self.P, self.N)
        if sc["model"] == "vector":
            self.shards = [O.OracleVector(O.part_range(s, e), self.code) for s, e in zip(starts, ends)]
        else:
            self.shards = [O.OracleMatrix(O.part_range(s, e), sc["cols"], self.code) for s, e in zip(starts, ends)]

    def push(self, op):
        keys = np.array(op.get("keys", op.get("rows")), np.int64)
        vals = np.array(op["values"], O.NP[self.code])
        _, off, order = O.bucket_range(keys, self.P, self.N)
        for p, sh in enumerate(self.shards):
            idx = order[off[p]:off[p + 1]]
            if idx.size == 0:
                continue
            if self.sc["model"] == "vector":
                assert sh.update(keys[idx], vals[idx]) == -1
            else:
                cols = np.array(op["cols"], np.int32)
                assert sh.update(keys[idx], cols[idx], vals[idx]) == -1

    def pull(self, op):
        keys = np.array(op.get("keys", op.get("rows")), np.int64)
        _, off, order = O.bucket_range(keys, self.P, self.N)
        if op["op"] == "pull_rows":
            out = np.zeros((keys.size, self.sc["cols"]), O.NP[self.code])
        else:
            out = np.zeros(keys.size, O.NP[self.code])
        for p, sh in enumerate(self.shards):
            idx = order[off[p]:off[p + 1]]
            if idx.size == 0:
                continue
            if op["op"] == "pull_rows":
                res, bad = sh.get_rows(keys[idx])
            elif self.sc["model"] == "vector":
                res, bad = sh.get(keys[idx])
            else:
                res, bad = sh.get(keys[idx], np.array(op["cols"], np.int32)[idx])
            assert bad == -1
            out[idx] = res
        return out


def expected_array(op, code, cols=None):
    if op["op"] == "pull_rows":
        exp = np.zeros((len(op["rows"]), cols), O.NP[code])
        for i, row in enumerate(op["expect"]):
            for c, v in row.items():
                exp[i, int(c)] = v
        return exp
    return np.array(op["expect"], O.NP[code])


def replay(sc):
    m = OracleModel(sc)
    for op in sc["ops"]:
        if op["op"] == "push":
            m.push(op)
        else:
            got = m.pull(op)
            exp = expected_array(op, m.code, sc.get("cols"))
            # the reference asserts exact equality (`should equal`) for every type
            assert got.dtype == exp.dtype
            np.testing.assert_array_equal(got, exp, err_msg=sc["spec"])


def test_scenarios(kat):
    assert len(kat["scenarios"]) >= 15
    for sc in kat["scenarios"]:
        replay(sc)


def test_buffered_double_order_is_sequential(kat):
    """BufferedBigMatrixSpec.scala:119 asserts 7.02 exactly: only the reference's sequential order
    produces it (a regrouped sum does not)."""
    vals = [0.54, 1.5, 0.3] * 3
    acc = 0.0
    for v in vals:
        acc += v
    assert acc == 7.02
    reordered = 0.0
    for v in (0.3, 0.54, 0.3, 0.54, 0.3, 1.5, 1.5, 1.5, 0.54):  # same multiset, another order
        reordered += v
    assert reordered == 7.0200000000000005 != 7.02


def test_granular_big_vector(kat):
    """GranularBigVectorSpec.scala:14-35: 1M Double keys on 2 servers, values from
    java.util.Random(42), pushed in messages of <= 1000 records, pulled back exactly."""
    spec = kat["large"][0]
    n = spec["keys"]
    rnd = O.JavaRandom(42)
    values = rnd.nextDoubles(n)
    assert list(values[:3]) == spec["first_values"]
    keys = np.arange(n, dtype=np.int64)
    P = spec["servers"]
    starts, ends, _, _ = O.range_partitioner(P, n)
    shards = [O.OracleVector(O.part_range(s, e), O.O_F64) for s, e in zip(starts, ends)]
    m = spec["maximumMessageSize"]
    for i in range(0, n, m):  # GranularBigVector.push (GranularBigVector.scala:69-80)
        k, v = keys[i:i + m], values[i:i + m]
        _, off, order = O.bucket_range(k, P, n)
        for p, sh in enumerate(shards):
            idx = order[off[p]:off[p + 1]]
            if idx.size:
                assert sh.update(k[idx], v[idx]) == -1
    got = np.concatenate([sh.data for sh in shards])
    np.testing.assert_array_equal(got, values)


@pytest.mark.parametrize("which", [1, 2])
def test_granular_big_matrix(kat, which):
    """GranularBigMatrixSpec.scala:12-70: 1000x1000 Double, 1e6 cells pushed as i*3.14."""
    spec = kat["large"][which]
    R, Cn = spec["rows"], spec["cols"]
    i = np.arange(1_000_000, dtype=np.int64)
    rows, cols, vals = i % 1000, (i // 1000).astype(np.int32), i.astype(np.float64) * 3.14
    P = spec["servers"]
    starts, ends, _, _ = O.range_partitioner(P, R)
    shards = [O.OracleMatrix(O.part_range(s, e), Cn, O.O_F64) for s, e in zip(starts, ends)]
    m = spec["maximumMessageSize"]
    for s0 in range(0, rows.size, m):
        r, c, v = rows[s0:s0 + m], cols[s0:s0 + m], vals[s0:s0 + m]
        _, off, order = O.bucket_range(r, P, R)
        for p, sh in enumerate(shards):
            idx = order[off[p]:off[p + 1]]
            if idx.size:
                assert sh.update(r[idx], c[idx], v[idx]) == -1
    full = np.concatenate([sh.data for sh in shards])
    np.testing.assert_array_equal(full[rows, cols], vals)


# ---- PartitioningSpec ------------------------------------------------------------------------------
def _range_contains(key, s, e):
    return s <= key < e


def test_range_partitioning_invariants(kat):
    P_ = kat["partitioning"]
    for P, N in P_["range_contains"]:
        starts, ends, ns, q = O.range_partitioner(P, N)
        for key in range(N):
            idx = O.range_partition_of(key, ns, q, N)
            assert 0 <= idx < P
            for j in range(P):  # assertKeyInCorrectPartition (PartitioningSpec.scala:20-30)
                assert _range_contains(key, starts[j], ends[j]) == (j == idx)
    for P, N in P_["range_unique"]:
        starts, ends, _, _ = O.range_partitioner(P, N)
        for s, e in zip(starts, ends):
            seen = np.zeros(N, bool)
            for key in range(N):
                if s <= key < e:
                    loc = key - s
                    assert not seen[loc]
                    seen[loc] = True
    oob = P_["range_oob"]
    _, _, ns, q = O.range_partitioner(oob["P"], oob["N"])
    for key in oob["keys"]:
        assert O.range_partition_of(key, ns, q, oob["N"]) == -1


def test_cyclic_partitioning_invariants(kat):
    P_ = kat["partitioning"]
    for P, N in P_["cyclic_contains"]:
        for key in range(N):
            idx = O.cyclic_partition_of(key, P, N)
            assert 0 <= idx < P
            for j in range(P):
                assert ((key % P) == j) == (j == idx)
    for P, N in P_["cyclic_unique"]:
        for j in range(P):
            seen = set()
            for key in range(N):
                if key % P == j:
                    loc = (key - j) // P
                    assert loc not in seen
                    seen.add(loc)
    oob = P_["cyclic_oob"]
    for key in oob["keys"]:
        assert O.cyclic_partition_of(key, oob["P"], oob["N"]) == -1


def test_range_partitioner_sizes():
    """Small partitions first, then N % P partitions of q + 1 (RangePartitioner.scala:62-84)."""
    for P, N in [(8, 1 << 31), (3, 100), (7, 1000003), (33, 12), (1, 5)]:
        starts, ends, ns, q = O.range_partitioner(P, N)
        sizes = ends - starts
        assert sizes.sum() == N
        assert list(sizes) == [q] * ns + [q + 1] * (P - ns)
        assert starts[0] == 0 and all(starts[1:] == ends[:-1])
    starts, ends, _, q = O.range_partitioner(8, 1 << 31)
    assert q == 1 << 28 and ends[-1] == 1 << 31


# RangePartitioner at the Int edge: q = smallPartitionSize = 2^31 - 1, so largePartitionSize
# (an Int, RangePartitioner.scala:18) wraps to Int.MinValue and apply's `start += q + 1` (:78) wraps
# too. Expected values worked by hand from the JVM's rules (Int + wraps; Long / truncates).
INT_EDGE_Q = (1 << 31) - 1
INT_EDGE_CASES = [
    # (P, N, [(key, expected index or -1 for a throw)])
    (3, 3 * INT_EDGE_Q + 2, [(0, 0), (INT_EDGE_Q - 1, 0), (INT_EDGE_Q, 1), (INT_EDGE_Q + (1 << 31) - 1, 1),
                            (INT_EDGE_Q + (1 << 31), 0), (3 * INT_EDGE_Q + 1, 0)]),
    (5, 5 * INT_EDGE_Q + 4, [(INT_EDGE_Q + (1 << 32) - 1, 0), (INT_EDGE_Q + (1 << 32), -1),
                            (5 * INT_EDGE_Q + 3, -1), (5 * INT_EDGE_Q + 4, -1)]),
]


def test_range_partitioner_int_edge():
    from glint_amd.errors import IndexOutOfBoundsException
    from glint_amd.partitioning import RangePartitioner
    for P, N, cases in INT_EDGE_CASES:
        starts, ends, ns, q = O.range_partitioner(P, N)
        assert q == INT_EDGE_Q and ns == 1
        # start after the first large partition: q + (Int)(q + 1) = q - 2^31 = -1 (ends stay Long)
        assert starts[2] == -1 and ends[1] == 2 * q + 1 and ends[2] == 3 * q + 2
        rp = RangePartitioner.apply(P, N)
        assert rp.largePartitionSize == -(1 << 31)
        assert [p.start for p in rp.partitions] == list(starts) and [p.end for p in rp.partitions] == list(ends)
        keys = np.array([k for k, _ in cases if k < N], np.int64)
        for key, want in cases:
            assert O.range_partition_of(key, ns, q, N) == want, (P, key)
            if want < 0:
                with pytest.raises(IndexOutOfBoundsException):
                    rp.partition(key)
            else:
                assert rp.partition(key).index == want
        good = np.array([k for k, w in cases if w >= 0], np.int64)
        np.testing.assert_array_equal(rp.partition_indices(good), [w for _, w in cases if w >= 0])
        if len(good) < len(keys):
            with pytest.raises(IndexOutOfBoundsException):
                rp.partition_indices(keys)


def test_client_partition_counts(kat):
    for c in kat["client"]:
        assert min(c["keys"], c["modelsPerServer"] * c["servers"]) == c["partitions"], c["spec"]


# ---- SerializationSpec ---------------------------------------------------------------------------
def test_serialization_round_trips(kat):
    for m in kat["serialization"]:
        t = m["type"]
        if t == "PullMatrix":
            b = O.encode_pull_matrix(m["rows"], m["cols"])
            assert len(b) == 5 + 12 * len(m["rows"])
            d = O.decode_request(b)
            assert list(d["rows"]) == m["rows"] and list(d["cols"]) == m["cols"]
        elif t == "PullMatrixRows":
            d = O.decode_request(O.encode_pull_matrix_rows(m["rows"]))
            assert list(d["rows"]) == m["rows"]
        elif t == "PullVector":
            b = O.encode_pull_vector(m["keys"])
            assert b[0] == 0x02 and len(b) == 5 + 8 * len(m["keys"])
            assert list(O.decode_request(b)["keys"]) == m["keys"]
        elif t == "PushMatrix":
            code = O.CODE[m["dtype"]]
            b = O.encode_push_matrix(code, m["id"], m["rows"], m["cols"], m["values"])
            assert len(b) == 9 + len(m["rows"]) * (12 + np.dtype(O.NP[code]).itemsize)
            d = O.decode_request(b)
            assert d["id"] == m["id"] and list(d["rows"]) == m["rows"] and list(d["cols"]) == m["cols"]
            np.testing.assert_array_equal(d["values"], np.array(m["values"], O.NP[code]))
        elif t == "PushVector":
            code = O.CODE[m["dtype"]]
            b = O.encode_push_vector(code, m["id"], m["keys"], m["values"])
            assert len(b) == 9 + len(m["keys"]) * (8 + np.dtype(O.NP[code]).itemsize)
            d = O.decode_request(b)
            assert d["id"] == m["id"] and list(d["keys"]) == m["keys"]
            np.testing.assert_array_equal(d["values"], np.array(m["values"], O.NP[code]))
        elif t == "Response":
            code = O.CODE[m["dtype"]]
            d = O.decode_response(O.encode_response(code, m["values"]))
            np.testing.assert_array_equal(d["values"], np.array(m["values"], O.NP[code]))
        else:
            raise AssertionError(t)


def test_push_vector_double_byte_image():
    """Byte layout of PushVectorDouble (RequestSerializer.scala:205-213): type 0x07, n, id, keys, values."""
    b = O.encode_push_vector(O.O_F64, 123, [0, 5, 9], [0.0, 0.5, 0.99])
    assert b[:9] == bytes([0x07, 3, 0, 0, 0, 123, 0, 0, 0])
    assert b[9:17] == (0).to_bytes(8, "little") and b[17:25] == (5).to_bytes(8, "little")
    assert np.frombuffer(b[33:], "<f8").tolist() == [0.0, 0.5, 0.99]


def test_zipf_fixture_matches_oracle():
    """The committed duplicate-key fixture is reproduced by the sequential oracle."""
    from pathlib import Path
    z = np.load(Path(__file__).parent / "golden" / "zipf_push.npz")
    start, size = int(z["start"]), int(z["size"])
    v = O.OracleVector(O.part_range(start, start + size), O.O_F64)
    assert v.update(z["keys"], z["values_f64"]) == -1
    np.testing.assert_array_equal(v.data, z["expect_f64"])
    w = O.OracleVector(O.part_range(start, start + size), O.O_I64)
    assert w.update(z["keys"], z["values_i64"]) == -1
    np.testing.assert_array_equal(w.data, z["expect_i64"])


def test_out_of_range_partial_apply():
    """The reference applies records before the bad one, then throws (PartialVector.scala:37-41)."""
    v = O.OracleVector(O.part_range(10, 20), O.O_I64)
    assert v.update([10, 11, 25, 12], [1, 2, 3, 4]) == 2
    assert list(v.data[:3]) == [1, 2, 0]
    # a key far enough away that (key - start).toInt wraps into range is silently applied
    assert v.update([10 + (1 << 32) + 5], [7]) == -1
    assert v.data[5] == 7
