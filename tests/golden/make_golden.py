"""Writes tests/golden/reference_kat.json and tests/golden/zipf_push.npz.

reference_kat.json is a transcription of the known-answer tests of the reference's own test suite
(rjagerman/glint, src/test/scala/glint/...): the inputs each spec pushes and the outputs it asserts,
as data. Scenario semantics follow SystemTest (src/test/scala/glint/SystemTest.scala:125-184): a
master, `servers` servers and a client; models are created by Client.vector/matrix with
`modelsPerServer` (default 1), i.e. P = min(keys, modelsPerServer * servers) range partitions.

zipf_push.npz is a regression vector for the duplicate-key push path: a seeded Zipf(1.1) push into
a 4096-key Double/Long shard with the shard state the sequential oracle (oracle/glint_oracle.c)
produces. The reference holds no fixture of this kind (its tests are all small), so this one is
pinned only through the oracle, which the KATs above pin.

Run from the repo root:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))

T = "src/test/scala/glint/"


def vec(spec, dtype, keys_total, servers, ops, mps=1):
    return {"spec": spec, "model": "vector", "dtype": dtype, "keys": keys_total, "servers": servers,
            "modelsPerServer": mps, "ops": ops}


def mat(spec, dtype, rows, cols, servers, ops, mps=1):
    return {"spec": spec, "model": "matrix", "dtype": dtype, "rows": rows, "cols": cols, "servers": servers,
            "modelsPerServer": mps, "ops": ops}


def push(keys, values):
    return {"op": "push", "keys": keys, "values": values}


def mpush(rows, cols, values):
    return {"op": "push", "rows": rows, "cols": cols, "values": values}


def pull(keys, expect):
    return {"op": "pull", "keys": keys, "expect": expect}


def mpull(rows, cols, expect):
    return {"op": "pull", "rows": rows, "cols": cols, "expect": expect}


def rowpull(rows, expect_sparse):
    """expect_sparse: per requested row, {col: value}; every other column must be 0."""
    return {"op": "pull_rows", "rows": rows, "expect": expect_sparse}


SCENARIOS = [
    # ---- BigVectorSpec ----------------------------------------------------------------------------
    vec(T + "vector/BigVectorSpec.scala:14-29", "double", 1000, 1,
        [push([0, 999], [0.54, -0.9999]), pull([0, 999], [0.54, -0.9999])]),
    # "store Float values" -- the spec actually creates vector[Double] (BigVectorSpec.scala:34)
    vec(T + "vector/BigVectorSpec.scala:31-46", "double", 9, 1,
        [push([0, 2, 5, 8], [0.0, -0.001, 100.001, 3.14152]), pull([0, 2, 5, 8], [0.0, -0.001, 100.001, 3.14152])]),
    vec(T + "vector/BigVectorSpec.scala:48-63", "int", 1000, 1,
        [push([0, 999, 99, 98, 100], [1090807, -23, 100, 45, 90]),
         pull([0, 999, 99, 98, 100], [1090807, -23, 100, 45, 90])]),
    vec(T + "vector/BigVectorSpec.scala:65-80", "long", 9, 2,
        [push([0, 2, 5, 8], [0, -1, 900800700600, -100200300400500]),
         pull([0, 2, 5, 8], [0, -1, 900800700600, -100200300400500])]),
    vec(T + "vector/BigVectorSpec.scala:82-101", "int", 100, 3,
        [push([0, 2, 5, 8], [10, 10, 20, 30]), push([0, 2, 5, 8], [1, -1, 2, 3]),
         pull([0, 2, 5, 8], [11, 9, 22, 33])]),
    vec(T + "vector/BigVectorSpec.scala:103-128", "int", 10, 3,
        [push([0], [42]), pull([0], [42])]),
    # ---- BigMatrixSpec ----------------------------------------------------------------------------
    mat(T + "matrix/BigMatrixSpec.scala:15-29", "double", 49, 6, 1,
        [mpush([0], [1], [0.54]), mpull([0], [1], [0.54])]),
    mat(T + "matrix/BigMatrixSpec.scala:32-47", "float", 49, 6, 1,
        [mpush([10, 0, 48], [0, 1, 5], [0.0, 0.54, 0.33333]), mpull([10, 0, 48], [0, 1, 5], [0.0, 0.54, 0.33333])],
        mps=8),
    mat(T + "matrix/BigMatrixSpec.scala:49-64", "int", 23, 10, 1,
        [mpush([1, 5, 20], [0, 1, 8], [0, -1000, 23451234]), mpull([1, 5, 20], [0, 1, 8], [0, -1000, 23451234])]),
    mat(T + "matrix/BigMatrixSpec.scala:66-81", "long", 23, 10, 3,
        [mpush([1, 5, 20], [0, 8, 1], [0, -789300200100, 987100200300]),
         mpull([1, 5, 20], [0, 8, 1], [0, -789300200100, 987100200300])]),
    mat(T + "matrix/BigMatrixSpec.scala:82-113", "int", 100, 100, 2,
        [mpush([0, 20, 50, 81], [0, 10, 99, 80], [100, 100, 20, 30]),
         rowpull([0, 20, 50, 81], [{"0": 100}, {"10": 100}, {"99": 20}, {"80": 30}]),
         mpush([0, 20, 50, 81], [0, 10, 99, 80], [1, -1, 2, 3]),
         rowpull([0, 20, 50, 81], [{"0": 101}, {"10": 99}, {"99": 22}, {"80": 33}])], mps=3),
    mat(T + "matrix/BigMatrixSpec.scala:115-134", "int", 9, 100, 2,
        [mpush([0, 2, 5, 8], [0, 10, 99, 80], [100, 100, 20, 30]),
         mpush([0, 2, 5, 8], [0, 10, 99, 80], [1, -1, 2, 3]),
         mpull([0, 2, 5, 8], [0, 10, 99, 80], [101, 99, 22, 33])]),
    mat(T + "matrix/BigMatrixSpec.scala:136-162", "int", 9, 10, 2,
        [mpush([0, 7], [1, 2], [12, 42]), mpull([0, 7], [1, 2], [12, 42])]),
    # ---- BufferedBigMatrixSpec (Double accumulation order, exact equality) -------------------------
    # a flush is one push of the buffered records in insertion order (BufferedBigMatrix.scala:96-111)
    mat(T + "matrix/BufferedBigMatrixSpec.scala:12-45", "double", 49, 6, 2,
        [mpull([0, 48], [1, 5], [0.0, 0.0]),
         mpush([0, 48, 0], [1, 5, 1], [0.54, -0.33, 1.5]),
         mpull([0, 48], [1, 5], [2.04, -0.33])]),
    mat(T + "matrix/BufferedBigMatrixSpec.scala:47-83", "double", 49, 6, 2,
        [mpush([0, 48, 0, 0], [1, 5, 1, 1], [0.54, -0.33, 1.5, 0.3]),
         mpull([0, 48], [1, 5], [2.34, -0.33])]),
    mat(T + "matrix/BufferedBigMatrixSpec.scala:85-121", "double", 49, 6, 2,
        [mpush([0, 48, 0, 0], [1, 5, 1, 1], [0.54, -0.33, 1.5, 0.3]),
         mpush([0, 48, 0, 0], [1, 5, 1, 1], [0.54, -0.33, 1.5, 0.3]),
         mpush([0, 48, 0, 0], [1, 5, 1, 1], [0.54, -0.33, 1.5, 0.3]),
         mpull([0, 48], [1, 5], [7.02, -0.99])]),
]

# large seeded specs: parameters only (inputs are regenerated exactly by the test)
LARGE = [
    {"spec": T + "vector/GranularBigVectorSpec.scala:14-35", "model": "vector", "dtype": "double",
     "keys": 1000000, "servers": 2, "maximumMessageSize": 1000, "values": "java.util.Random(42).nextDouble",
     "first_values": [0.7275636800328681, 0.6832234717598454, 0.30871945533265976]},
    {"spec": T + "matrix/GranularBigMatrixSpec.scala:12-38", "model": "matrix", "dtype": "double",
     "rows": 1000, "cols": 1000, "servers": 2, "maximumMessageSize": 10000,
     "records": "rows(i)=i%1000, cols(i)=i/1000, values(i)=i*3.14, i<1e6", "pull": "elements"},
    {"spec": T + "matrix/GranularBigMatrixSpec.scala:40-70", "model": "matrix", "dtype": "double",
     "rows": 1000, "cols": 1000, "servers": 3, "maximumMessageSize": 10000,
     "records": "rows(i)=i%1000, cols(i)=i/1000, values(i)=i*3.14, i<1e6", "pull": "rows 0..999"},
]

# PartitioningSpec (src/test/scala/glint/partitioning/PartitioningSpec.scala)
PARTITIONING = {
    "cyclic_contains": [[5, 37], [20, 50], [13, 13], [33, 12]],    # :32-62
    "cyclic_unique": [[17, 137]],                                 # :64-77
    "cyclic_oob": {"P": 13, "N": 105, "keys": [105, -2]},         # :79-83
    "range_contains": [[5, 109], [20, 50], [13, 13], [33, 12]],   # :85-115
    "range_unique": [[15, 97]],                                   # :117-130
    "range_oob": {"P": 12, "N": 105, "keys": [105, -2]},          # :132-136
}

# SerializationSpec (src/test/scala/glint/serialization/SerializationSpec.scala): round trips
SERIALIZATION = [
    {"spec": T + "serialization/SerializationSpec.scala:12-20", "type": "PullMatrix", "rows": [0, 1, 2], "cols": [3, 4, 5]},
    {"spec": T + "serialization/SerializationSpec.scala:22-29", "type": "PullMatrixRows", "rows": [0, 1, 2, 5]},
    {"spec": T + "serialization/SerializationSpec.scala:31-38", "type": "PullVector", "keys": [0, 16, 2, 5]},
    {"spec": T + "serialization/SerializationSpec.scala:40-49", "type": "PushMatrix", "dtype": "double", "id": 2, "rows": [0, 5, 9], "cols": [2, 10, 3],
     "values": [0.0, 0.5, 0.99]},
    {"spec": T + "serialization/SerializationSpec.scala:51-60", "type": "PushMatrix", "dtype": "float", "id": 32, "rows": [0, 5, 9], "cols": [2, 10, 3],
     "values": [0.3, 0.6, 10.314]},
    {"spec": T + "serialization/SerializationSpec.scala:62-71", "type": "PushMatrix", "dtype": "int", "id": 16, "rows": [1, 2, 100000000000],
     "cols": [10000, 10, 1], "values": [99, -20, -3500]},
    {"spec": T + "serialization/SerializationSpec.scala:73-82", "type": "PushMatrix", "dtype": "long", "id": 0, "rows": [1, 2, 100000000000],
     "cols": [10000, 10, 1], "values": [5000300200100, -9000100200300, 0]},
    {"spec": T + "serialization/SerializationSpec.scala:84-92", "type": "PushVector", "dtype": "double", "id": 123, "keys": [0, 5, 9],
     "values": [0.0, 0.5, 0.99]},
    {"spec": T + "serialization/SerializationSpec.scala:94-102", "type": "PushVector", "dtype": "float", "id": 9999, "keys": [0, 5, 9],
     "values": [0.3, 0.6, 10.314]},
    {"spec": T + "serialization/SerializationSpec.scala:104-112", "type": "PushVector", "dtype": "int", "id": 231, "keys": [1, 2, 100000000000],
     "values": [99, -20, -3500]},
    {"spec": T + "serialization/SerializationSpec.scala:114-122", "type": "PushVector", "dtype": "long", "id": 213, "keys": [1, 2, 100000000000],
     "values": [5000300200100, -9000100200300, 0]},
    {"spec": T + "serialization/SerializationSpec.scala:124-131", "type": "Response", "dtype": "double", "values": [0.01, 3.1415, -0.999]},
    {"spec": T + "serialization/SerializationSpec.scala:133-140", "type": "Response", "dtype": "float", "values": [100.001, -3.1415, 0.1234]},
    {"spec": T + "serialization/SerializationSpec.scala:142-149", "type": "Response", "dtype": "int", "values": [100, -200, 999123]},
    {"spec": T + "serialization/SerializationSpec.scala:151-158", "type": "Response", "dtype": "long", "values": [0, -200, 9876300200100]},
]

# ClientSpec: number of partitions P = modelsPerServer x servers (ClientSpec.scala:69-107)
CLIENT = [
    {"spec": T + "ClientSpec.scala:69-77", "model": "matrix", "keys": 49, "servers": 2, "modelsPerServer": 1,
     "partitions": 2},
    {"spec": T + "ClientSpec.scala:79-87", "model": "matrix", "keys": 49, "servers": 2, "modelsPerServer": 3,
     "partitions": 6},
    {"spec": T + "ClientSpec.scala:89-97", "model": "vector", "keys": 4200, "servers": 3, "modelsPerServer": 1,
     "partitions": 3},
    {"spec": T + "ClientSpec.scala:99-107", "model": "vector", "keys": 4200, "servers": 3, "modelsPerServer": 8,
     "partitions": 24},
    {"spec": T + "ClientSpec.scala:51-58", "model": "matrix", "keys": 2, "servers": 3, "modelsPerServer": 1,
     "partitions": 2},
]


def zipf_fixture(path: Path) -> None:
    from oracle import oracle as O
    rng = np.random.default_rng(20240607)
    size = 4096
    n = 1 << 14
    ranks = rng.zipf(1.1, size=4 * n)
    ranks = ranks[ranks <= size][:n] - 1
    perm = rng.permutation(size)
    keys = perm[ranks].astype(np.int64) + 1000  # shard range [1000, 1000 + size)
    vals_f = rng.uniform(-1.0, 1.0, size=n)
    vals_l = rng.integers(-(1 << 40), 1 << 40, size=n, dtype=np.int64)
    part = O.part_range(1000, 1000 + size)
    vf = O.OracleVector(part, O.O_F64)
    assert vf.update(keys, vals_f) == -1
    vl = O.OracleVector(part, O.O_I64)
    assert vl.update(keys, vals_l) == -1
    np.savez_compressed(path, start=np.int64(1000), size=np.int64(size), keys=keys, values_f64=vals_f,
                        values_i64=vals_l, expect_f64=vf.data, expect_i64=vl.data)


def main() -> None:
    out = {"source": "rjagerman/glint test suite (transcribed inputs and asserted outputs)",
           "scenarios": SCENARIOS, "large": LARGE, "partitioning": PARTITIONING, "serialization": SERIALIZATION,
           "client": CLIENT}
    (HERE / "reference_kat.json").write_text(json.dumps(out, indent=1) + "\n")
    zipf_fixture(HERE / "zipf_push.npz")
    print("wrote", HERE / "reference_kat.json", HERE / "zipf_push.npz")


if __name__ == "__main__":
    main()
