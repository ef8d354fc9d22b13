"""Python side of the parity oracle -- TEST INFRASTRUCTURE ONLY.

Loads the C restatement (oracle/glint_oracle.c -> oracle/build/libglint_oracle.so) and adds the
pieces that are byte/integer bookkeeping best expressed in numpy/struct:

* ``JavaRandom`` -- java.util.Random (the generator behind scala.util.Random), needed to reproduce
  GranularBigVectorSpec's seeded values (src/test/scala/glint/vector/GranularBigVectorSpec.scala:14-35).
* the wire codec -- RequestSerializer / ResponseSerializer byte images
  (src/main/scala/glint/serialization/RequestSerializer.scala:59-245,
  ResponseSerializer.scala:19-117, type bytes SerializationConstants.scala:24-38).
* ``OracleVector`` / ``OracleMatrix`` -- shard state held in numpy, updated by the C loops.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; the
product (glint_amd) never does. Parity is pinned by the reference's own known-answer tests
(tests/golden/), see oracle/README.md.
"""
from __future__ import annotations

import ctypes as C
import struct
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "build" / "libglint_oracle.so"

O_I32, O_I64, O_F32, O_F64 = 0, 1, 2, 3
NP = {O_I32: np.int32, O_I64: np.int64, O_F32: np.float32, O_F64: np.float64}
CODE = {"int": O_I32, "long": O_I64, "float": O_F32, "double": O_F64}


class _Part(C.Structure):
    _fields_ = [("kind", C.c_int32), ("start", C.c_int64), ("end", C.c_int64), ("index", C.c_int32),
                ("nparts", C.c_int32), ("nkeys", C.c_int64)]


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():  # build only the oracle (gcc), not the product; the build module is
            import importlib.util  # loaded by path (the glint_amd package needs the built product)
            spec = importlib.util.spec_from_file_location("_glint_build", HERE.parent / "glint_amd" / "build.py")
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            mod.build_oracle()
        L = C.CDLL(str(LIB_PATH))
        P, I64, I32 = C.c_void_p, C.c_int64, C.c_int32
        L.oracle_range_partitioner.argtypes = [I32, I64, P, P, P, P]
        L.oracle_range_partitioner.restype = None
        L.oracle_range_partition.argtypes = [I64, I32, I32, I64]
        L.oracle_range_partition.restype = I32
        L.oracle_cyclic_partition.argtypes = [I64, I32, I64]
        L.oracle_cyclic_partition.restype = I32
        L.oracle_cyclic_size.argtypes = [I32, I32, I64]
        L.oracle_cyclic_size.restype = I32
        L.oracle_partition_size.argtypes = [C.POINTER(_Part)]
        L.oracle_partition_size.restype = I32
        L.oracle_vec_update.argtypes = [C.POINTER(_Part), C.c_int, P, I32, P, P, I64]
        L.oracle_vec_update.restype = I64
        L.oracle_vec_get.argtypes = [C.POINTER(_Part), C.c_int, P, I32, P, P, I64]
        L.oracle_vec_get.restype = I64
        L.oracle_mat_update.argtypes = [C.POINTER(_Part), C.c_int, P, I32, I32, P, P, P, I64]
        L.oracle_mat_update.restype = I64
        L.oracle_mat_get.argtypes = [C.POINTER(_Part), C.c_int, P, I32, I32, P, P, P, I64]
        L.oracle_mat_get.restype = I64
        L.oracle_mat_get_rows.argtypes = [C.POINTER(_Part), C.c_int, P, I32, I32, P, P, I64]
        L.oracle_mat_get_rows.restype = I64
        L.oracle_bucket_range.argtypes = [P, I64, I32, I32, I32, I64, P, P, P]
        L.oracle_bucket_range.restype = I64
        L.oracle_vec_update_f64_parallel.argtypes = [I32, P, P, P, P, P, P, I32]
        L.oracle_vec_update_f64_parallel.restype = C.c_int
        _lib = L
    return _lib


# ---- partitioning --------------------------------------------------------------------------------
def range_partitioner(P: int, N: int):
    """RangePartitioner.apply (RangePartitioner.scala:62-84): (starts, ends, n_small, small_size)."""
    starts = np.zeros(P, np.int64)
    ends = np.zeros(P, np.int64)
    ns, q = C.c_int32(), C.c_int32()
    lib().oracle_range_partitioner(P, N, starts.ctypes.data, ends.ctypes.data, C.byref(ns), C.byref(q))
    return starts, ends, ns.value, q.value


def range_partition_of(key: int, n_small: int, small_size: int, N: int) -> int:
    """RangePartitioner.partition (RangePartitioner.scala:27-43) as the .toInt index; -1 where the
    reference throws for the key or a negative index. An Int-overflowed partitioner can also give an
    index >= P (the reference's partitions(idx) throws there too)."""
    return lib().oracle_range_partition(key, n_small, small_size, N)


def cyclic_partition_of(key: int, P: int, N: int) -> int:
    return lib().oracle_cyclic_partition(key, P, N)


def bucket_range(keys: np.ndarray, P: int, N: int):
    """AsyncBigVector.mapPartitions (AsyncBigVector.scala:96-98) as (counts, offsets, order)."""
    keys = np.ascontiguousarray(keys, np.int64)
    _, _, ns, q = range_partitioner(P, N)
    counts = np.zeros(P, np.int64)
    offsets = np.zeros(P + 1, np.int64)
    order = np.zeros(max(keys.size, 1), np.int64)
    bad = lib().oracle_bucket_range(keys.ctypes.data, keys.size, P, ns, q, N, counts.ctypes.data,
                                    offsets.ctypes.data, order.ctypes.data)
    if bad >= 0:
        raise IndexError(f"key {int(keys[bad])} outside the key space")
    return counts, offsets, order[:keys.size]


def part_range(start: int, end: int) -> _Part:
    return _Part(0, start, end, 0, 1, 0)


def part_cyclic(index: int, P: int, N: int) -> _Part:
    return _Part(1, 0, 0, index, P, N)


# ---- shards ----------------------------------------------------------------------------------------
class OracleVector:
    """PartialVector[V] (PartialVector.scala:16-64) with a numpy `data` array."""

    def __init__(self, part: _Part, code: int):
        self.part, self.code = part, code
        self.size = lib().oracle_partition_size(C.byref(part))
        self.data = np.zeros(max(self.size, 0), NP[code])

    def update(self, keys, vals) -> int:
        k = np.ascontiguousarray(keys, np.int64)
        v = np.ascontiguousarray(vals, NP[self.code])
        return lib().oracle_vec_update(C.byref(self.part), self.code, self.data.ctypes.data, self.size,
                                       k.ctypes.data, v.ctypes.data, k.size)

    def get(self, keys):
        k = np.ascontiguousarray(keys, np.int64)
        out = np.zeros(k.size, NP[self.code])
        bad = lib().oracle_vec_get(C.byref(self.part), self.code, self.data.ctypes.data, self.size,
                                   k.ctypes.data, out.ctypes.data, k.size)
        return out, bad


class OracleMatrix:
    """PartialMatrix[V] (PartialMatrix.scala:17-87), row-major (rows x cols)."""

    def __init__(self, part: _Part, cols: int, code: int):
        self.part, self.code, self.cols = part, code, cols
        self.rows = lib().oracle_partition_size(C.byref(part))
        self.data = np.zeros((max(self.rows, 0), cols), NP[code])

    def update(self, rows, cols, vals) -> int:
        r = np.ascontiguousarray(rows, np.int64)
        c = np.ascontiguousarray(cols, np.int32)
        v = np.ascontiguousarray(vals, NP[self.code])
        return lib().oracle_mat_update(C.byref(self.part), self.code, self.data.ctypes.data, self.rows, self.cols,
                                       r.ctypes.data, c.ctypes.data, v.ctypes.data, r.size)

    def get(self, rows, cols):
        r = np.ascontiguousarray(rows, np.int64)
        c = np.ascontiguousarray(cols, np.int32)
        out = np.zeros(r.size, NP[self.code])
        bad = lib().oracle_mat_get(C.byref(self.part), self.code, self.data.ctypes.data, self.rows, self.cols,
                                   r.ctypes.data, c.ctypes.data, out.ctypes.data, r.size)
        return out, bad

    def get_rows(self, rows):
        r = np.ascontiguousarray(rows, np.int64)
        out = np.zeros((r.size, self.cols), NP[self.code])
        bad = lib().oracle_mat_get_rows(C.byref(self.part), self.code, self.data.ctypes.data, self.rows, self.cols,
                                        r.ctypes.data, out.ctypes.data, r.size)
        return out, bad


def vec_update_f64_parallel(starts, ends, datas, keys, vals, nthreads: int) -> int:
    """One scalar update loop per shard on `nthreads` threads (cpu_baseline)."""
    S = len(datas)
    ptr = lambda arrs: (C.c_void_p * S)(*[a.ctypes.data for a in arrs])  # noqa: E731
    ns = np.array([k.size for k in keys], np.int64)
    st = np.ascontiguousarray(starts, np.int64)
    en = np.ascontiguousarray(ends, np.int64)
    return lib().oracle_vec_update_f64_parallel(S, st.ctypes.data, en.ctypes.data, ptr(datas), ptr(keys),
                                                ptr(vals), ns.ctypes.data, nthreads)


# ---- java.util.Random -------------------------------------------------------------------------------
class JavaRandom:
    """java.util.Random's 48-bit LCG (scala.util.Random delegates to it)."""

    MULT, ADD, MASK = 0x5DEECE66D, 0xB, (1 << 48) - 1

    def __init__(self, seed: int):
        self.seed = (seed ^ self.MULT) & self.MASK

    def next(self, bits: int) -> int:
        self.seed = (self.seed * self.MULT + self.ADD) & self.MASK
        r = self.seed >> (48 - bits)
        return r - (1 << bits) if r >= (1 << (bits - 1)) and bits == 32 else r

    def nextDouble(self) -> float:
        return ((self.next(26) << 27) + self.next(27)) * (1.0 / (1 << 53))

    def nextDoubles(self, n: int) -> np.ndarray:
        """n consecutive nextDouble() values (a tight loop over the 48-bit state)."""
        out = np.empty(n, np.float64)
        s, M, A, MASK = self.seed, self.MULT, self.ADD, self.MASK
        scale = 1.0 / (1 << 53)
        for i in range(n):
            s = (s * M + A) & MASK
            hi = s >> 22
            s = (s * M + A) & MASK
            out[i] = ((hi << 27) + (s >> 21)) * scale
        self.seed = s
        return out


# ---- wire codec --------------------------------------------------------------------------------------
PULL_MATRIX, PULL_MATRIX_ROWS, PULL_VECTOR = 0x00, 0x01, 0x02
PUSH_MATRIX = {O_F64: 0x03, O_F32: 0x04, O_I32: 0x05, O_I64: 0x06}
PUSH_VECTOR = {O_F64: 0x07, O_F32: 0x08, O_I32: 0x09, O_I64: 0x0A}
RESPONSE = {O_F64: 0x10, O_F32: 0x11, O_I32: 0x12, O_I64: 0x13}
_PUSH_MATRIX_INV = {v: k for k, v in PUSH_MATRIX.items()}
_PUSH_VECTOR_INV = {v: k for k, v in PUSH_VECTOR.items()}
_RESPONSE_INV = {v: k for k, v in RESPONSE.items()}
_LE = "<"  # the JVM writes native order through Unsafe; x86/MI355X hosts are little-endian


def _arr(a, dt) -> bytes:
    return np.ascontiguousarray(a, dtype=np.dtype(dt).newbyteorder(_LE)).tobytes()


def encode_pull_matrix(rows, cols) -> bytes:  # RequestSerializer.scala:134-141
    return struct.pack("<Bi", PULL_MATRIX, len(rows)) + _arr(rows, np.int64) + _arr(cols, np.int32)


def encode_pull_matrix_rows(rows) -> bytes:  # :143-148
    return struct.pack("<Bi", PULL_MATRIX_ROWS, len(rows)) + _arr(rows, np.int64)


def encode_pull_vector(keys) -> bytes:  # :150-155
    return struct.pack("<Bi", PULL_VECTOR, len(keys)) + _arr(keys, np.int64)


def encode_push_matrix(code: int, mid: int, rows, cols, vals) -> bytes:  # :157-203
    return (struct.pack("<Bii", PUSH_MATRIX[code], len(rows), mid) + _arr(rows, np.int64) + _arr(cols, np.int32)
            + _arr(vals, NP[code]))


def encode_push_vector(code: int, mid: int, keys, vals) -> bytes:  # :205-243
    return struct.pack("<Bii", PUSH_VECTOR[code], len(keys), mid) + _arr(keys, np.int64) + _arr(vals, NP[code])


def encode_response(code: int, vals) -> bytes:  # ResponseSerializer.scala:291-350
    return struct.pack("<Bi", RESPONSE[code], len(vals)) + _arr(vals, NP[code])


def encode_response_rows(code: int, rows) -> bytes:  # ResponseSerializer.scala:298-307 (flattened)
    rows = np.asarray(rows, NP[code])
    return struct.pack("<Bi", RESPONSE[code], rows.size) + _arr(rows.reshape(-1), NP[code])


def decode_request(b: bytes) -> dict:
    """RequestSerializer.fromBinary (RequestSerializer.scala:59-130)."""
    t, n = struct.unpack_from("<Bi", b, 0)
    pos = 5

    def take(dt, count):
        nonlocal pos
        dt = np.dtype(dt).newbyteorder(_LE)
        a = np.frombuffer(b, dtype=dt, count=count, offset=pos).astype(dt.newbyteorder("="))
        pos += count * dt.itemsize
        return a

    if t == PULL_MATRIX:
        return {"type": "PullMatrix", "rows": take(np.int64, n), "cols": take(np.int32, n)}
    if t == PULL_MATRIX_ROWS:
        return {"type": "PullMatrixRows", "rows": take(np.int64, n)}
    if t == PULL_VECTOR:
        return {"type": "PullVector", "keys": take(np.int64, n)}
    (mid,) = struct.unpack_from("<i", b, pos)
    pos += 4
    if t in _PUSH_MATRIX_INV:
        code = _PUSH_MATRIX_INV[t]
        return {"type": "PushMatrix", "code": code, "id": mid, "rows": take(np.int64, n),
                "cols": take(np.int32, n), "values": take(NP[code], n)}
    if t in _PUSH_VECTOR_INV:
        code = _PUSH_VECTOR_INV[t]
        return {"type": "PushVector", "code": code, "id": mid, "keys": take(np.int64, n),
                "values": take(NP[code], n)}
    raise ValueError(f"unknown request type byte {t:#x}")


def decode_response(b: bytes) -> dict:
    """ResponseSerializer.fromBinary (ResponseSerializer.scala:19-41)."""
    t, n = struct.unpack_from("<Bi", b, 0)
    code = _RESPONSE_INV[t]
    dt = np.dtype(NP[code]).newbyteorder(_LE)
    return {"code": code, "values": np.frombuffer(b, dtype=dt, count=n, offset=5).astype(NP[code])}
