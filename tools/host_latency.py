"""Per-call latency of the host-pointer entry points (what the JNI shim calls once per Akka message):
glint_vec_push / glint_vec_pull / glint_push_wire with pageable numpy arrays, by message size, and
the pipelined glint_push_wire_async (messages enqueued back to back, one wait at the end). The
small sizes are the reference's own message shapes: 1000 records per push in
GranularBigVectorSpec.scala:21, and the 79 999-record frame cap of the granular client.
One JSON line per (op, n) on stdout.

    python tools/host_latency.py [--reps R]
"""
import ctypes as C
import json
import os
import struct
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402
from glint_amd import _native as N  # noqa: E402

REPS = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 200
lib = N.load()
SIZE = 1 << 24


def ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def per_call(fn, reps):
    for _ in range(5):
        fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps


h = C.c_void_p()
assert lib.glint_shard_create(0, N.GLINT_F64, 0, SIZE, 0, C.byref(h)) == 0
rng = np.random.default_rng(42)
for n in (1, 1000, 10_000, 79_999, 1 << 18, 1 << 20, 1 << 24):
    keys = rng.integers(0, SIZE, n, dtype=np.int64)
    vals = rng.random(n)
    out = np.empty(n)
    reps = max(8, min(REPS, int(REPS * 1000 / max(n, 1000))))

    def push():
        rc = lib.glint_vec_push(h, ptr(keys), ptr(vals), n, 0)
        assert rc == 0, rc

    def pull():
        rc = lib.glint_vec_pull(h, ptr(keys), ptr(out), n)
        assert rc == 0, rc

    wire = bytes([0x07]) + struct.pack("<ii", n, 1) + keys.tobytes() + vals.tobytes()
    wbuf = (C.c_uint8 * len(wire)).from_buffer_copy(wire)
    mid = C.c_int32()

    def push_wire():
        rc = lib.glint_push_wire(h, wbuf, len(wire), C.byref(mid), 0)
        assert rc == 0, rc

    ticket = C.c_uint64()

    def push_wire_async():
        rc = lib.glint_push_wire_async(h, wbuf, len(wire), C.byref(mid), 0, C.byref(ticket))
        assert rc == 0, rc

    def pipelined(fn, reps):  # enqueue `reps` messages, one wait at the end: per-message throughput cost
        for _ in range(2 * N.GLINT_RING_SLOTS):  # every ring slot sized for this message first
            fn()
        lib.glint_shard_wait(h, ticket.value, None)
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        assert lib.glint_shard_wait(h, ticket.value, None) == 0
        return (time.perf_counter() - t0) / reps

    for op, fn, bpr in (("vec_push", push, 16), ("vec_pull", pull, 16), ("push_wire", push_wire, 16),
                        ("push_wire_async", push_wire_async, 16)):
        if op == "push_wire_async" and n > 1 << 20:
            continue  # the ring takes messages up to 2^20 records
        dt = pipelined(fn, reps) if op == "push_wire_async" else per_call(fn, reps)
        print(json.dumps({"op": op, "records": n, "pinned_stage_max": os.environ.get("GLINT_PINNED_STAGE_MAX", "default"), "us_per_call": round(dt * 1e6, 2),
                          "Mrecords_per_s": round(n / dt / 1e6, 2), "host_GBps": round(n * bpr / dt / 1e9, 2),
                          "reps": reps}), flush=True)
lib.glint_shard_destroy(h)
