"""Pipelined message-sized wire pushes only (tuning probe for rocprofv3 --kernel-trace): M messages
of n records enqueued back to back with glint_push_wire_async, one wait at the end.

    python tools/ring_probe.py [n] [M]
"""
import ctypes as C
import struct
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402
from glint_amd import _native as N  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
M = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
SIZE = 1 << 24
lib = N.load()
h = C.c_void_p()
assert lib.glint_shard_create(0, N.GLINT_F64, 0, SIZE, 0, C.byref(h)) == 0
rng = np.random.default_rng(42)
msgs = []
for i in range(64):
    keys = rng.integers(0, SIZE, n, dtype=np.int64)
    wire = bytes([0x07]) + struct.pack("<ii", n, i) + keys.tobytes() + rng.random(n).tobytes()
    msgs.append((C.c_uint8 * len(wire)).from_buffer_copy(wire))
mid, ticket = C.c_int32(), C.c_uint64()
for rep in range(2):
    t0 = time.perf_counter()
    for i in range(M):
        w = msgs[i % 64]
        assert lib.glint_push_wire_async(h, w, len(w), C.byref(mid), 0, C.byref(ticket)) == 0
    t1 = time.perf_counter()
    assert lib.glint_shard_wait(h, ticket.value, None) == 0
    t2 = time.perf_counter()
    print(f"n={n} M={M}: enqueue {1e6 * (t1 - t0) / M:.2f} us/msg, total {1e6 * (t2 - t0) / M:.2f} us/msg", flush=True)
lib.glint_shard_destroy(h)
