"""Tuning sweep for the push kernels (run on the GPU box): times glint_vec_push_dev on a 2^lg push
for blocks-per-CU values of one kernel (knob GLINT_CHECK_BPC or GLINT_APPLY_BPC), in one process.
Usage: sweep_push.py [lg] [dense|sorted_sparse] [knob]"""
import ctypes as C
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402
import glint_amd  # noqa: E402
from glint_amd import _native as N  # noqa: E402

lg = int(sys.argv[1]) if len(sys.argv) > 1 else 28
pattern = sys.argv[2] if len(sys.argv) > 2 else "dense"
n = 1 << lg
dev = torch.device("cuda", 0)
lib = N.load()
sh = glint_amd.PartialVector(glint_amd.RangePartition(0, 0, n), "double", 0)
keys = torch.arange(n, dtype=torch.int64, device=dev)
if pattern == "sorted_sparse":
    keys = torch.arange(0, n, 2, dtype=torch.int64, device=dev)
vals = torch.rand(keys.numel(), dtype=torch.float64, device=dev)
stream = torch.cuda.current_stream(dev).cuda_stream


def kms(kid):
    ms, cnt = C.c_double(), C.c_int64()
    lib.glint_prof_read(sh.handle, kid, C.byref(ms), C.byref(cnt))
    return ms.value / max(cnt.value, 1)


knob = sys.argv[3] if len(sys.argv) > 3 else "GLINT_APPLY_BPC"
for bpc in (1, 2, 3, 4, 6, 8):
    os.environ[knob] = str(bpc)
    for _ in range(2):
        lib.glint_vec_push_dev(sh.handle, keys.data_ptr(), vals.data_ptr(), keys.numel(), 0, stream)
    torch.cuda.synchronize()
    lib.glint_prof_reset(sh.handle)
    lib.glint_prof_enable(sh.handle, 1)
    t0 = time.perf_counter()
    for _ in range(10):
        lib.glint_vec_push_dev(sh.handle, keys.data_ptr(), vals.data_ptr(), keys.numel(), 0, stream)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 10
    lib.glint_prof_enable(sh.handle, 0)
    gbs = 32.0 * keys.numel() / dt / 1e9
    print(f"{pattern} {knob}={bpc}: step {dt*1e3:.3f} ms  {gbs:7.0f} GB/s   check {kms(N.GLINT_K_PUSH_CHECK):.3f} "
          f"apply {kms(N.GLINT_K_PUSH_APPLY):.3f} scatter {kms(N.GLINT_K_PUSH_SCATTER):.3f} ms", flush=True)
sh.sync(stream)
