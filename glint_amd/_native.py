"""ctypes binding of the C ABI in include/glint_gpu.h (libglint_gpu.so).

The binding is the Python analogue of the JNI shim described in INTEGRATION.md: plain pointers,
sizes and status codes. There is no fallback: if the library is missing or cannot be loaded,
importing ``glint_amd`` fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

LIB_PATH = Path(__file__).resolve().parent / "lib" / "libglint_gpu.so"

GLINT_I32, GLINT_I64, GLINT_F32, GLINT_F64 = 0, 1, 2, 3
GLINT_OK, GLINT_EOUTOFRANGE, GLINT_EDEVICE, GLINT_EINVAL, GLINT_ENOMEM = 0, 1, 2, 3, 4
GLINT_PUSH_DEFAULT, GLINT_PUSH_DETERMINISTIC, GLINT_PUSH_UNORDERED, GLINT_PUSH_VALIDATE = 0, 1, 2, 4
GLINT_K_PUSH_APPLY, GLINT_K_PUSH_SCATTER, GLINT_K_VEC_PULL, GLINT_K_MAT_PULL, GLINT_K_MAT_PULL_ROWS = 0, 1, 2, 3, 4
GLINT_K_PUSH_CHECK = 5
GLINT_K_PUSH_BINNED = 6
GLINT_K_PUSH_ORDERED = 7
GLINT_ROUTE_RANGE, GLINT_ROUTE_CYCLIC = 0, 1
GLINT_RING_SLOTS, GLINT_ZERO_COPY_MAX = 16, 4096

# every symbol include/glint_gpu.h declares, with its C signature
_P = C.c_void_p
_I = C.c_int
_I32 = C.c_int32
_I64 = C.c_int64
_SZ = C.c_size_t
SIGNATURES = {
    "glint_shard_create": (_I, [_I, _I, _I64, _I64, _I32, C.POINTER(_P)]),
    "glint_shard_create_cyclic": (_I, [_I, _I, _I32, _I32, _I64, _I32, C.POINTER(_P)]),
    "glint_shard_create_in": (_I, [_P, _I64, _I64, _I64, C.POINTER(_P)]),
    "glint_vec_push_dev_shards": (_I, [_P, _I, _P, _P, _I64, _P, _P]),
    "glint_shard_destroy": (_I, [_P]),
    "glint_shard_zero": (_I, [_P]),
    "glint_shard_info": (_I, [_P, C.POINTER(_I32), C.POINTER(_I32), C.POINTER(_I), C.POINTER(_I)]),
    "glint_vec_push": (_I, [_P, _P, _P, _I64, _I]),
    "glint_vec_pull": (_I, [_P, _P, _P, _I64]),
    "glint_mat_push": (_I, [_P, _P, _P, _P, _I64, _I]),
    "glint_mat_pull": (_I, [_P, _P, _P, _P, _I64]),
    "glint_mat_pull_rows": (_I, [_P, _P, _P, _I64]),
    "glint_shard_last_error": (_I, [_P, C.POINTER(_I64)]),
    "glint_vec_push_dev": (_I, [_P, _P, _P, _I64, _I, _P]),
    "glint_vec_push_dev_gated": (_I, [_P, _P, _P, _I64, _I, _P, _P]),
    "glint_mat_push_dev_gated": (_I, [_P, _P, _P, _P, _I64, _I, _P, _P]),
    "glint_vec_pull_dev": (_I, [_P, _P, _P, _I64, _P]),
    "glint_mat_push_dev": (_I, [_P, _P, _P, _P, _I64, _I, _P]),
    "glint_mat_pull_dev": (_I, [_P, _P, _P, _P, _I64, _P]),
    "glint_mat_pull_rows_dev": (_I, [_P, _P, _P, _I64, _P]),
    "glint_shard_sync": (_I, [_P, _P, C.POINTER(_I64)]),
    "glint_shards_sync": (_I, [_P, _P, _I, C.POINTER(_I), C.POINTER(_I64)]),
    "glint_shard_data": (_I, [_P, C.POINTER(_P)]),
    "glint_shard_pitch": (_I, [_P, C.POINTER(_I64)]),
    "glint_push_wire": (_I, [_P, _P, _SZ, C.POINTER(_I32), _I]),
    "glint_stage_acquire": (_I, [_P, _I64, C.POINTER(_P), C.POINTER(_P), C.POINTER(_P), C.POINTER(_I)]),
    "glint_push_staged": (_I, [_P, _I, _I64, _I, C.POINTER(C.c_uint64)]),
    "glint_push_wire_async": (_I, [_P, _P, _SZ, C.POINTER(_I32), _I, C.POINTER(C.c_uint64)]),
    "glint_shard_wait": (_I, [_P, C.c_uint64, C.POINTER(_I64)]),
    "glint_pull_async": (_I, [_P, _I, _P, _P, _P, _I64, C.POINTER(C.c_uint64)]),
    "glint_pull_wire_async": (_I, [_P, _P, _SZ, _P, _SZ, C.POINTER(_SZ), C.POINTER(C.c_uint64)]),
    "glint_pull_wire": (_I, [_P, _P, _SZ, _P, _SZ, C.POINTER(_SZ)]),
    "glint_route_dev": (_I, [_P, _I64, _I, _I32, _I64, _P, _P, C.POINTER(_I64), _P]),
    "glint_route_gather_dev": (_I, [_P, _P, _P, _I, _I64, _I, _I32, _I64, _P, _P, _P, _P, _P, _P, _P, _P]),
    "glint_route_gather_rebased_dev": (_I, [_P, _P, _P, _I, _I64, _I, _I32, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "glint_scatter_rows_dev": (_I, [_P, _P, _I64, _I64, _P, _P]),
    "glint_copy_segments_dev": (_I, [_P, _P, C.POINTER(_I64), _I, _P]),
    "glint_send_matrix_dev": (_I, [_P, _P, _I32, _I32, _P, _P, _P]),
    "glint_prof_enable": (_I, [_P, _I]),
    "glint_prof_read": (_I, [_P, _I, C.POINTER(C.c_double), C.POINTER(_I64)]),
    "glint_prof_reset": (_I, [_P]),
    "glint_strerror": (C.c_char_p, [_I]),
    "glint_device_count": (_I, []),
    "glint_version": (_I, []),
    "glint_reload_env": (_I, []),
    "glint_push_flags_supported": (_I, []),
    "glint_host_alloc": (_I, [C.c_size_t, _P]),
    "glint_host_free": (_I, [_P]),
}

_lib = None


def load() -> C.CDLL:
    """Load libglint_gpu.so (in-tree). Raises if it is missing -- no CPU fallback exists."""
    global _lib
    if _lib is not None:
        return _lib
    path = Path(os.environ.get("GLINT_GPU_LIB", str(LIB_PATH)))
    if not path.exists():
        raise ImportError(
            f"glint_amd native library not found at {path}: run `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950). There is no CPU fallback for the push/pull plane.")
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64.so.7. If torch is present,
    # load it first so this library binds to that same runtime (same soname) -- device pointers and
    # hipStream_t handles from torch are then valid here. Without torch, /opt/rocm's runtime is used.
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    lib = C.CDLL(str(path))
    ab = "GLINT_GPU_LIB" in os.environ  # an older library loaded for a same-box A/B may lack newer symbols
    for name, (res, args) in SIGNATURES.items():
        if ab and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def reload_env() -> None:
    """Make the library re-read its GLINT_* environment knobs (it caches them)."""
    load().glint_reload_env()


def strerror(code: int) -> str:
    return load().glint_strerror(code).decode()
