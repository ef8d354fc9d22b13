"""Builds the in-tree native libraries.

* ``glint_amd/lib/libglint_gpu.so`` -- the product: HIP kernels + C ABI (include/glint_gpu.h),
  compiled for gfx950 only. hipcc cross-compiles it without a GPU.
* ``oracle/build/libglint_oracle.so`` -- the CPU restatement used by tests as the parity checker
  (never linked into the product).

Outputs stay in-tree so they travel to the GPU box with the repository snapshot.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "glint_amd"
LIB_DIR = PKG / "lib"
LIB = LIB_DIR / "libglint_gpu.so"
ORACLE_DIR = ROOT / "oracle"
ORACLE_LIB = ORACLE_DIR / "build" / "libglint_oracle.so"

CSRC = PKG / "csrc"
HIP_SOURCES = [CSRC / "glint_gpu.hip", CSRC / "glint_sort.hip", CSRC / "glint_route.hip", CSRC / "glint_ordered.hip", CSRC / "glint_bin.hip",
               CSRC / "glint_exchange.hip"]
HIP_HEADERS = [CSRC / "glint_kernels.h", CSRC / "glint_device.h", CSRC / "glint_host.h", ROOT / "include" / "glint_gpu.h"]
HIP_DEPS = HIP_SOURCES + HIP_HEADERS
OBJ_DIR = ROOT / "build" / "obj"
ORACLE_SOURCES = [ORACLE_DIR / "glint_oracle.c"]
LOOPBACK_SRC = ROOT / "tools" / "loopback" / "glint_loopback.c"
LOOPBACK_BIN = ROOT / "tools" / "loopback" / "build" / "glint_loopback"


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found: the glint_amd native library cannot be built")


def _stale(out: Path, deps) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def build_gpu_lib(force: bool = False, verbose: bool = False) -> Path:
    """Compile libglint_gpu.so for gfx950 (no other target): one object per source, rebuilt when
    it or a header changed (sources compile in parallel), then one link. No library beyond the HIP
    runtime is linked: every sort, scan and partition is hand-written."""
    if not force and not _stale(LIB, HIP_DEPS):
        return LIB
    OBJ_DIR.mkdir(parents=True, exist_ok=True)
    LIB_DIR.mkdir(parents=True, exist_ok=True)
    flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-result"]
    objs, procs = [], []
    for src in HIP_SOURCES:
        obj = OBJ_DIR / (src.stem + ".o")
        objs.append(obj)
        if force or _stale(obj, [src] + HIP_HEADERS):
            cmd = [_hipcc(), *flags, "-c", "-o", str(obj) + ".tmp", str(src)]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            procs.append((subprocess.Popen(cmd, cwd=str(ROOT)), obj))
    for p, obj in procs:  # sources compile in parallel
        if p.wait() != 0:
            raise subprocess.CalledProcessError(p.returncode, f"hipcc -c {obj.name}")
        os.replace(str(obj) + ".tmp", obj)
    tmp = LIB.with_suffix(".so.tmp")
    cmd = [_hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs)]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=str(ROOT))
    os.replace(tmp, LIB)
    return LIB


def build_oracle(force: bool = False, verbose: bool = False) -> Path:
    """Compile the CPU restatement (test infrastructure) with gcc."""
    if not force and not _stale(ORACLE_LIB, ORACLE_SOURCES):
        return ORACLE_LIB
    ORACLE_LIB.parent.mkdir(parents=True, exist_ok=True)
    tmp = ORACLE_LIB.with_suffix(".so.tmp")
    cc = shutil.which("gcc") or "cc"
    cmd = [cc, "-O2", "-std=c11", "-fPIC", "-shared", "-fwrapv", "-pthread", "-o", str(tmp),
           *map(str, ORACLE_SOURCES)]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=str(ROOT))
    os.replace(tmp, ORACLE_LIB)
    return ORACLE_LIB


def build_loopback(force: bool = False, verbose: bool = False) -> Path:
    """The loopback-TCP client/server harness (BASELINE.json configs[0]); it dlopens its shard
    backend at run time and links neither library."""
    if not force and not _stale(LOOPBACK_BIN, [LOOPBACK_SRC]):
        return LOOPBACK_BIN
    LOOPBACK_BIN.parent.mkdir(parents=True, exist_ok=True)
    tmp = LOOPBACK_BIN.with_suffix(".tmp")
    cc = shutil.which("gcc") or "cc"
    cmd = [cc, "-O2", "-std=c11", "-Wall", "-pthread", "-o", str(tmp), str(LOOPBACK_SRC), "-ldl", "-lm"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=str(ROOT))
    os.replace(tmp, LOOPBACK_BIN)
    return LOOPBACK_BIN


JNI_SHIM = ROOT / "integration" / "jni" / "glint_jni.c"
JNI_DRIVER_SRC = ROOT / "tests" / "c" / "fake_jvm.c"
JNI_DRIVER = ROOT / "tests" / "c" / "build" / "fake_jvm"


def build_jni_driver(force: bool = False, verbose: bool = False) -> Path:
    """The JNI shim (integration/jni/glint_jni.c) compiled against tests/c/jni.h -- a minimal JNI
    environment -- and linked with a driver that calls its native methods as the actors do. This is
    the shim's compile check (there is no JDK in the image) and, on a GPU, its end-to-end test."""
    deps = [JNI_SHIM, JNI_DRIVER_SRC, ROOT / "tests" / "c" / "jni.h", ROOT / "include" / "glint_gpu.h", LIB]
    if not force and not _stale(JNI_DRIVER, deps):
        return JNI_DRIVER
    JNI_DRIVER.parent.mkdir(parents=True, exist_ok=True)
    tmp = JNI_DRIVER.with_suffix(".tmp")
    cc = shutil.which("gcc") or "cc"
    cmd = [cc, "-O2", "-Wall", "-Werror", "-std=c11", "-I", str(ROOT / "tests" / "c"), "-I", str(ROOT / "include"),
           str(JNI_DRIVER_SRC), str(JNI_SHIM), "-L", str(LIB_DIR), "-lglint_gpu", f"-Wl,-rpath,{LIB_DIR}",
           "-o", str(tmp)]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=str(ROOT))
    os.replace(tmp, JNI_DRIVER)
    return JNI_DRIVER


def build_all(force: bool = False, verbose: bool = False) -> None:
    build_gpu_lib(force=force, verbose=verbose)
    build_oracle(force=force, verbose=verbose)
    build_loopback(force=force, verbose=verbose)
    build_jni_driver(force=force, verbose=verbose)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv, verbose=True)
    print(LIB)
    print(ORACLE_LIB)
    print(LOOPBACK_BIN)
