"""Builds a variant of libglint_gpu.so for A/B runs on one box: glint_bin.hip (or another source)
recompiled with extra -D defines, linked with the other objects of the current build.

    python tools/variant.py NAME -DGLINT_BIN_NT=1 [--src glint_bin]   # -> tools/ablibs/libglint_gpu_NAME.so
    python tools/variant.py NAME -DGLINT_RING_SLOTS=64 --all          # every source (layout-changing defines)

Load it with GLINT_GPU_LIB=tools/ablibs/libglint_gpu_NAME.so (the `ab` stage of tools/gpu_run.sh).
"""
import importlib.util
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def main():
    name = sys.argv[1]
    defines = [a for a in sys.argv[2:] if a.startswith("-D")]
    src = sys.argv[sys.argv.index("--src") + 1] if "--src" in sys.argv else "glint_bin"
    spec = importlib.util.spec_from_file_location("_b", ROOT / "glint_amd" / "build.py")
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    b.build_gpu_lib()
    flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", *defines]
    srcs = [s.stem for s in b.HIP_SOURCES] if "--all" in sys.argv else [src]
    objs = [str(ROOT / "build" / "obj" / (s.stem + ".o")) for s in b.HIP_SOURCES if s.stem not in srcs]
    for sname in srcs:
        out = ROOT / "build" / "obj" / f"{sname}_{name}.o"
        subprocess.run([b._hipcc(), *flags, "-c", "-o", str(out), str(ROOT / "glint_amd" / "csrc" / f"{sname}.hip")],
                       check=True)
        objs.append(str(out))
    # (tools/ablibs travels to the GPU box with the tree; tools/build does not)
    lib = ROOT / "tools" / "ablibs" / f"libglint_gpu_{name}.so"
    lib.parent.mkdir(parents=True, exist_ok=True)
    subprocess.run([b._hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", str(lib), *objs], check=True)
    print(lib)


if __name__ == "__main__":
    main()
