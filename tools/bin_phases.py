"""Phase breakdown of the binned push kernels (clock64 sums per phase, thread 0 of each workgroup),
from a tuning build of the library (glint_bin.hip with -DGLINT_BIN_PROF).

    python tools/bin_phases.py --build        # here: compile tools/build/libglint_gpu_prof.so
    python tools/bin_phases.py                # on the GPU box: cfg3 Zipf, cfg4b uniform, cfg5 matrix
"""
import ctypes as C
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
TAG = sys.argv[sys.argv.index("--tag") + 1] if "--tag" in sys.argv else ""
PROF_LIB = ROOT / "tools" / "ablibs" / f"libglint_gpu_prof{'_' + TAG if TAG else ''}.so"  # (travels to the box)
DEFINES = [a for a in sys.argv[1:] if a.startswith("-D")]

PHASES = {
    "bin_part (plain)": (0, ["setup", "addr", "issue loads", "rank+sync", "scan", "stage+sync", "store+sync",
                             "clear+sync"]),
    "bin_part (dedup)": (8, ["setup", "hash insert", "issue loads", "sync+extract+sync", "rank+sync", "scan",
                             "stage+sync", "store+sync", "clear+sync", "hv clear+sync"]),
    "bin_fsort (v2)": (32, ["window+clear", "marks+fill", "loads+sync", "rank+sync", "scan", "stage e+store",
                            "values"]),
    "bin_plan (v2)": (48, ["stage+walk", "groups+scan", "atomic+sync", "emit+sync"]),
    "bin_apply2 (v2)": (56, ["records", "publish+sync", "prefetch issue", "write-back", "sync"]),
}


def build():
    sys.path.insert(0, str(ROOT))
    import importlib.util
    spec = importlib.util.spec_from_file_location("_b", ROOT / "glint_amd" / "build.py")
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    b.build_gpu_lib()
    out = ROOT / "build" / "obj" / f"glint_bin_prof{'_' + TAG if TAG else ''}.o"
    flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-DGLINT_BIN_PROF", *DEFINES]
    subprocess.run([b._hipcc(), *flags, "-c", "-o", str(out), str(ROOT / "glint_amd/csrc/glint_bin.hip")], check=True)
    objs = [str(ROOT / "build" / "obj" / (s.stem + ".o")) for s in b.HIP_SOURCES if s.stem != "glint_bin"] + [str(out)]
    PROF_LIB.parent.mkdir(parents=True, exist_ok=True)
    subprocess.run([b._hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", str(PROF_LIB), *objs], check=True)
    print(PROF_LIB)


def run():
    os.environ["GLINT_GPU_LIB"] = str(PROF_LIB)
    os.environ.setdefault("GLINT_BINNED", "1")  # every push binned (no adaptive fallback to the scatter)
    sys.path.insert(0, str(ROOT))
    import numpy as np
    import torch
    from glint_amd import _native as N
    lib = N.load()
    lib.glint_debug_bin_prof.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    buf = (C.c_ulonglong * 64)()
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev).cuda_stream

    def case(name, n_elems, keys, vals, cols=None, ncols=0):
        h = C.c_void_p()
        if ncols:
            assert lib.glint_shard_create(0, N.GLINT_F64, 0, n_elems, ncols, C.byref(h)) == 0
        else:
            assert lib.glint_shard_create(0, N.GLINT_F64, 0, n_elems, 0, C.byref(h)) == 0

        def push():
            if ncols:
                rc = lib.glint_mat_push_dev(h, keys.data_ptr(), cols.data_ptr(), vals.data_ptr(), keys.numel(), 0, st)
            else:
                rc = lib.glint_vec_push_dev(h, keys.data_ptr(), vals.data_ptr(), keys.numel(), 0, st)
            assert rc == 0, rc
        for _ in range(3):  # each ended by the shard's sync point, as the bench's warm-up (the front end
            push()          # decides from the hints latched there)
            assert lib.glint_shard_sync(h, st, None) == 0
        torch.cuda.synchronize()
        lib.glint_debug_bin_prof(buf, 1)
        reps = 5
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            push()
        e1.record()
        torch.cuda.synchronize()
        lib.glint_debug_bin_prof(buf, 1)
        lib.glint_shard_destroy(h)
        print(f"== {name} [{TAG or 'base'}]: {e0.elapsed_time(e1) / reps:.3f} ms per push")
        for kname, (base, labels) in PHASES.items():
            v = [buf[base + i] for i in range(len(labels))]
            tot = sum(v)
            if tot == 0:
                continue
            print(f"  {kname}: {tot / reps / 1e6:.1f} M clocks per push (summed over workgroups)")
            for lab, x in zip(labels, v):
                print(f"     {lab:22s} {100.0 * x / tot:5.1f}%")

    n = 1 << 28
    rng = np.random.default_rng(42)
    nrec = n // 4
    r = rng.zipf(1.1, size=int(nrec * 1.3))
    r = r[r <= n][:nrec] - 1
    k = rng.permutation(n)[r].astype(np.int64)
    keys = torch.from_numpy(k).to(dev)
    vals = torch.rand(keys.numel(), dtype=torch.float64, device=dev)
    case("cfg3 zipf", n, keys, vals)
    keys = torch.randint(0, n, (nrec,), dtype=torch.int64, device=dev)
    case("cfg4b uniform (N=1)", n, keys, vals[:nrec])
    del keys, vals
    rows, ncols = 1 << 17, 512
    nm = 1 << 23
    rk = np.minimum(np.floor(np.power(float(rows), rng.random(nm))).astype(np.int64) - 1, rows - 1)
    keys = torch.from_numpy(rng.permutation(rows)[rk].astype(np.int64)).to(dev)
    cols = torch.from_numpy(rng.integers(0, ncols, nm).astype(np.int32)).to(dev)
    vals = torch.rand(nm, dtype=torch.float64, device=dev)
    case("cfg5 matrix", rows, keys, vals, cols, ncols)


if __name__ == "__main__":
    build() if "--build" in sys.argv else run()
