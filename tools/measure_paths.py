"""Measures every push/pull path of the plane on one MI355X (besides bench.py's headline):
device-resident rates from HIP events around each kernel (glint_prof_*), and host-pointer
("end-to-end": pageable host memory -> H2D -> kernels -> D2H) rates by wall clock, which is what
the JNI shim sees. One JSON line per measurement on stdout.

    python tools/measure_paths.py [--quick]
"""
import ctypes as C
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import glint_amd  # noqa: E402
from glint_amd import _native as N  # noqa: E402

QUICK = "--quick" in sys.argv
dev = torch.device("cuda", 0)
lib = N.load()
stream = torch.cuda.current_stream(dev).cuda_stream


def kernel_ms(h, kid):
    ms, cnt = C.c_double(), C.c_int64()
    lib.glint_prof_read(h, kid, C.byref(ms), C.byref(cnt))
    return ms.value / max(cnt.value, 1)


def timed(fn, reps, h):
    fn()
    torch.cuda.synchronize()
    lib.glint_prof_reset(h)
    lib.glint_prof_enable(h, 1)
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    lib.glint_prof_enable(h, 0)
    return dt


def emit(**kw):
    print(json.dumps(kw), flush=True)


def zipf_keys(rng, n_keys, n, s):
    """Zipf(s) ranks over [0, n_keys) mapped through a seeded permutation (hot keys scattered).
    s > 1: numpy's sampler, truncated; s == 1: inverse-CDF of the 1/k law, k ~ n_keys^u."""
    if s > 1.0:
        ranks = rng.zipf(s, size=int(n * 1.4))
        ranks = ranks[ranks <= n_keys][:n] - 1
    else:
        ranks = np.minimum(np.floor(np.power(float(n_keys), rng.random(n))).astype(np.int64) - 1, n_keys - 1)
    perm = rng.permutation(n_keys)
    return perm[ranks].astype(np.int64)


def main():
    lg = 26 if QUICK else 28
    n = 1 << lg
    rng = np.random.default_rng(42)

    # ---- vector pull (device-resident), dense and random ------------------------------------------
    sh = glint_amd.PartialVector(glint_amd.RangePartition(0, 0, n), "double", 0)
    h = sh.handle
    keys = torch.arange(n, dtype=torch.int64, device=dev)
    vals = torch.rand(n, dtype=torch.float64, device=dev)
    out = torch.empty_like(vals)
    sh.update(keys, vals)
    dt = timed(lambda: lib.glint_vec_pull_dev(h, keys.data_ptr(), out.data_ptr(), n, stream), 10, h)
    k = kernel_ms(h, N.GLINT_K_VEC_PULL)
    emit(op="vec_pull_dev", pattern="dense", records=n, ms=dt * 1e3, kernel_ms=k,
         algorithmic_GBps=24.0 * n / (k * 1e-3) / 1e9, note="24 B/record: key 8 + shard 8 + out 8")
    rkeys = torch.randint(0, n, (n,), dtype=torch.int64, device=dev)
    dt = timed(lambda: lib.glint_vec_pull_dev(h, rkeys.data_ptr(), out.data_ptr(), n, stream), 5, h)
    k = kernel_ms(h, N.GLINT_K_VEC_PULL)
    emit(op="vec_pull_dev", pattern="uniform random", records=n, ms=dt * 1e3, kernel_ms=k,
         algorithmic_GBps=24.0 * n / (k * 1e-3) / 1e9, Grecords_per_s=n / (k * 1e-3) / 1e9)

    # ---- deterministic push of a dense run (same bytes as default mode) --------------------------
    dt = timed(lambda: lib.glint_vec_push_dev(h, keys.data_ptr(), vals.data_ptr(), n, 1, stream), 5, h)
    emit(op="vec_push_dev", mode="deterministic", pattern="dense", records=n, ms=dt * 1e3,
         algorithmic_GBps=32.0 * n / dt / 1e9)

    # ---- end-to-end host-pointer push / pull (pageable numpy, what the JNI shim passes) -----------
    m = 1 << (24 if QUICK else 26)
    hk = np.arange(m, dtype=np.int64)
    hv = np.random.default_rng(1).uniform(-1, 1, m)
    ho = np.empty(m, np.float64)
    lib.glint_vec_push(h, hk.ctypes.data, hv.ctypes.data, m, 0)
    t0 = time.perf_counter()
    for _ in range(5):
        lib.glint_vec_push(h, hk.ctypes.data, hv.ctypes.data, m, 0)
    dt = (time.perf_counter() - t0) / 5
    emit(op="vec_push_host", pattern="dense", records=m, ms=dt * 1e3, host_bytes_per_s=16.0 * m / dt / 1e9,
         algorithmic_GBps=32.0 * m / dt / 1e9, note="pageable H2D of keys+values + push kernels, synchronous")
    t0 = time.perf_counter()
    for _ in range(5):
        lib.glint_vec_pull(h, hk.ctypes.data, ho.ctypes.data, m)
    dt = (time.perf_counter() - t0) / 5
    emit(op="vec_pull_host", pattern="dense", records=m, ms=dt * 1e3, host_bytes_per_s=16.0 * m / dt / 1e9,
         note="pageable H2D of keys + gather + D2H of values, synchronous")
    sh.destroy()
    del keys, vals, out, rkeys

    # ---- client routing: stable grouping of a 2^26-record batch by owning partition ----------------
    m = 1 << 26
    rkeys = torch.randint(0, 1 << 30, (m,), dtype=torch.int64, device=dev)
    counts = torch.empty(4096, dtype=torch.int64, device=dev)
    order = torch.empty(m, dtype=torch.int64, device=dev)
    bad = C.c_int64()
    for nparts in (8, 64, 4096):
        fn = lambda: lib.glint_route_dev(rkeys.data_ptr(), m, N.GLINT_ROUTE_RANGE, nparts, 1 << 30,  # noqa: E731
                                         counts.data_ptr(), order.data_ptr(), C.byref(bad), stream)
        fn()
        t0 = time.perf_counter()
        for _ in range(5):
            assert fn() == 0
        dt = (time.perf_counter() - t0) / 5
        emit(op="route_dev", nparts=nparts, records=m, ms=dt * 1e3, Grecords_per_s=m / dt / 1e9,
             algorithmic_GBps=(8.0 * 2 + 8.0) * m / dt / 1e9,
             note="keys read twice (histogram, scatter) + 8 B index written; includes the D2H status sync")
    del rkeys, order

    # ---- cfg3: Zipf(1.1) sparse push with duplicates into a 2^28 shard -----------------------------
    sh = glint_amd.PartialVector(glint_amd.RangePartition(0, 0, n), "double", 0)
    h = sh.handle
    nz = n // 4
    zk = zipf_keys(rng, n, nz, 1.1)
    U = int(np.unique(zk).size)
    zkeys = torch.from_numpy(zk).to(dev)
    zvals = torch.rand(zk.size, dtype=torch.float64, device=dev)
    uk = torch.randint(0, n, (nz,), dtype=torch.int64, device=dev)
    for pat, kt, Uk in (("zipf1.1", zkeys, U), ("uniform random", uk, None)):
        for mode, flags, env in (("atomic", 0, "0"), ("binned (UNORDERED hint)", N.GLINT_PUSH_UNORDERED, ""),
                                 ("adaptive (no hint)", 0, "")):
            os.environ["GLINT_BINNED"] = env
            glint_amd._native.reload_env()  # the library caches its knobs
            dt = timed(lambda: lib.glint_vec_push_dev(h, kt.data_ptr(), zvals.data_ptr(), nz, flags, stream), 5, h)
            rec = dict(op="vec_push_dev", pattern=pat, path=mode, records=nz, ms=dt * 1e3,
                       Grecords_per_s=nz / dt / 1e9,
                       scatter_kernel_ms=kernel_ms(h, N.GLINT_K_PUSH_SCATTER),
                       binned_pipeline_ms=kernel_ms(h, N.GLINT_K_PUSH_BINNED))
            if Uk is not None:
                rec.update(distinct=Uk, dup_ratio=1 - Uk / nz, algorithmic_GBps=(16.0 * nz + 16.0 * Uk) / dt / 1e9)
            else:
                rec.update(algorithmic_GBps=32.0 * nz / dt / 1e9)
            emit(**rec)
        os.environ["GLINT_BINNED"] = ""
        glint_amd._native.reload_env()  # the library caches its knobs
    dt = timed(lambda: lib.glint_vec_push_dev(h, zkeys.data_ptr(), zvals.data_ptr(), zk.size, 1, stream), 2, h)
    emit(op="vec_push_dev", mode="deterministic", pattern="zipf1.1", records=int(zk.size), ms=dt * 1e3,
         algorithmic_GBps=(16.0 * zk.size + 16.0 * U) / dt / 1e9)
    sh.destroy()
    del zkeys, zvals, uk

    # ---- cfg5 (one of 8 shards): 2^17 x 512 Double matrix, Zipf(1.0) rows, row pull -----------------
    rows_total, cols = 1 << 20, 512
    shard_rows = rows_total // 8
    msh = glint_amd.PartialMatrix(glint_amd.RangePartition(0, 0, shard_rows), cols, "double", 0)
    h = msh.handle
    npush = (1 << 26) // 8
    r = zipf_keys(rng, shard_rows, npush, 1.0)
    c = rng.integers(0, cols, r.size).astype(np.int32)
    U = int(np.unique(r.astype(np.int64) * cols + c).size)
    mr = torch.from_numpy(r).to(dev)
    mc = torch.from_numpy(c).to(dev)
    mv = torch.rand(r.size, dtype=torch.float64, device=dev)
    dt = timed(lambda: lib.glint_mat_push_dev(h, mr.data_ptr(), mc.data_ptr(), mv.data_ptr(), r.size, 0, stream),
               5, h)
    emit(op="mat_push_dev", pattern="zipf1.0 rows x uniform cols", shape=[shard_rows, cols], records=int(r.size),
         distinct=U, ms=dt * 1e3, algorithmic_GBps=(20.0 * r.size + 16.0 * U) / dt / 1e9,
         Grecords_per_s=r.size / dt / 1e9)
    for mode, flags, env in (("atomic", 0, "0"), ("binned (UNORDERED hint)", N.GLINT_PUSH_UNORDERED, "")):
        os.environ["GLINT_BINNED"] = env
        glint_amd._native.reload_env()  # the library caches its knobs
        dt = timed(lambda: lib.glint_mat_push_dev(h, mr.data_ptr(), mc.data_ptr(), mv.data_ptr(), r.size, flags,
                                                  stream), 5, h)
        emit(op="mat_push_dev", pattern="zipf1.0 rows x uniform cols", path=mode, records=int(r.size), distinct=U,
             ms=dt * 1e3, algorithmic_GBps=(20.0 * r.size + 16.0 * U) / dt / 1e9, Grecords_per_s=r.size / dt / 1e9)
    os.environ["GLINT_BINNED"] = ""
    glint_amd._native.reload_env()  # the library caches its knobs
    nrow = (1 << 16) // 8
    qr = torch.from_numpy(zipf_keys(rng, shard_rows, nrow, 1.0)).to(dev)
    rout = torch.empty((qr.numel(), cols), dtype=torch.float64, device=dev)
    dt = timed(lambda: lib.glint_mat_pull_rows_dev(h, qr.data_ptr(), rout.data_ptr(), qr.numel(), stream), 10, h)
    k = kernel_ms(h, N.GLINT_K_MAT_PULL_ROWS)
    emit(op="mat_pull_rows_dev", pattern="zipf1.0 rows", rows=qr.numel(), cols=cols, ms=dt * 1e3, kernel_ms=k,
         algorithmic_GBps=qr.numel() * (8 + 2 * cols * 8) / (k * 1e-3) / 1e9)
    # dense row-major sweep push of the whole shard (affine: the ordered plain path)
    dr = torch.arange(shard_rows, dtype=torch.int64, device=dev).repeat_interleave(cols)
    dc = torch.arange(cols, dtype=torch.int32, device=dev).repeat(shard_rows)
    dv = torch.rand(dr.numel(), dtype=torch.float64, device=dev)
    dt = timed(lambda: lib.glint_mat_push_dev(h, dr.data_ptr(), dc.data_ptr(), dv.data_ptr(), dr.numel(), 0, stream),
               5, h)
    emit(op="mat_push_dev", pattern="dense row-major sweep", records=dr.numel(), ms=dt * 1e3,
         algorithmic_GBps=36.0 * dr.numel() / dt / 1e9, note="36 B/record: row 8 + col 4 + value 8 + shard 16")
    msh.destroy()

    # ---- configs[0] end to end over loopback TCP: HBM shards behind the wire ingest ----------------
    import subprocess
    from glint_amd.build import LIB, LOOPBACK_BIN
    for servers, keys, msg in ((2, 1_000_000, 1000), (2, 1 << 24, 79_999)):
        r = subprocess.run([str(LOOPBACK_BIN), "--backend", "gpu", "--lib", str(LIB), "--servers", str(servers),
                            "--keys", str(keys), "--msg", str(msg)], capture_output=True, text=True, timeout=300)
        rec = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else {"error": r.stderr[-300:]}
        emit(op="loopback_tcp", **rec)


if __name__ == "__main__":
    main()
