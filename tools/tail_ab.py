"""Unordered-tail A/B: the LDS-hash atomic scatter (push_scatter) against the binned pipeline
(push_binned), as a function of the push's density (records per 4096-element slab), for the shapes
the bench lines push: uniform keys into a 2^28-element shard at 2^20 .. 2^26 records (the cfg4 key
space's 8-partition shards take 2^23, cfg4b's one shard 2^26), cfg3's Zipf(1.1) 2^26 and cfg5's
2^23 matrix triplets. Each case is timed on one stream, and the uniform ones also as 8 shards pushed
on 8 concurrent streams (the 8-partition exchange line's shape). Prints one JSON line per case:

    python tools/tail_ab.py [--reps 10]

GLINT_BINNED=0 / 1 (re-read through glint_reload_env) forces the path, and GLINT_BIN_DENSITY=0 lifts the
density floor of the adaptive switch, so both paths are timed at every density; the library is
GLINT_GPU_LIB or the in-tree build.
"""
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    import numpy as np
    import torch
    from glint_amd import PartialMatrix, PartialVector, RangePartition
    from glint_amd import _native as N

    reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 10
    lib = N.load()
    dev = torch.device("cuda", 0)
    elems = 1 << 28

    os.environ["GLINT_BIN_DENSITY"] = "0"

    def timed(shards, batches, mode, streams):
        os.environ["GLINT_BINNED"] = mode
        N.reload_env()
        sts = [torch.cuda.Stream(dev) for _ in shards] if streams else [torch.cuda.current_stream(dev)] * len(shards)

        def push_all():
            for sh, st, b in zip(shards, sts, batches):
                h = sh.handle
                if len(b) == 3:
                    rc = lib.glint_mat_push_dev(h, b[0].data_ptr(), b[1].data_ptr(), b[2].data_ptr(), b[0].numel(), 0,
                                                st.cuda_stream)
                else:
                    rc = lib.glint_vec_push_dev(h, b[0].data_ptr(), b[1].data_ptr(), b[0].numel(), 0,
                                                st.cuda_stream)  # check + apply + the tail, as the bench lines
                assert rc == 0, rc
        for _ in range(3):  # warm-up: scratch allocations and the front end's measurements, one push at a
            push_all()      # time, each ended by the shard's sync point (where the library latches them)
            for sh, st in zip(shards, sts):
                sh.sync(st.cuda_stream)
        t0 = time.perf_counter()
        for _ in range(reps):
            push_all()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / reps * 1e3

    def run(name, make, nshards, streams):
        shards, batches = [], []
        for i in range(nshards):
            sh, b = make(i)
            shards.append(sh)
            batches.append(b)
        out = {"case": name, "shards": nshards, "streams": nshards if streams else 1}
        for mode, tag in (("0", "scatter_ms"), ("1", "binned_ms")):
            out[tag] = round(timed(shards, batches, mode, streams), 4)
        out["records_per_push"] = int(batches[0][0].numel())
        out["records_per_slab"] = round(out["records_per_push"] / (elems / 4096.0 if "cfg5" not in name else
                                                                      (1 << 26) / 4096.0), 3)
        print(json.dumps(out), flush=True)
        for sh in shards:
            sh.destroy()
        del shards, batches
        torch.cuda.empty_cache()

    gen = torch.Generator(device=dev)
    gen.manual_seed(7)

    def uniform(nrec):
        def make(i):
            sh = PartialVector(RangePartition(i, 0, elems), "double", device=0)
            k = torch.randint(0, elems, (nrec,), dtype=torch.int64, device=dev, generator=gen)
            return sh, (k, torch.rand(nrec, dtype=torch.float64, device=dev, generator=gen))
        return make

    for lg in range(20, 27):
        run(f"uniform 2^{lg} into 2^28", uniform(1 << lg), 1, False)
    for lg in (21, 22, 23, 24):  # 8 shards on 8 streams (the cfg4 key space's local pushes)
        run(f"uniform 2^{lg} into 2^28 x 8 shards", uniform(1 << lg), 8, True)

    rng = np.random.default_rng(42)

    def zipf(i):  # cfg3
        nrec = 1 << 26
        r = rng.zipf(1.1, size=int(nrec * 1.3))
        r = r[r <= elems][:nrec] - 1
        k = torch.from_numpy(rng.permutation(elems)[r].astype(np.int64)).to(dev)
        return PartialVector(RangePartition(0, 0, elems), "double", device=0), \
            (k, torch.rand(k.numel(), dtype=torch.float64, device=dev, generator=gen))
    run("cfg3 zipf(1.1) 2^26 into 2^28", zipf, 1, False)

    def matrix(i):  # cfg5 per GPU
        rows, cols, nrec = 1 << 17, 512, 1 << 23
        rk = np.minimum(np.floor(np.power(float(rows), rng.random(nrec))).astype(np.int64) - 1, rows - 1)
        r = torch.from_numpy(rng.permutation(rows)[rk].astype(np.int64)).to(dev)
        c = torch.from_numpy(rng.integers(0, cols, nrec).astype(np.int32)).to(dev)
        return PartialMatrix(RangePartition(0, 0, rows), cols, "double", device=0), \
            (r, c, torch.rand(nrec, dtype=torch.float64, device=dev, generator=gen))
    run("cfg5 matrix 2^23 into 2^17 x 512", matrix, 1, False)


if __name__ == "__main__":
    main()
