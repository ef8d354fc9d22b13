"""Binned (GLINT_PUSH_UNORDERED) pushes of the cfg3 Zipf(1.1) and uniform-random 2^26-record batches
into a 2^28 Double shard, 4 per front end of the tail (GLINT_BIN_FRONT = dedup | prep), with
wall-clock times -- and, under rocprofv3 --kernel-trace --stats, the stage breakdown.

    python3 tools/binned_probe.py
    rocprofv3 --kernel-trace --stats -d gpurun_out/bin -o bin -- python3 tools/binned_probe.py
"""
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import glint_amd  # noqa: E402


def zipf_keys(rng, n_keys, n, s):
    """Zipf(s) ranks over [0, n_keys) mapped through a seeded permutation (as tools/measure_paths.py)."""
    ranks = rng.zipf(s, size=int(n * 1.4))
    ranks = ranks[ranks <= n_keys][:n] - 1
    return rng.permutation(n_keys)[ranks].astype(np.int64)


n = 1 << 28
rng = np.random.default_rng(42)
dev = torch.device("cuda", 0)
dtype = os.environ.get("GLINT_PROBE_DTYPE", "double")  # double | float
sh = glint_amd.PartialVector(glint_amd.RangePartition(0, 0, n), dtype, 0)
vals = torch.rand(n // 4, dtype=torch.float64 if dtype == "double" else torch.float32, device=dev)
fronts = sys.argv[1:] or ["dedup", "prep"]
for name, keys in (("zipf1.1", torch.from_numpy(zipf_keys(rng, n, n // 4, 1.1)).to(dev)),
                   ("uniform", torch.randint(0, n, (n // 4,), dtype=torch.int64, device=dev))):
    for front in fronts:
        os.environ["GLINT_BIN_FRONT"] = front
        glint_amd._native.reload_env()  # the library caches its knobs
        ts = []
        for _ in range(4):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            sh.update(keys, vals, unordered=True)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        print(json.dumps({"dtype": dtype, "pattern": name, "front": front, "records": int(keys.numel()),
                          "push_ms": [round(t, 3) for t in ts], "best_ms": round(min(ts[1:]), 3)}), flush=True)
sh.destroy()
