"""Binned (GLINT_PUSH_UNORDERED) pushes of the cfg3 Zipf(1.1) and uniform-random 2^26-record batches
into a 2^28 Double shard, 3 each -- for a rocprofv3 --kernel-trace --stats stage breakdown.

    rocprofv3 --kernel-trace --stats -d gpurun_out/bin -o bin -- python3 tools/binned_probe.py
"""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
sys.path.insert(0, str(Path(__file__).resolve().parent))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import glint_amd  # noqa: E402
from measure_paths import zipf_keys  # noqa: E402

n = 1 << 28
rng = np.random.default_rng(42)
dev = torch.device("cuda", 0)
sh = glint_amd.PartialVector(glint_amd.RangePartition(0, 0, n), "double", 0)
vals = torch.rand(n // 4, dtype=torch.float64, device=dev)
for name, keys in (("zipf1.1", torch.from_numpy(zipf_keys(rng, n, n // 4, 1.1)).to(dev)),
                   ("uniform", torch.randint(0, n, (n // 4,), dtype=torch.int64, device=dev))):
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sh.update(keys, vals, unordered=True)
        torch.cuda.synchronize()
        print(name, "binned push ms", (time.perf_counter() - t0) * 1e3, flush=True)
sh.destroy()
