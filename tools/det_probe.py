"""Deterministic push of the cfg3 Zipf(1.1) batch (2^26 records into a 2^28 shard), 3 times --
for a rocprofv3 --kernel-trace --stats breakdown of the sort + fold stages.

    rocprofv3 --kernel-trace --stats -d gpurun_out/det -- python3 tools/det_probe.py
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
zk = zipf_keys(rng, n, n // 4, 1.1)
uniq, counts = np.unique(zk, return_counts=True)
print("records", zk.size, "distinct", uniq.size, "hottest", int(counts.max()), "runs>64", int((counts > 64).sum()),
      "records in runs>64", int(counts[counts > 64].sum()), flush=True)
dev = torch.device("cuda", 0)
sh = glint_amd.PartialVector(glint_amd.RangePartition(0, 0, n), "double", 0)
keys = torch.from_numpy(zk).to(dev)
vals = torch.rand(zk.size, dtype=torch.float64, device=dev)
for _ in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sh.update(keys, vals, deterministic=True)
    torch.cuda.synchronize()
    print("det push ms", (time.perf_counter() - t0) * 1e3, flush=True)
sh.destroy()
