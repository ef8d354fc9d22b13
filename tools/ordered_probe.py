"""Order-preserving fold timing by message size and key pattern (tuning probe): device pushes with
deterministic=True (the fold for n <= 131072) and host pushes (glint_vec_push), per call, in us."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from glint_amd import PartialVector, RangePartition  # noqa: E402

SIZE = 1 << 24
rng = np.random.default_rng(1)
with PartialVector(RangePartition(0, 0, SIZE), "double", 0) as sh:
    for n in (1000, 4096, 8192, 10000, 32768, 79999):
        pats = {"random": rng.integers(0, SIZE, n), "distinct": rng.permutation(SIZE)[:n],
                "sorted": np.arange(n) * 7, "hot16": rng.integers(0, 16, n)}
        for name, k in pats.items():
            k = k.astype(np.int64)
            v = rng.random(n)
            kd, vd = torch.from_numpy(k).cuda(), torch.from_numpy(v).cuda()
            for _ in range(3):
                sh.update(kd, vd, deterministic=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            R = 50
            for _ in range(R):
                sh.update(kd, vd, deterministic=True, sync=False)
            torch.cuda.synchronize()
            dev = (time.perf_counter() - t0) / R * 1e6
            t0 = time.perf_counter()
            for _ in range(R):
                sh.update(k, v)
            host = (time.perf_counter() - t0) / R * 1e6
            print(f"n={n:6d} {name:9s} device {dev:8.1f} us  host {host:8.1f} us", flush=True)
