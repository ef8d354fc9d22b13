"""Binned-push debugging probe: replays pushes on one shard with a forced front end and reports, per
push, how many elements (and which slabs) differ from the oracle."""
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from glint_amd import PartialVector, RangePartition  # noqa: E402
from oracle import oracle as O  # noqa: E402


def run(front, seq, size=1 << 20, seed=3):
    os.environ["GLINT_BIN_FRONT"] = front
    rng = np.random.default_rng(seed)
    hot = rng.integers(0, 5000, 1 << 20).astype(np.int64)
    uniq = rng.permutation(size).astype(np.int64)
    pats = {"hot": hot, "uniq": uniq}
    ref = O.OracleVector(O.part_range(0, size), O.CODE["long"])
    with PartialVector(RangePartition(0, 0, size), "long", 0) as sh:
        for i, name in enumerate(seq):
            keys = pats[name]
            vals = rng.integers(-9, 9, keys.size).astype(np.int64)
            sh.update(keys, vals, unordered=True)
            ref.update(keys, vals)
            got = sh.to_numpy()
            bad = np.nonzero(got != ref.data)[0]
            slabs = np.unique(bad >> 12)
            print(f"front={front} push {i} ({name}): {bad.size} bad elements, slabs {slabs[:12].tolist()}"
                  f"{'...' if slabs.size > 12 else ''} diff sample {(got - ref.data)[bad[:5]].tolist()}", flush=True)


for front in ("dedup", "prep"):
    run(front, ["uniq", "uniq", "hot", "hot"])
