"""Per-kernel averages of the SQ counters collected by tools/gpu_sqprof.sh.

    python tools/sq_summary.py gpurun_out/sq/zipf_a gpurun_out/sq/zipf_b
"""
import csv
import glob
import sys
from collections import defaultdict


def load(d):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "glint::" not in k:
                continue
            name = k.split("(")[0].replace("void ", "").replace("glint::", "")
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


res = defaultdict(dict)
for d in sys.argv[1:]:
    for k, cs in load(d).items():
        for c, v in cs.items():
            res[k][c] = sum(v) / len(v)
for k, cs in sorted(res.items()):
    print(k)
    wc = cs.get("SQ_WAVE_CYCLES", 0) or 1
    for c in sorted(cs):
        extra = f"  ({100.0 * cs[c] / wc:5.1f}% of wave-cycles)" if c.startswith(("SQ_WAIT", "SQ_ACTIVE", "SQ_BUSY")) else ""
        print(f"   {c:26s} {cs[c]:16.0f}{extra}")
