"""Summarises an `abn` session of tools/gpu_run.sh: ms per step of each (library, pattern) over rounds,
and the push kernels' summed device time per step (steadier than the wall time across rounds).

    python tools/ab_summary.py gpurun_out/<TAG>
"""
import json
import re
import sys
from collections import defaultdict
from pathlib import Path

rows = defaultdict(list)
for f in sorted(Path(sys.argv[1]).glob("ab_*.log")):
    m = re.match(r"ab_(.+)_(\w+)_(\d+)\.log", f.name)
    line = [l for l in f.read_text().splitlines() if l.startswith("{")]
    if not m or not line:
        continue
    d = json.loads(line[-1])
    rows[(m.group(2), m.group(1))].append((d["ms_per_step"], d.get("check"), d["roofline"].get("kernel_ms")))
for (pat, lib), v in sorted(rows.items()):
    print(f"{pat:10s} {lib:12s} ms {[x[0] for x in v]} kernel ms {[x[2] for x in v]} check {[x[1] for x in v]}")
