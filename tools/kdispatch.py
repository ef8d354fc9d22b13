"""Per-dispatch kernel durations (us) from a rocprofv3 rocpd SQLite output, grouped by kernel.
    python tools/kdispatch.py <results.db> [substring-filter]"""
import sqlite3
import sys
from collections import defaultdict

rows = sqlite3.connect(sys.argv[1]).execute("select name, start, end from kernels order by start").fetchall()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
d = defaultdict(list)
for name, s, e in rows:
    n = name.replace("void ", "").split("(")[0]
    if "rocprim" in name:
        n = "rocprim " + ("onesweep_iteration" if "onesweep_iteration" in name else
                          "onesweep_histogram" if "onesweep" in name else "scan" if "scan" in name else "other")
    if flt in n:
        d[n].append(round((e - s) / 1e3, 1))
for k, v in d.items():
    print(f"{k[:60]:60s} {v}")
