"""Print a rocprofv3 kernel summary (name, calls, avg us, total %) from its rocpd SQLite output or
its *_kernel_stats.csv.   python tools/kstats.py <results.db | kernel_stats.csv> [name-width]"""
import csv
import sqlite3
import sys

path = sys.argv[1]
w = int(sys.argv[2]) if len(sys.argv) > 2 else 90
if path.endswith(".db"):
    rows = sqlite3.connect(path).execute(
        "select name, total_calls, average, percentage from top_kernels order by total_duration desc").fetchall()
    rows = [(r[0], r[1], r[2], r[3]) for r in rows]  # rocpd averages are in us
else:
    rows = [(r["Name"], int(r["Calls"]), float(r["AverageNs"]) / 1e3, float(r["Percentage"]))
            for r in csv.DictReader(open(path))]
for name, calls, avg_us, pct in rows:
    short = name.replace("void ", "").split("(")[0] if "rocprim" not in name else \
        "rocprim::" + ("onesweep_iteration" if "onesweep_iteration" in name else "histogram/offsets" if "onesweep" in name
                       else "scan" if "scan" in name else "other")
    print(f"{short[:w]:{w}s} {calls:6d} {avg_us:10.1f} us {pct:6.2f} %")
