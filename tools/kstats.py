"""Per-kernel average durations from rocprofv3 --stats directories.

    python tools/kstats.py gpurun_out/bin5/zipf_trace [more dirs]
"""
import csv
import glob
import sys

for d in sys.argv[1:]:
    f = glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True)
    if not f:
        continue
    print(d)
    tot = 0.0
    for r in csv.DictReader(open(f[0])):
        name = r["Name"].split("(")[0].replace("void ", "")
        us = float(r["AverageNs"]) / 1e3
        if "glint::" in name and int(r["Calls"]) >= 10:
            tot += us
        print(f"  {name[-58:]:58s} {r['Calls']:>5s} {us:10.1f} us")
    print(f"  {'sum of glint kernels called >= 10 times':58s} {'':>5s} {tot:10.1f} us")
