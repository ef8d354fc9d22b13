"""Per-kernel HBM traffic summary from two separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

Prints, per glint kernel, the average raw counter values (KiB) per dispatch and the byte estimates
with the gfx950 corrections of MI355X_MICROARCH.md section HBM (reads = 2 x 1024 x FETCH_SIZE, exact
for 16-B-per-lane streaming reads and uncalibrated for other widths; writes = 1024 x WRITE_SIZE).

    python tools/pmc_kernels.py <fetch counter_collection.csv> <write counter_collection.csv> [out.json]
"""
import csv
import json
import sys
from collections import defaultdict


def per_kernel(path, counter):
    vals = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter or "glint::" not in row["Kernel_Name"]:
                continue
            name = row["Kernel_Name"].split("(")[0].replace("void ", "")
            vals[name].append(float(row["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in vals.items()}


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    res = {}
    for name in sorted(set(fetch) | set(write)):
        f, nf = fetch.get(name, (0.0, 0))
        w, nw = write.get(name, (0.0, 0))
        res[name] = {"FETCH_SIZE_KiB": f, "WRITE_SIZE_KiB": w, "dispatches": [nf, nw],
                     "read_bytes_x2": 2048.0 * f, "write_bytes": 1024.0 * w}
        print(f"{name[:70]:70s} reads {2048.0 * f / 1e6:10.1f} MB (raw {1024.0 * f / 1e6:8.1f})"
              f"  writes {1024.0 * w / 1e6:10.1f} MB  n={nf}/{nw}")
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as fo:
            json.dump(res, fo, indent=1)


if __name__ == "__main__":
    main()
