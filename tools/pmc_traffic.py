"""Per-launch HBM traffic of the push kernels from rocprofv3 PMC passes.

Reads the FETCH_SIZE and WRITE_SIZE counter CSVs of two separate `rocprofv3 --pmc` passes
(tools/profile_session.sh) and applies the gfx950 corrections of MI355X_MICROARCH.md §HBM:
  * FETCH_SIZE is in KiB and on gfx950 counts exactly half the bytes of a wide (16 B/lane)
    coalesced streaming read -> bytes = 2 * 1024 * FETCH_SIZE (all push/pull loads are 16 B/lane);
  * WRITE_SIZE is in KiB and exact for 16-B-per-lane streaming stores -> bytes = 1024 * WRITE_SIZE.
Writes profiles/<round>/pmc_<tag>.json with the per-kernel and per-push averages.

    python tools/pmc_traffic.py <fetch.csv> <write.csv> <out.json> <records_per_push> [algorithmic_bytes_per_push]

Every glint push kernel (push_*, bin_*) that runs on (nearly) every push of the profiled command is
summed; one-off dispatches (the first push of a shard, taken before the adaptive switch has a
history) are listed but not counted.
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
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def main():
    fetch_csv, write_csv, out, records = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    algorithmic = float(sys.argv[5]) if len(sys.argv) > 5 else 32.0 * records
    fetch, nf = per_kernel(fetch_csv, "FETCH_SIZE")
    write, nw = per_kernel(write_csv, "WRITE_SIZE")
    kernels = {}
    total = 0.0
    # pushes profiled: push_check runs once per push (the apply may run once per window of records,
    # so a kernel's bytes per push = its mean per dispatch x dispatches / pushes)
    checks = [c for k, c in nf.items() if k.startswith("glint::push_check_kernel")]
    pushes = max(checks) if checks else max(list(nf.values()) + [1])
    for name in sorted(set(fetch) | set(write)):
        per = nf.get(name, 0) / pushes
        rd = 2.0 * 1024.0 * fetch.get(name, 0.0) * per
        wr = 1024.0 * write.get(name, 0.0) * nw.get(name, 0) / pushes
        kernels[name] = {"read_bytes_per_push": rd, "write_bytes_per_push": wr,
                         "dispatches": [nf.get(name, 0), nw.get(name, 0)],
                         "FETCH_SIZE_KiB_per_dispatch": fetch.get(name, 0.0),
                         "WRITE_SIZE_KiB_per_dispatch": write.get(name, 0.0)}
        counted = ("push_" in name or "bin_" in name) and nf.get(name, 0) * 2 >= pushes
        kernels[name]["counted"] = counted
        if counted:
            total += rd + wr
    res = {"records_per_push": records, "algorithmic_bytes_per_push": algorithmic, "pushes_profiled": pushes,
           "hbm_bytes_per_launch": total, "traffic_over_algorithmic": total / algorithmic,
           "correction": "read = 2*1024*FETCH_SIZE (gfx950 half-count of 16 B/lane streaming reads); "
                         "write = 1024*WRITE_SIZE", "kernels": kernels}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "kernels"}))


if __name__ == "__main__":
    main()
