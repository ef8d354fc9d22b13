"""Per-launch HBM traffic of the push kernels from rocprofv3 PMC passes.

Reads the FETCH_SIZE and WRITE_SIZE counter CSVs of two separate `rocprofv3 --pmc` passes
(tools/gpu_run.sh stage pmc) and applies, per kernel, the factors of its access shapes from the
newest per-shape calibration (profiles/<round>/pmc_calibration.json, tools/microbench_pmc.hip):
  * FETCH_SIZE is in KiB; on gfx950 it counts half the bytes of a coalesced streaming read of 16-,
    8- or 4-B lanes, and of 4-B loads at an 8-B stride (the i64 keys' low words), all measured 2.000;
  * WRITE_SIZE is in KiB and exact (0.997-0.999) for 16-, 8- and 4-B coalesced stores.
Writes profiles/<round>/pmc_<tag>.json with the per-kernel and per-push averages.

    python tools/pmc_traffic.py <fetch.csv> <write.csv> <out.json> <records_per_push> [algorithmic_bytes_per_push]

Every glint push kernel (push_*, bin_*) that runs on (nearly) every push of the profiled command is
summed; one-off dispatches (the first push of a shard, taken before the adaptive switch has a
history) are listed but not counted.
"""
import csv
import glob
import json
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent

# The access shapes of each kernel's HBM streams (tools/microbench_pmc.hip names): the calibration of
# the shape gives the kernel's FETCH_SIZE / WRITE_SIZE factor. Shapes marked * are not full-line
# streams (random gathers, short store runs): the counter reports the fabric requests they cost, the
# calibrated factor of the same width is applied, and the bytes read as request bytes, not payload.
SHAPES = {
    "push_check": (["ld16"], []),
    "push_apply": (["ld16"], ["st16"]),
    "push_scatter": (["ld8", "*gather8"], ["*atomic8"]),
    "bin_count": (["ld4s8", "ld4"], []),
    # (round 6: the chunk-local partition stores each chunk as one contiguous range; bin_scan reads the
    # chunk table's bucket rows and writes each bucket's prefix / place rows)
    "bin_part": (["ld4s8", "ld8", "ld4"], ["st4", "st8"]),
    "bin_part_dedup": (["ld4s8", "ld8", "ld4"], ["st4", "st8"]),
    "bin_scan": (["ld4"], ["st4"]),
    "bin_fcount": (["ld4"], []),
    "bin_fpart": (["ld4", "ld8"], ["*st4runs", "*st8runs"]),
    "bin_apply": (["ld4", "ld8", "rmw16"], ["rmw16"]),
    "bin_hot": (["ld8"], ["st8"]),
    # v2 fine stage: the item sort gathers its item from its chunks' runs (~64 records each) and writes
    # it (u16 offsets, values) as whole-wave runs; the apply gathers ~16-32-record runs per item and
    # read-modify-writes lines
    "bin_fsort": (["*ld4", "*ld8"], ["st8"]),
    "bin_plan": (["ld4"], ["st8"]),
    "bin_apply2": (["*ld4", "*ld8", "rmw16"], ["rmw16"]),
    # one push over several shards (glint_vec_push_dev_shards): the key check streams the keys, the
    # scatter is push_scatter's shape
    "set_validate": (["ld8"], []),
    "set_scatter": (["ld8", "*gather8"], ["*atomic8"]),
}


def calibration():
    """The newest committed per-shape calibration (tools/pmc_calibrate.py), or None."""
    files = sorted(glob.glob(str(ROOT / "profiles" / "*" / "pmc_calibration.json")))
    if not files:
        return None, None
    return json.loads(Path(files[-1]).read_text()), str(Path(files[-1]).relative_to(ROOT))


def kernel_factor(name, cal):
    """(read factor, write factor, shapes, source note) for a kernel: the calibrated factors of its
    shapes (they must agree; the guide's 2 / 1 when no calibration is committed)."""
    short = name.replace("glint::", "").split("<")[0].replace("_kernel", "")
    key = next((k for k in sorted(SHAPES, key=len, reverse=True) if short.startswith(k)), None)
    rshapes, wshapes = SHAPES.get(key, ([], []))
    if cal is None:
        return 2.0, 1.0, (rshapes, wshapes), "guide (uncalibrated)"
    sh = cal["shapes"]
    rf = [sh[x.lstrip("*")]["read_factor"] for x in rshapes if x.lstrip("*") in sh and sh[x.lstrip("*")]["read_factor"]]
    wf = [sh[x.lstrip("*")]["write_factor"] for x in wshapes if x.lstrip("*") in sh and sh[x.lstrip("*")]["write_factor"]]
    r = sum(rf) / len(rf) if rf else 2.0
    w = sum(wf) / len(wf) if wf else 1.0
    note = "calibrated" if rf or wf else "guide (no calibrated shape)"
    if any(x.startswith("*") for x in rshapes + wshapes):
        note += "; includes non-full-line shapes (request bytes)"
    return r, w, (rshapes, wshapes), note


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
    cal, cal_src = calibration()
    kernels = {}
    total = 0.0
    # pushes profiled: the most dispatched of the kernels that run once per push -- push_check (the
    # checked path), bin_scan (every binned push, bin_count before round 6; whole-push bins run no
    # check) and push_scatter (a
    # whole-push scatter runs alone) -- (the apply may run once per window of records, so a kernel's
    # bytes per push = its mean per dispatch x dispatches / pushes)
    once = [c for k, c in nf.items()
            if k.startswith(("glint::push_check_kernel", "glint::bin_count_kernel", "glint::bin_scan_kernel",
                             "glint::push_scatter_kernel",
                             "glint::set_scatter_kernel"))]
    pushes = max(once) if once else max(list(nf.values()) + [1])
    for name in sorted(set(fetch) | set(write)):
        per = nf.get(name, 0) / pushes
        rfac, wfac, shapes, note = kernel_factor(name, cal)
        rd = rfac * 1024.0 * fetch.get(name, 0.0) * per
        wr = wfac * 1024.0 * write.get(name, 0.0) * nw.get(name, 0) / pushes
        kernels[name] = {"read_bytes_per_push": rd, "write_bytes_per_push": wr,
                         "dispatches": [nf.get(name, 0), nw.get(name, 0)],
                         "FETCH_SIZE_KiB_per_dispatch": fetch.get(name, 0.0),
                         "WRITE_SIZE_KiB_per_dispatch": write.get(name, 0.0),
                         "correction": {"read_factor": rfac, "write_factor": wfac, "read_shapes": shapes[0],
                                        "write_shapes": shapes[1], "source": (cal_src or "MI355X_MICROARCH.md")
                                        + ": " + note}}
        counted = ("push_" in name or "bin_" in name or "set_" in name) and nf.get(name, 0) * 2 >= pushes
        kernels[name]["counted"] = counted
        if counted:
            total += rd + wr
    res = {"records_per_push": records, "algorithmic_bytes_per_push": algorithmic, "pushes_profiled": pushes,
           "hbm_bytes_per_launch": total, "traffic_over_algorithmic": total / algorithmic,
           "correction": "per kernel (kernels[*].correction): read = f_r*1024*FETCH_SIZE, write = f_w*1024*WRITE_SIZE "
                         "with the factors of the kernel's access shapes calibrated by tools/microbench_pmc.hip "
                         f"({cal_src or 'none committed: the guide 2 / 1'})", "kernels": kernels}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "kernels"}))


if __name__ == "__main__":
    main()
