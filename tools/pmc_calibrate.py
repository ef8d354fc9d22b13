"""PMC calibration of FETCH_SIZE / WRITE_SIZE per access shape (tools/microbench_pmc.hip).

    python tools/pmc_calibrate.py <known.jsonl> <fetch.csv> <write.csv> <out.json>

known.jsonl is the microbench's stdout (one {"kernel", "read_bytes", "write_bytes"} line per
dispatch); the CSVs are the counter_collection files of two separate rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE) of the same program. For every shape:
    read_factor  = known read bytes  / (1024 * FETCH_SIZE)   (the guide: 2.0 for 16-B streaming reads)
    write_factor = known write bytes / (1024 * WRITE_SIZE)   (the guide: 1.0 for 16-B streaming stores)
averaged over the shape's dispatches. tools/pmc_traffic.py applies them per kernel.
"""
import csv
import json
import sys
from collections import defaultdict


def counters(path, counter):
    vals = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            name = row["Kernel_Name"].split("(")[0].replace("void ", "").strip()
            vals[name].append(float(row["Counter_Value"]))
    return vals


def main():
    known_path, fetch_csv, write_csv, out = sys.argv[1:5]
    known = {}
    for line in open(known_path):
        line = line.strip()
        if line.startswith("{"):
            d = json.loads(line)
            known[d["kernel"]] = (d["read_bytes"], d["write_bytes"])
    fetch, write = counters(fetch_csv, "FETCH_SIZE"), counters(write_csv, "WRITE_SIZE")
    shapes = {}
    for k, (rd, wr) in known.items():
        f = fetch.get(k, [])
        w = write.get(k, [])
        fk = sum(f) / len(f) if f else None
        wk = sum(w) / len(w) if w else None
        shapes[k] = {
            "known_read_bytes": rd, "known_write_bytes": wr,
            "FETCH_SIZE_KiB": fk, "WRITE_SIZE_KiB": wk,
            "read_factor": round(rd / (1024.0 * fk), 4) if rd and fk else None,
            "write_factor": round(wr / (1024.0 * wk), 4) if wr and wk else None,
            "dispatches": [len(f), len(w)],
        }
    res = {"source": "tools/microbench_pmc.hip (2 GiB buffers, every line covered once), separate FETCH_SIZE "
                     "and WRITE_SIZE passes", "shapes": shapes}
    with open(out, "w") as fo:
        json.dump(res, fo, indent=1)
    print(json.dumps({k: (v["read_factor"], v["write_factor"]) for k, v in shapes.items()}))


if __name__ == "__main__":
    main()
