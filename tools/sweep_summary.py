"""Summarise gpurun_out/sweep_env.txt (tools/sweep_bench_env.sh): one line per knob setting."""
import json
import sys

for line in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/sweep_env.txt"):
    if line.startswith("CHECK"):
        print(line.strip(), end="  ")
    elif line.startswith("{"):
        d = json.loads(line)
        r = d["roofline"]
        print(d["value"], r["frac"], r["push_kernels_ms"], d["check"])
