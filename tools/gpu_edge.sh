#!/bin/bash
# Int-edge route test + exchange tests + the strong-scaling line at BASELINE's 2^30 keys.
set -o pipefail
OUT=gpurun_out/edge
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_exchange.py -m gpu > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -3 $OUT/pytest.txt
timeout -k 10 300 python3 bench.py --no-cpu-baseline --scaling strong --log2-keys 30 --steps 10 > $OUT/bench_strong_2p30.json 2>&1 || { cat $OUT/bench_strong_2p30.json; exit 1; }
cat $OUT/bench_strong_2p30.json
