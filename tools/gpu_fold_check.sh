# ordered-fold / message-path check: ingest, order and parity suites, then the pipelined ring probe,
# the fold timing probe, host per-message latency and the cfg1 loopback for both backends
set -o pipefail
O=gpurun_out/fold
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_order.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
bash tools/ring_probe.sh || exit 1
timeout -k 10 200 python tools/ordered_probe.py > $O/oprobe.txt 2>&1 || exit 1
timeout -k 10 200 python tools/host_latency.py --reps 300 > $O/hl.jsonl 2>&1 || exit 1
LB=tools/loopback/build/glint_loopback
timeout -k 10 100 $LB --backend gpu --lib glint_amd/lib/libglint_gpu.so > $O/lb.jsonl 2>&1 || exit 1
timeout -k 10 100 $LB --backend oracle --lib oracle/build/libglint_oracle.so >> $O/lb.jsonl 2>&1 || exit 1
