# GPU suite, then host per-message latency and the loopback harness (cfg1, cfg4 shapes) for both backends
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.txt 2>&1
rc=$?
echo "rc=$rc" >> $OUT/pytest.txt
[ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python tools/host_latency.py --reps 300 > $OUT/host_latency.jsonl 2>$OUT/host_latency.err || exit 1
LB=tools/loopback/build/glint_loopback
G="--backend gpu --lib glint_amd/lib/libglint_gpu.so"
O="--backend oracle --lib oracle/build/libglint_oracle.so"
for args in "" "--window 1" "--keys 16777216 --msg 79999" "--clients 64 --servers 8 --keys 33554432" \
            "--clients 64 --servers 8 --keys 33554432 --pattern uniform --records 524288 --dtype long"; do
  timeout -k 10 200 $LB $G $args >> $OUT/loopback_gpu.jsonl 2>>$OUT/loopback.err || exit 1
  timeout -k 10 200 $LB $O $args >> $OUT/loopback_oracle.jsonl 2>>$OUT/loopback.err || exit 1
done
