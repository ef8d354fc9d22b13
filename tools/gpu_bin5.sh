# binned parity, then cfg3 / cfg5 / cfg4b(N=1) bench lines and kernel breakdowns
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/bin5
mkdir -p $OUT
R=$(pwd)
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -k "binned or cfg or adaptive" --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.txt 2>&1 || exit 1
for pat in zipf matrix exchange; do
  timeout -k 10 200 python3 bench.py --pattern $pat --no-cpu-baseline > $OUT/bench_$pat.json 2>&1 || exit 1
done
cd /tmp
for pat in zipf matrix exchange; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/${pat}_trace -o run -- python3 $R/bench.py --no-cpu-baseline --pattern $pat --steps 10 --no-check > $R/$OUT/${pat}_traced.txt 2>&1 || exit 1
done
