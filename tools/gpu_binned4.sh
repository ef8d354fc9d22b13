# binned parity + cfg3/cfg5 bench lines + kernel breakdowns (+ cfg3 with the plain front end forced)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/bin
mkdir -p $OUT
R=$(pwd)
timeout -k 10 100 python tools/debug_binned.py > $OUT/debug.txt 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -k "binned or cfg or adaptive" --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || exit 1
timeout -k 10 200 python3 bench.py --pattern zipf --no-cpu-baseline > $OUT/bench_zipf.json 2>&1 || exit 1
timeout -k 10 200 python3 bench.py --pattern matrix --no-cpu-baseline > $OUT/bench_matrix.json 2>&1 || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/ztrace -o run -- python3 $R/bench.py --no-cpu-baseline --pattern zipf --steps 10 --no-check > $R/$OUT/zipf_traced.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/mtrace -o run -- python3 $R/bench.py --no-cpu-baseline --pattern matrix --steps 10 --no-check > $R/$OUT/matrix_traced.txt 2>&1 || exit 1
GLINT_BIN_FRONT=prep timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/ptrace -o run -- python3 $R/bench.py --no-cpu-baseline --pattern zipf --steps 10 --no-check > $R/$OUT/zipf_prep_traced.txt 2>&1 || exit 1
