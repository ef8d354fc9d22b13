set -o pipefail
timeout -k 10 300 python tools/sweep_push.py 28 dense GLINT_CHECK_BPC > gpurun_out/sweep28c.txt 2>&1 || exit 1
timeout -k 10 300 python tools/sweep_push.py 28 dense GLINT_APPLY_BPC > gpurun_out/sweep28a.txt 2>&1 || exit 1
timeout -k 10 150 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/bench_28.txt 2>&1 || exit 1
