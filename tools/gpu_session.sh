# one GPU session: parity tests, occupancy sweep, profiles (run via gpurun from the repo root)
set -o pipefail
timeout -k 10 500 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.txt 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.txt
for b in 1 2 4; do GLINT_BLOCKS_PER_CU=$b timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_b$b.txt 2>&1 || exit 1; done
timeout -k 10 150 python bench.py --no-cpu-baseline --steps 10 --log2-keys 30 > gpurun_out/bench_30.txt 2>&1 || exit 1
timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 --pattern zipf > gpurun_out/bench_zipf.txt 2>&1 || exit 1
