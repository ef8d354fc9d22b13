set -o pipefail
timeout -k 10 500 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.txt 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.txt
timeout -k 10 600 python tools/measure_paths.py > gpurun_out/paths.jsonl 2> gpurun_out/paths.err
