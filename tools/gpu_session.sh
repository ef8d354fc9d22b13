# One GPU session: parity suite, then (unless it crashed or timed out) the per-path measurements.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q --maxfail=5 > gpurun_out/pytest_gpu.txt 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 500 python tools/measure_paths.py > gpurun_out/paths.jsonl 2> gpurun_out/paths.err
