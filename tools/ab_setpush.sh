set -o pipefail
mkdir -p gpurun_out/r05l
timeout -k 10 420 python -u -m pytest tests/test_gpu_slab.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v --timeout 180 --timeout-method thread -k 'slab or set or dist_exchange or cfg4' > gpurun_out/r05l/pytest.log 2>&1 || exit 1
B="python bench.py --no-cpu-baseline --no-north-star --pattern exchange --parts-per-gpu 8"
for r in 1 2; do
  timeout -k 10 200 $B > gpurun_out/r05l/set_$r.json 2> gpurun_out/r05l/set_$r.err || exit 1
  GLINT_DIST_SET=0 timeout -k 10 200 $B > gpurun_out/r05l/noset_$r.json 2> gpurun_out/r05l/noset_$r.err || exit 1
done
