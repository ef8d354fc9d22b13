set -o pipefail
O=gpurun_out/r05m
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests/test_gpu_slab.py tests/test_gpu_parity.py -m gpu -x -v --timeout 180 --timeout-method thread -k 'slab or set or dist_exchange' > $O/pytest_new.log 2>&1 || exit 1
B="python bench.py --no-cpu-baseline --no-north-star --pattern exchange --parts-per-gpu 8"
for r in 1 2; do
  timeout -k 10 200 $B > $O/set_$r.json 2> $O/set_$r.err || exit 1
  GLINT_DIST_SET=0 timeout -k 10 200 $B > $O/noset_$r.json 2> $O/noset_$r.err || exit 1
done
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
