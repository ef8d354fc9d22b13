set -o pipefail
O=gpurun_out/r05p
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests/test_gpu_slab.py tests/test_gpu_parity.py -m gpu -x -v --timeout 180 --timeout-method thread -k 'slab or set or dist_exchange' > $O/pytest_new.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
