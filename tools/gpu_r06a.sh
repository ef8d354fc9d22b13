# round 6, first GPU pass: the retired v1 binned pipeline's replacement (wide partition stores) and the
# new tests first, then the whole GPU suite, smoke and the default bench line
set -o pipefail
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_wide.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_exchange.py -m gpu -x -v --timeout 240 --timeout-method thread -k 'fine_stage or stream_of_batches or windowed or rotated or self_launches or set' > $O/pytest_new.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/suite.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
