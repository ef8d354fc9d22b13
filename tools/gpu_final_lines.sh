# end-of-round check on the committed build: GPU suite, smoke, the default and binned bench lines
set -o pipefail
O=gpurun_out/endr2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 200 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
for pat in zipf matrix exchange; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --pattern $pat > $O/bench_$pat.json 2> $O/bench_$pat.err || exit 1
done
