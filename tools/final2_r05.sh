set -o pipefail
O=gpurun_out/r05o
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
for pat in zipf matrix exchange; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-north-star --pattern $pat > $O/bench_$pat.json 2> $O/bench_$pat.err || exit 1
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-north-star --pattern exchange --parts-per-gpu 8 > $O/bench_exchange_mps8.json 2> $O/bench_exchange_mps8.err || exit 1
