# round 6, the last check of the final tree on one box: the whole GPU suite, smoke and every bench line
set -o pipefail
TAG=${TAG:-r06f2}
O=gpurun_out/$TAG
mkdir -p $O
run() {  # run <name> <seconds> <command...>
  local name=$1 secs=$2
  shift 2
  echo "[$(date +%T)] $name" >&2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -30 $O/$name.log >&2; exit $rc; fi
}
run suite 1200 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run bench_default 400 python3 bench.py
for pat in zipf matrix exchange pull rowpull; do
  run bench_$pat 300 python3 bench.py --no-cpu-baseline --no-north-star --pattern $pat
done
run bench_exchange_mps8 300 python3 bench.py --no-cpu-baseline --no-north-star --pattern exchange --parts-per-gpu 8
for pat in zipf matrix exchange; do
  run bench_${pat}_batches8 400 python3 bench.py --no-cpu-baseline --no-north-star --pattern $pat --batches 8
done
echo "session done" >&2
