# round 6, the final measurement session on one box: the wide tests, the whole GPU suite and smoke, every bench
# line (and the sparse lines on 8 rotated batches), kernel stats and PMC passes of the sparse lines
set -o pipefail
TAG=${TAG:-r06z}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
R=$(pwd)
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
echo "[$(date +%T)] kstats dense_2p30" >&2
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_dense_2p30 -o run \
   -- python3 $R/bench.py --no-cpu-baseline --steps 10 > $R/$O/prof_dense_2p30.log 2>&1) || { tail -30 $O/prof_dense_2p30.log >&2; exit 1; }
find /tmp/prof_dense_2p30 -name "*kernel_stats.csv" -exec cp {} $O/kstats_dense_2p30.csv \;
for pat in zipf matrix exchange; do
  echo "[$(date +%T)] kstats $pat" >&2
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$pat -o run \
     -- python3 $R/bench.py --no-cpu-baseline --no-north-star --pattern $pat --steps 10 --warmup 2 > $R/$O/prof_$pat.log 2>&1) || { tail -30 $O/prof_$pat.log >&2; exit 1; }
  find /tmp/prof_$pat -name "*kernel_stats.csv" -exec cp {} $O/kstats_$pat.csv \;
done
for pat in zipf matrix exchange; do
  for c in FETCH_SIZE WRITE_SIZE; do
    echo "[$(date +%T)] pmc $pat $c" >&2
    (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d /tmp/pmc_${pat}_$c -o run \
       -- python3 $R/bench.py --no-cpu-baseline --no-north-star --no-check --steps 5 --warmup 2 --pattern $pat > $R/$O/pmc_${pat}_$c.log 2>&1) \
       || { tail -30 $O/pmc_${pat}_$c.log >&2; exit 1; }
    find /tmp/pmc_${pat}_$c -name "*counter_collection.csv" -exec cp {} $O/pmc_${pat}_$c.csv \;
  done
done
echo "session done" >&2
