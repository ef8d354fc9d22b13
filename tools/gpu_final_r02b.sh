# Round-2 evidence refresh after the binned-push / ordered-fold work (run via gpurun from the repo
# root): full GPU suite, host per-message latency + loopback (gpu_round2.sh), kernel stats of the
# binned bench commands, FETCH_SIZE / WRITE_SIZE in separate --pmc passes for cfg3 / cfg5, then the
# bench lines. Only the stats / counter CSVs are kept (the traces exceed gpurun's 64 MiB return).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/final2
mkdir -p $OUT
R=$(pwd)
if [ -z "$SKIP_SUITE" ]; then bash tools/gpu_round2.sh || exit 1; fi
cd /tmp
for pat in zipf matrix exchange; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/tr_$pat -o run -- python3 $R/bench.py --no-cpu-baseline --pattern $pat --no-check > $R/$OUT/${pat}_traced.txt 2>&1 || exit 1
  find /tmp/tr_$pat -name "*kernel_stats.csv" -exec cp {} $R/$OUT/kstats_$pat.csv \;
  rm -rf /tmp/tr_$pat
done
for pat in zipf matrix; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d /tmp/pmc_$pat_$c -o run -- python3 $R/bench.py --no-cpu-baseline --pattern $pat --steps 5 --warmup 2 --no-check > $R/$OUT/${pat}_$c.txt 2>&1 || exit 1
    find /tmp/pmc_$pat_$c -name "*counter_collection.csv" -exec cp {} $R/$OUT/pmc_${pat}_$c.csv \;
    rm -rf /tmp/pmc_$pat_$c
  done
done
cd $R
timeout -k 10 300 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit 1
for pat in zipf matrix exchange; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --pattern $pat > $OUT/bench_$pat.json 2> $OUT/bench_$pat.err || exit 1
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline --log2-keys 30 --steps 10 > $OUT/bench_2p30.json 2>&1 || exit 1
