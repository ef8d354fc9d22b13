# rocprofv3 kernel statistics of the binned bench patterns (only the stats CSVs are kept)
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for pat in ${PATTERNS:-zipf exchange matrix}; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$pat -o run -- python3 $R/bench.py --no-cpu-baseline --no-check --pattern $pat --steps 20 --warmup 3 > $R/gpurun_out/prof_$pat.log 2>&1
  find /tmp/prof_$pat -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/kstats_$pat.csv \;
done
