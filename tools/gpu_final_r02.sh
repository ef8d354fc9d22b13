# Round-2 evidence for profiles/r02 (run via gpurun from the repo root):
#   kernel trace + stats of the default bench command (cfg2) and of cfg3 / cfg5 / cfg4b(N=1),
#   FETCH_SIZE and WRITE_SIZE in separate --pmc passes (never with tracing domains) for cfg2/3/5,
#   then the bench lines themselves (default with the CPU baseline; 2^30; pull; rowpull).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/final
mkdir -p $OUT
R=$(pwd)
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/dense_trace -o run -- python3 $R/bench.py --no-cpu-baseline > $R/$OUT/bench_dense_traced.txt 2>&1 || exit 1
for pat in dense zipf matrix; do
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$OUT/${pat}_fetch -o run -- python3 $R/bench.py --no-cpu-baseline --pattern $pat --steps 5 --warmup 2 --no-check > $R/$OUT/${pat}_fetch.txt 2>&1 || exit 1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$OUT/${pat}_write -o run -- python3 $R/bench.py --no-cpu-baseline --pattern $pat --steps 5 --warmup 2 --no-check > $R/$OUT/${pat}_write.txt 2>&1 || exit 1
done
cd $R
timeout -k 10 300 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --log2-keys 30 --steps 10 > $OUT/bench_2p30.json 2>&1 || exit 1
for pat in pull rowpull; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --pattern $pat > $OUT/bench_$pat.json 2>&1 || exit 1
done
timeout -k 10 200 python3 bench.py --no-cpu-baseline --scaling strong --log2-keys 28 > $OUT/bench_strong.json 2>&1 || exit 1
