# rocprofv3 evidence for profiles/ (run via gpurun from the repo root):
#   1. kernel trace + stats of the default bench command (cfg2 dense) and of the cfg3 Zipf bench
#   2. FETCH_SIZE and WRITE_SIZE in separate --pmc passes (never combined with tracing domains)
#   3. the default bench line itself (with the CPU baseline)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --no-cpu-baseline > $OUT/bench_traced.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 --no-check > $OUT/bench_fetch.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 --no-check > $OUT/bench_write.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ztrace -o run -- python3 bench.py --no-cpu-baseline --pattern zipf > $OUT/bench_zipf_traced.txt 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > $OUT/bench_default.txt 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --log2-keys 30 --steps 10 > $OUT/bench_2p30.txt 2>&1 || exit 1
timeout -k 10 400 python3 tools/measure_paths.py > $OUT/measure_paths.jsonl 2> $OUT/measure_paths.err || exit 1
timeout -k 10 200 python3 tools/binned_probe.py > $OUT/binned_probe.jsonl 2>&1 || exit 1
