# A/B: buffer-descriptor stores (product) vs plain global stores in the partition kernels, cfg3 Zipf
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/ab
mkdir -p $OUT
R=$(pwd)
cd /tmp
for v in prod gs; do
  if [ $v = gs ]; then export GLINT_GPU_LIB=$R/tools/build/gs/libglint_gpu.so; else unset GLINT_GPU_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/${v}_trace -o run -- python3 $R/bench.py --no-cpu-baseline --pattern zipf --steps 10 --no-check > $R/$OUT/${v}_traced.txt 2>&1 || exit 1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$OUT/${v}_write -o run -- python3 $R/bench.py --no-cpu-baseline --pattern zipf --steps 5 --warmup 2 --no-check > $R/$OUT/${v}_write.txt 2>&1 || exit 1
done
