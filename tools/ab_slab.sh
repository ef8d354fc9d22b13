set -o pipefail
mkdir -p gpurun_out/r05j
B="python bench.py --no-cpu-baseline --no-north-star --pattern exchange --parts-per-gpu 8 --log2-keys 25"
for r in 1 2; do
  timeout -k 10 200 $B > gpurun_out/r05j/slab_$r.json 2> gpurun_out/r05j/slab_$r.err || exit 1
  GLINT_DIST_SLAB=0 timeout -k 10 200 $B > gpurun_out/r05j/noslab_$r.json 2> gpurun_out/r05j/noslab_$r.err || exit 1
done
R="python bench.py --gpus 2 --no-cpu-baseline --no-north-star --pattern exchange --parts-per-gpu 8 --log2-keys 24 --steps 4 --warmup 2"
GLINT_BENCH_DEVICE=0 GLINT_BENCH_BACKEND=gloo timeout -k 10 300 $R > gpurun_out/r05j/w2_slab.json 2> gpurun_out/r05j/w2_slab.err || exit 1
GLINT_DIST_SLAB=0 GLINT_BENCH_DEVICE=0 GLINT_BENCH_BACKEND=gloo timeout -k 10 300 $R > gpurun_out/r05j/w2_noslab.json 2> gpurun_out/r05j/w2_noslab.err || exit 1
