set -o pipefail
mkdir -p gpurun_out/r05k
B="python bench.py --no-cpu-baseline --no-north-star --pattern exchange --parts-per-gpu 8"
for r in 1 2; do
  GLINT_SYNC_FLUSH=1 timeout -k 10 200 $B > gpurun_out/r05k/flush_$r.json 2> gpurun_out/r05k/flush_$r.err || exit 1
  GLINT_SYNC_FLUSH=0 timeout -k 10 200 $B > gpurun_out/r05k/noflush_$r.json 2> gpurun_out/r05k/noflush_$r.err || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r05k/tr -o run -- python3 bench.py --no-cpu-baseline --no-north-star --no-check --pattern exchange --parts-per-gpu 8 --steps 5 --warmup 2 > gpurun_out/r05k/tr.log 2>&1 || exit 1
