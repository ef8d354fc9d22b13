# Bench the dense push under launch-shape knobs: CHECKS / SWEEPS = lists of GLINT_CHECK_BPC / GLINT_SWEEP_BPC
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/sweep_env.txt
: > $out
for cb in ${CHECKS:-2}; do for sb in ${SWEEPS:-1}; do
  echo "CHECK_BPC=$cb SWEEP_BPC=$sb" >> $out
  GLINT_CHECK_BPC=$cb GLINT_SWEEP_BPC=$sb timeout -k 10 120 python bench.py --no-cpu-baseline --steps 30 >> $out 2>&1 || exit 1
done; done
