set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/sweep1.txt
: > $out
for cb in 2 4 8; do for sb in 1 2; do
  echo "CHECK_BPC=$cb SWEEP_BPC=$sb" >> $out
  GLINT_CHECK_BPC=$cb GLINT_SWEEP_BPC=$sb timeout -k 10 120 python bench.py --no-cpu-baseline --steps 30 >> $out 2>&1 || exit 1
done; done
