# binned-push knob sweep (tuning only): ms per push of the binned bench patterns
set -e
run() {  # tag pattern env...
  tag=$1; pat=$2; shift 2
  env "$@" timeout -k 10 120 python bench.py --pattern $pat --steps 20 --warmup 3 > gpurun_out/sw_${pat}_${tag}.json 2>gpurun_out/sw_${pat}_${tag}.err
  python -c "import json;d=json.loads(open('gpurun_out/sw_${pat}_${tag}.json').read().strip().splitlines()[-1]);print('$pat','$tag',d['ms_per_step'],d['roofline']['kernels_ms']['push_binned'],d.get('check'))"
}
for pat in exchange zipf matrix; do
  run base $pat GLINT_BIN_FULL_MIN=4294967295
  run fp4 $pat GLINT_BIN_FULL_MIN=4294967295 GLINT_FPART_BPC=4
  run pw1 $pat GLINT_BIN_FULL_MIN=4294967295 GLINT_PART_WPC=1
done
