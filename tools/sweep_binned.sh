# binned-push knob sweep (tuning only): ms per push of the binned bench patterns
# usage: bash tools/sweep_binned.sh "tag:ENV=V,ENV2=V2" ...   (tag "base" = no overrides)
set -e
run() {  # tag pattern env...
  tag=$1; pat=$2; shift 2
  env "$@" timeout -k 10 120 python bench.py --pattern $pat --steps 20 --warmup 3 > gpurun_out/sw_${pat}_${tag}.json 2>gpurun_out/sw_${pat}_${tag}.err
  python -c "import json;d=json.loads(open('gpurun_out/sw_${pat}_${tag}.json').read().strip().splitlines()[-1]);print('$pat','$tag',d['ms_per_step'],d['roofline']['kernels_ms']['push_binned'],d.get('check'))"
}
for pat in exchange zipf matrix; do
  for v in "$@"; do
    tag=${v%%:*}; envs=${v#*:}; [ "$envs" = "$v" ] && envs=""
    run $tag $pat GLINT_SWEEP=1 ${envs//,/ }
  done
done
