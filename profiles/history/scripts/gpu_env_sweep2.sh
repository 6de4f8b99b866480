#!/bin/bash
# same-box sweep of environment settings at one scale: tools/gpu_env_sweep2.sh SCALE "A=1" "B=2 C=3" ...
set -o pipefail
mkdir -p gpurun_out
sc=$1; shift
for rep in 1 2; do
  for envset in base "$@"; do
    if [ "$envset" = base ]; then e=""; else e="env $envset"; fi
    st=5; [ $sc -le 18 ] && st=30
    $e timeout -k 10 300 python bench.py --no-cpu-baseline --scale $sc --steps $st > gpurun_out/sw.json 2>>gpurun_out/sw.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/sw.json'));print('s$sc [$envset]', round(d['value']/1e9,2), 'G nnz/s', round(d['ms_per_step'],3), 'ms')"
  done
done
