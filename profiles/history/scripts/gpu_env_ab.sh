#!/bin/bash
# same-box A/B of an environment setting: tools/gpu_env_ab.sh "VAR=value" [scales...]
set -o pipefail
mkdir -p gpurun_out
envset=$1; shift
for sc in ${@:-22 18}; do
  for rep in 1 2; do
    for mode in base alt; do
      if [ $mode = alt ]; then e="env $envset"; else e=""; fi
      st=5; [ $sc -le 18 ] && st=30
      $e timeout -k 10 300 python bench.py --no-cpu-baseline --scale $sc --steps $st > gpurun_out/ab.json 2>>gpurun_out/ab.err || exit 1
      python3 -c "import json;d=json.load(open('gpurun_out/ab.json'));print('s$sc $mode', round(d['value']/1e9,2), 'G nnz/s', round(d['ms_per_step'],3), 'ms')"
    done
  done
done
