#!/bin/bash
# A/B of an env knob on the bench: tools/gpu_ab.sh "<env A>" "<env B>" [scale...]
# (run on the GPU box from the repo root; lines in gpurun_out/ab_*.json)
set -o pipefail
mkdir -p gpurun_out
A=$1; B=$2; shift 2
for sc in "${@:-22}"; do
  for tag in A B; do
    envs=$([ $tag = A ] && echo "$A" || echo "$B")
    env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --scale $sc > gpurun_out/ab_${tag}_s$sc.json 2>> gpurun_out/ab.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/ab_${tag}_s$sc.json'));print('$tag s$sc [$envs]', round(d['value']/1e9,2), 'G nnz/s', round(d['ms_per_step'],2), 'ms', round(d['roofline']['frac'],3))"
  done
done
