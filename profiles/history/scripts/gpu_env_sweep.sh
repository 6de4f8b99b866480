#!/bin/bash
# bench at one scale under several env settings: SCALE=22 tools/gpu_env_sweep.sh "" "X=1" "X=2 Y=3" ...
# (run on the GPU box from the repo root; lines in gpurun_out/sweep_*.json)
set -o pipefail
mkdir -p gpurun_out
sc=${SCALE:-22}
i=0
for envs in "$@"; do
  env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --scale $sc > gpurun_out/sweep_$i.json 2>> gpurun_out/sweep.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/sweep_$i.json'));print('s$sc [$envs]', round(d['value']/1e9,2), 'G nnz/s', round(d['ms_per_step'],2), 'ms', round(d['roofline']['frac'],3))"
  i=$((i+1))
done
