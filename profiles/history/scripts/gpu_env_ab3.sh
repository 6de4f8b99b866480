#!/bin/bash
# parity (local GPU tests, default env), then the bench under several env settings, twice, at 22 and 18:
#   ENVS=("A=1" "B=2") style list in $ENV_LIST separated by ';'
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_local.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tm.log 2>&1 || { tail -30 gpurun_out/tm.log; exit 1; }
tail -1 gpurun_out/tm.log
IFS=';' read -ra L <<< "$ENV_LIST"
for sc in 22 22 18 18; do
  for i in "${!L[@]}"; do
    e=${L[$i]}
    env $e timeout -k 10 200 python bench.py --no-cpu-baseline --scale $sc > gpurun_out/e_$i.json 2>> gpurun_out/e.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/e_$i.json'));print('s$sc [$e]', round(d['value']/1e9,2), 'G nnz/s', round(d['ms_per_step'],3), 'ms')"
  done
done
