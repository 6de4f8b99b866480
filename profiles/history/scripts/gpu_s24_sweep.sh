#!/bin/bash
# scale-24 one-GPU environment sweep: tools/gpu_s24_sweep.sh "VAR=v ..." ...  ("" = defaults)
set -o pipefail
mkdir -p gpurun_out
for envset in "$@"; do
  timeout -k 10 300 env $envset python bench.py --no-cpu-baseline --scale 24 --steps 3 > gpurun_out/s24sw.json 2>>gpurun_out/s24sw.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/s24sw.json'));print('s24 [$envset]', round(d['value']/1e9,2), 'G nnz/s', round(d['ms_per_step'],1), 'ms', d['timing']['step_ms'], round(d['roofline']['frac'],3))"
done
