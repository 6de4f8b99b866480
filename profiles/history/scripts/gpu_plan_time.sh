#!/bin/bash
# phase-plan cost at scale 22 on one GPU (CBG_DEBUG_PLAN marks) + the sym ablation
set -o pipefail
mkdir -p gpurun_out
CBG_DEBUG_PLAN=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 > gpurun_out/plan_bench.json 2> gpurun_out/plan_bench.err || { tail -20 gpurun_out/plan_bench.err; exit 1; }
grep "cbg plan" gpurun_out/plan_bench.err | tail -6
python3 -c "import json;d=json.load(open('gpurun_out/plan_bench.json'));print(round(d['value']/1e9,2),'G',round(d['ms_per_step'],1),'ms', d['roofline']['ms_avg'], d['config']['phase_plan']['plan_ms_per_step'])"
bash tools/gpu_sym_ablate.sh
