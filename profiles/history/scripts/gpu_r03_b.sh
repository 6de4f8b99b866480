#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
CBG_DEBUG_PLAN=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 > gpurun_out/plan_bench.json 2> gpurun_out/plan_bench.err || { tail -20 gpurun_out/plan_bench.err; exit 1; }
grep "cbg plan" gpurun_out/plan_bench.err | tail -4
python3 -c "import json;d=json.load(open('gpurun_out/plan_bench.json'));print(round(d['value']/1e9,2),'G',round(d['ms_per_step'],1),'ms', round(d['roofline']['ms_avg'],1), d['config']['phase_plan']['plan_ms_per_step'])"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "auto_phases or phase_split or rccl_multirank or (summa_multiprocess and rmat)" > gpurun_out/r03b_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03b_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_overlap_trace.sh 20
