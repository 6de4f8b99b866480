#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 > gpurun_out/d_bench.json 2> gpurun_out/d_bench.err || { tail -5 gpurun_out/d_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/d_bench.json'));p=d['config']['phase_plan'];print('s22', round(d['value']/1e9,2),'G',round(d['ms_per_step'],1),'ms', d['config']['phases'], p['plan_ms_per_step'], p['nnz_est_rank0'], p['oom_splits'])"
CBG_DBG=48 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 0 --phases 2 > /dev/null 2> gpurun_out/d_stats.err || { tail -5 gpurun_out/d_stats.err; exit 1; }
grep "cbg" gpurun_out/d_stats.err | tail -8
timeout -k 10 300 python bench.py --no-cpu-baseline --scale 24 --steps 3 > gpurun_out/d_s24.json 2> gpurun_out/d_s24.err || { tail -5 gpurun_out/d_s24.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/d_s24.json'));p=d['config']['phase_plan'];print('s24', round(d['value']/1e9,2),'G',round(d['ms_per_step'],1),'ms', d['config']['phases'], p['oom_splits'], d['timing']['step_ms'])"
