#!/bin/bash
# Round profile bundle on the GPU box: the default bench line (with its CPU baseline),
# scale-22 kernel stats + FETCH/WRITE traffic (2 phases, the bench's plan), scale 18 the same
# (C resident), then tools/profile_collect.sh here copies the summaries into profiles/.
#   R=r05 tools/gpu_profiles_round.sh
set -o pipefail
R=${R:-r05}
mkdir -p gpurun_out/prof_bundle
timeout -k 10 900 python bench.py > gpurun_out/prof_bundle/bench_default.json 2> gpurun_out/prof_bundle/bench_default.err || { tail -20 gpurun_out/prof_bundle/bench_default.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/prof_bundle/bench_default.json').read().strip().splitlines()[-1]);print('default', round(d['ms_per_step'],2), 'ms', round(d['roofline']['frac'],4), 'f64', round(d['roofline'].get('frac_f64_values',0),4), 'cpu', d.get('cpu_baseline',{}).get('value'))"
STEPS=3 bash tools/profile_round.sh $R 22 2 || exit 1
STEPS=10 bash tools/profile_round.sh $R 18 1 || exit 1
