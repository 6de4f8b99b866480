#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "panel_groups or tall_matrix or scale24 or rank_tiles" > gpurun_out/r03c_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03c_tests.log; [ $rc -eq 0 ] || exit $rc
for glm in ${GLMS:-4 6}; do
  CBG_GROUP_LOG_MAX=$glm timeout -k 10 300 python bench.py --no-cpu-baseline --scale 24 --steps ${STEPS:-3} > gpurun_out/s24_g$glm.json 2> gpurun_out/s24_g$glm.err || { tail -5 gpurun_out/s24_g$glm.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/s24_g$glm.json'));print('s24 glm=$glm', round(d['value']/1e9,2),'G',round(d['ms_per_step'],1),'ms frac',round(d['roofline']['frac'],3), d['config']['phases'])"
done
