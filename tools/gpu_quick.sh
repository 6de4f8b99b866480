#!/bin/bash
# quick GPU check: local GPU tests, bench at scale 22 and 18, phase breakdown at 22 (CBG_DBG=16)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_local.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tq.log 2>&1 || { tail -30 gpurun_out/tq.log; exit 1; }
tail -1 gpurun_out/tq.log
for sc in 22 18; do
  st=5; [ $sc -eq 18 ] && st=30
  timeout -k 10 200 python bench.py --no-cpu-baseline --scale $sc --steps $st > gpurun_out/q_s$sc.json 2> gpurun_out/q.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/q_s$sc.json'));print('s$sc', round(d['value']/1e9,2), 'G nnz/s', round(d['ms_per_step'],3), 'ms', round(d['roofline']['frac'],3), 'ms_avg', round(d['roofline']['ms_avg'],3))"
done
CBG_DBG=16 timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> gpurun_out/q_dbg.err || exit 1
tail -2 gpurun_out/q_dbg.err
