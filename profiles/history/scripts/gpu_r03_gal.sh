#!/bin/bash
# round 3 small-column work: local GPU tests, Galerkin trace + plain timing, scale-22 / 18 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_local.py -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/tq.log 2>&1 || { tail -30 gpurun_out/tq.log; exit 1; }
tail -1 gpurun_out/tq.log
bash tools/gpu_galerkin_trace.sh || exit 1
[ -n "$NO_BENCH" ] && exit 0
for sc in 22 18; do
  st=5; [ $sc -eq 18 ] && st=30
  timeout -k 10 200 python bench.py --no-cpu-baseline --scale $sc --steps $st > gpurun_out/q_s$sc.json 2> gpurun_out/q.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/q_s$sc.json'));print('s$sc', round(d['value']/1e9,2), 'G nnz/s', round(d['ms_per_step'],3), 'ms', round(d['roofline']['frac'],3), 'ms_avg', round(d['roofline']['ms_avg'],3))"
done
