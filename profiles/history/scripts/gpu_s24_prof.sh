#!/bin/bash
# scale-24 one-GPU step under a kernel trace: per-kernel totals of one timed step
set -o pipefail
mkdir -p gpurun_out/s24
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s24/prof -o k -- python3 bench.py --scale 24 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/s24/run.json 2> gpurun_out/s24/run.err || { tail -5 gpurun_out/s24/run.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/s24/run.json'));print('s24', round(d['value']/1e9,2), 'G', round(d['ms_per_step'],1), 'ms', d['config']['phases'], round(d['roofline']['frac'],3))"
f=$(find gpurun_out/s24/prof -name "k_kernel_stats.csv" | head -1)
python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:22]:
    print('%9.1f ms %6s calls avg %8.3f  %s'%(float(r['TotalDurationNs'])/1e6, r['Calls'], float(r['AverageNs'])/1e6, r['Name'][:90]))
"
