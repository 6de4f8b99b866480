#!/bin/bash
# Galerkin scale-22 kernel profile (one rank) + the s22 bench at 2 forced phases
set -o pipefail
mkdir -p gpurun_out/gal
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gal/prof -o k -- python3 tools/galerkin.py --scale 22 --iters 3 > gpurun_out/gal/run.json 2> gpurun_out/gal/run.err || { tail -5 gpurun_out/gal/run.err; exit 1; }
tail -1 gpurun_out/gal/run.json | head -c 400; echo
f=$(find gpurun_out/gal/prof -name "k_kernel_stats.csv" | head -1)
python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:25]:
    print('%8.3f ms %5s calls avg %7.3f  %s'%(float(r['TotalDurationNs'])/1e6, r['Calls'], float(r['AverageNs'])/1e6, r['Name'][:90]))
"
timeout -k 10 300 python bench.py --no-cpu-baseline --phases 2 --steps 3 > gpurun_out/ph2.json 2> gpurun_out/ph2.err || { tail -5 gpurun_out/ph2.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/ph2.json'));print('phases2', round(d['value']/1e9,2),'G',round(d['ms_per_step'],1),'ms', d['timing']['step_ms'])"
