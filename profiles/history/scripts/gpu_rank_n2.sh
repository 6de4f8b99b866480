#!/bin/bash
# N=2 at scale 22 (2x1 grid, one phase, C tile of ~149 GB resident) per rank on one
# GPU, through the PANEL SUMMA with the pipelined cut (CBG_PIPELINE=1/8) and without
set -o pipefail
mkdir -p gpurun_out
for pl in 1/8 1; do
  CBG_PIPELINE=$pl timeout -k 10 300 python tools/tile_totals.py --scale 22 --grid 2x1 --reps 2 --summa > gpurun_out/n2.json 2>> gpurun_out/n2.err || { tail -5 gpurun_out/n2.err; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/n2.json'):
    d = json.loads(l)
    if 'rank' in d: print('2x1 rank', d['rank'], 'pipeline $pl', round(d['s']*1e3, 2), 'ms', d['nnz_C'], 'nnz', round(d['nnzC_per_s']/1e9, 2), 'G/s')"
done
