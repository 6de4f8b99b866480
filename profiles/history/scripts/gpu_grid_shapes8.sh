#!/bin/bash
# rank 0's local product (one GPU) for each 8-rank grid shape at scale 22
set -o pipefail
mkdir -p gpurun_out
for g in 4x2 2x4 8x1 1x8; do
  timeout -k 10 300 python tools/tile_totals.py --scale 22 --grid $g --ranks 0,$(( ${g%x*} * ${g#*x} - 1 )) --reps 3 > gpurun_out/gs.json 2>> gpurun_out/gs.err || { tail -5 gpurun_out/gs.err; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/gs.json'):
    d = json.loads(l)
    if 'rank' in d: print('$g rank', d['rank'], round(d['s']*1e3, 2), 'ms', round(d['nnzC_per_s']/1e9, 2), 'G/s')"
done
