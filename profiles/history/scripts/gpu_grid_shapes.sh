#!/bin/bash
# per-rank tile time of scale-22 grids of 8 and 4 ranks (rank 0 and the last rank), one GPU, no pipelining
set -o pipefail
mkdir -p gpurun_out
for g in 8x1 4x2 2x4 4x1 2x2 1x4; do
  n=$(( ${g%x*} * ${g#*x} ))
  CBG_PIPELINE=1 timeout -k 10 300 python tools/tile_totals.py --scale 22 --grid $g --ranks 0,$((n-1)) --reps 2 --summa > gpurun_out/gs.json 2>> gpurun_out/gs.err || exit 1
  python3 -c "
import json
for l in open('gpurun_out/gs.json'):
    d=json.loads(l); print('$g rank', d['rank'], round(d['s']*1e3,2), 'ms', round(d['nnzC_per_s']/1e9,2), 'G/s')"
done
