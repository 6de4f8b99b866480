#!/bin/bash
# per-rank tile product of a scale-22 grid through the PANEL SUMMA on a one-rank grid,
# B in pipeline pieces (CBG_PIPELINE): compute cost of the pipelining (rank 0)
set -o pipefail
mkdir -p gpurun_out
for g in 4x2 2x2; do
  for pl in 1 1/8 1/4 2 4; do
    CBG_PIPELINE=$pl timeout -k 10 200 python tools/tile_totals.py --scale 22 --grid $g --ranks 0 --reps 3 --summa > gpurun_out/tp.json 2>> gpurun_out/tp.err || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/tp.json').readline());print('$g pipeline $pl', round(d['s']*1e3,2), 'ms', round(d['nnzC_per_s']/1e9,2), 'G/s')"
  done
done
