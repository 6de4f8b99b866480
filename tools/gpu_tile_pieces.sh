#!/bin/bash
# per-rank tile product of a scale-22 grid with B in 1/2/4 column pieces (rank 0)
set -o pipefail
mkdir -p gpurun_out
for g in 2x1 2x2 4x2; do
  for pc in 1 2 4; do
    timeout -k 10 200 python tools/tile_totals.py --scale 22 --grid $g --ranks 0 --reps 2 --pieces $pc > gpurun_out/tp_${g}_$pc.json 2>> gpurun_out/tp.err || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/tp_${g}_$pc.json').readline());print('$g pieces $pc', round(d['s']*1e3,1), 'ms', round(d['nnzC_per_s']/1e9,2), 'G/s')"
  done
done
