#!/bin/bash
# k_sym_panel cost split: kernel times of a scale-22 rank tile (4x2 grid, rank 0) with
# CBG_DBG=0 / 1 (skip bitmap-pair products) / 64 (skip hash-pair products): results are
# WRONG under the ablations; only the kernel times are read
set -o pipefail
mkdir -p gpurun_out/abl
export TMPDIR=/tmp
for d in ${DBGS:-0 1 64}; do
  CBG_DBG=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abl/d$d -o k -- python3 tools/tile_totals.py --scale 22 --grid 4x2 --ranks 0 --reps 2 > gpurun_out/abl/d$d.log 2>&1 || { tail gpurun_out/abl/d$d.log; exit 1; }
  f=$(find gpurun_out/abl/d$d -name "k_kernel_stats.csv" | head -1)
  python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if 'k_sym_panel' in r['Name'] or 'k_num_slab<' in r['Name']:
        print('dbg=$d', r['Name'][:60], r['Calls'], round(float(r['TotalDurationNs'])/1e6,2),'ms total')
"
done
