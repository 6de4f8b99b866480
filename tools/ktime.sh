#!/bin/bash
# Kernel-time table of one scale-22 2x4 rank-0 tile multiply under env settings (diagnostics).
# usage: tools/ktime.sh out_dir "ENV=.." ...
set -e -o pipefail
out=$1; shift
export TMPDIR=/tmp
mkdir -p $out
for e in "$@"; do
  tag=$(echo "$e" | tr ' =' '_-')
  env $e timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$tag -o k -- python3 tools/tile_totals.py --scale ${SCALE:-22} --grid ${GRID:-2x4} --ranks 0 --reps 2 > $out/$tag.log 2>&1
done
