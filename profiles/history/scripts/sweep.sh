#!/bin/bash
# GPU sweep of libcbg variants (tools/variants.sh): bench scales 18/20 + a scale-22 2x4 tile, one line each.
# usage: tools/sweep.sh out_dir variant... ("default" = the in-tree build)
set -e -o pipefail
out=$1; shift
mkdir -p $out
for v in "$@"; do
  if [ "$v" = default ]; then lib=""; else lib=$PWD/build/variants/$v/libcbg.so; fi
  for sc in 18 20; do
    CBG_LIB=$lib timeout -k 10 120 python3 bench.py --no-cpu-baseline --scale $sc --steps 5 > $out/$v.s$sc.json
    echo "$v s$sc $(python3 -c "import json,sys; d=json.load(open('$out/$v.s$sc.json')); print('%.2f G/s %.2f ms' % (d['value']/1e9, d['ms_per_step']))")"
  done
  if [ -z "$NO22" ]; then
    CBG_LIB=$lib timeout -k 10 200 python3 tools/tile_totals.py --scale 22 --grid 2x4 --ranks 0 --reps 2 > $out/$v.s22.json
    echo "$v s22 2x4 tile $(python3 -c "import json; d=json.loads(open('$out/$v.s22.json').readline()); print('%.1f ms' % (d['s']*1e3))")"
  fi
done
