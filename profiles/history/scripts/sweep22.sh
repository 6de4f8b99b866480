#!/bin/bash
# Same-box comparison of libcbg variants on the default bench (scale 22, one GPU, 4 phases) and scale 18.
set -e -o pipefail
out=$1; shift
mkdir -p $out
for v in "$@"; do
  if [ "$v" = default ]; then lib=""; else lib=$PWD/build/variants/$v/libcbg.so; fi
  CBG_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 > $out/$v.s22.json
  echo "$v s22p4 $(python3 -c "import json; d=json.load(open('$out/$v.s22.json')); print('%.2f G/s %.1f ms' % (d['value']/1e9, d['ms_per_step']))")"
  CBG_LIB=$lib timeout -k 10 120 python3 bench.py --no-cpu-baseline --scale 18 --steps 5 > $out/$v.s18.json
  echo "$v s18 $(python3 -c "import json; d=json.load(open('$out/$v.s18.json')); print('%.2f G/s %.2f ms' % (d['value']/1e9, d['ms_per_step']))")"
  CBG_LIB=$lib timeout -k 10 200 python3 tools/tile_totals.py --scale 22 --grid 4x2 --ranks 0 --reps 2 > $out/$v.t42.json
  echo "$v s22 4x2 tile $(python3 -c "import json; d=json.loads(open('$out/$v.t42.json').readline()); print('%.1f ms' % (d['s']*1e3))")"
done
