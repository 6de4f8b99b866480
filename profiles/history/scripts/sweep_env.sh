#!/bin/bash
# GPU sweep of env settings: tools/sweep_env.sh out_dir "VAR=a VAR2=b" ...  (scales 18, 20 and a scale-22 2x4 tile)
set -e -o pipefail
out=$1; shift
mkdir -p $out
for e in "$@"; do
  tag=$(echo "$e" | tr ' =' '_-')
  for sc in 18 20; do
    env $e timeout -k 10 120 python3 bench.py --no-cpu-baseline --scale $sc --steps 5 > $out/$tag.s$sc.json
    echo "[$e] s$sc $(python3 -c "import json; d=json.load(open('$out/$tag.s$sc.json')); print('%.2f G/s %.2f ms' % (d['value']/1e9, d['ms_per_step']))")"
  done
  env $e timeout -k 10 200 python3 tools/tile_totals.py --scale 22 --grid 2x4 --ranks 0 --reps 2 > $out/$tag.s22.json
  echo "[$e] s22 2x4 tile $(python3 -c "import json; d=json.loads(open('$out/$tag.s22.json').readline()); print('%.1f ms' % (d['s']*1e3))")"
done
