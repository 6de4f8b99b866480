#!/bin/bash
# Round 4: numeric small bins on the main stream too (CBG_SIDE=0) vs the default (side)
set -o pipefail
out=gpurun_out/bb
mkdir -p $out
for r in 1 2; do
  for f in def 0; do
    e=X=1; [ $f = 0 ] && e=CBG_SIDE=0
    env $e timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 1 > $out/b_${f}_$r.json 2>>$out/err.log || exit 1
    python3 -c "import json;d=json.load(open('$out/b_${f}_$r.json'));print('s22 round $r side=$f', round(d['ms_per_step'],2), 'ms')"
  done
done
