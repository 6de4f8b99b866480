#!/bin/bash
# Round 4: small-column bins' stream placement re-checked with the copy paths (CBG_SIDE 3 / 1 / 2)
set -o pipefail
out=gpurun_out/y
mkdir -p $out
for r in 1 2; do
  for f in 3 1 2; do
    CBG_SIDE=$f timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 1 > $out/b_${f}_$r.json 2>>$out/err.log || exit 1
    python3 -c "import json;d=json.load(open('$out/b_${f}_$r.json'));print('s22 round $r side=$f', round(d['ms_per_step'],2), 'ms')"
  done
done
