#!/bin/bash
# Round 4: numeric launch order (CBG_SLAB_ORDER) at scale 22 (2 rounds) and 24
set -o pipefail
out=gpurun_out/w
mkdir -p $out
for r in 1 2; do
  for f in 1 0; do
    CBG_SLAB_ORDER=$f timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 1 > $out/b_${f}_$r.json 2>>$out/err.log || exit 1
    python3 -c "import json;d=json.load(open('$out/b_${f}_$r.json'));print('s22 round $r order=$f', round(d['ms_per_step'],2), 'ms')"
  done
done
for f in 1 0; do
  CBG_SLAB_ORDER=$f timeout -k 10 400 python bench.py --no-cpu-baseline --scale 24 --steps 2 --warmup 1 > $out/s24_$f.json 2>>$out/err.log || exit 1
  python3 -c "import json;d=json.load(open('$out/s24_$f.json'));print('s24 order=$f', round(d['ms_per_step'],1), 'ms')"
done
