#!/bin/bash
# Round 4: adaptive symbolic stream vs CBG_SIDE=3 on scale 18 and GalerkinNew (3 rounds)
set -o pipefail
out=gpurun_out/ab2
mkdir -p $out
for r in 1 2 3; do
  for f in adapt side3; do
    e=X=1; [ $f = side3 ] && e=CBG_SIDE=3
    env $e timeout -k 10 200 python tools/galerkin.py --scale 22 --iters 5 --only-full > $out/gal_${f}_$r.json 2>>$out/err.log || exit 1
    python3 -c "import json;d=json.load(open('$out/gal_${f}_$r.json'));print('galerkin round $r $f', round(d['full_restriction_s']*1e3,3), 'ms')"
    env $e timeout -k 10 300 python bench.py --no-cpu-baseline --scale 18 --steps 30 --warmup 3 > $out/s18_${f}_$r.json 2>>$out/err.log || exit 1
    python3 -c "import json;d=json.load(open('$out/s18_${f}_$r.json'));print('s18 round $r $f', round(d['ms_per_step'],3), 'ms')"
  done
done
