#!/bin/bash
# Round 4: CBG_SIDE 2 (symbolic small bins on the main stream) vs 3 at scales 18 / 24 and GalerkinNew
set -o pipefail
out=gpurun_out/z
mkdir -p $out
for f in 2 3; do
  CBG_SIDE=$f timeout -k 10 300 python bench.py --no-cpu-baseline --scale 18 --steps 30 --warmup 3 > $out/s18_$f.json 2>>$out/err.log || exit 1
  python3 -c "import json;d=json.load(open('$out/s18_$f.json'));print('s18 side=$f', round(d['ms_per_step'],3), 'ms')"
done
for r in 1 2; do
  for f in 2 3; do
    CBG_SIDE=$f timeout -k 10 200 python tools/galerkin.py --scale 22 --iters 5 --only-full > $out/gal_${f}_$r.json 2>>$out/err.log || exit 1
    python3 -c "import json;d=json.load(open('$out/gal_${f}_$r.json'));print('galerkin round $r side=$f', round(d['full_restriction_s']*1e3,3), 'ms')"
  done
done
for f in 2 3; do
  CBG_SIDE=$f timeout -k 10 400 python bench.py --no-cpu-baseline --scale 24 --steps 2 --warmup 1 > $out/s24_$f.json 2>>$out/err.log || exit 1
  python3 -c "import json;d=json.load(open('$out/s24_$f.json'));print('s24 side=$f', round(d['ms_per_step'],1), 'ms')"
done
