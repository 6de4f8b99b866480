#!/bin/bash
# Round 4: columns of 513-1024 flops by expand-sort-compress at 16 products per
# lane (CBG_FUSED_LAST=10) -- parity subset with it, GalerkinNew scale 22 and the
# scale-22 bench at 9 / 10
set -o pipefail
out=gpurun_out/o
mkdir -p $out
CBG_FUSED_LAST=10 timeout -k 10 900 python -u -m pytest tests/test_gpu_local.py -x -q --timeout 300 --timeout-method thread -k "esc or galerkin or thin or local_digest or phased_scale22 or random_values_scale20" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for r in 1 2; do
  for f in 10 9; do
    CBG_FUSED_LAST=$f timeout -k 10 200 python tools/galerkin.py --scale 22 --iters 5 --only-full > $out/gal_${f}_$r.json 2>>$out/err.log || exit 1
    python3 -c "import json;d=json.load(open('$out/gal_${f}_$r.json'));print('galerkin round $r last=$f', round(d['full_restriction_s']*1e3,3), 'ms')"
  done
done
for f in 10 9; do
  CBG_FUSED_LAST=$f timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 1 > $out/b_$f.json 2>>$out/err.log || exit 1
  python3 -c "import json;d=json.load(open('$out/b_$f.json'));print('s22 last=$f', round(d['ms_per_step'],2), 'ms')"
done
