#!/bin/bash
# Round 4: inline A column records for the small-column / thin passes (CBG_AINL)
# -- parity subset, GalerkinNew scale 22 on / off (2 rounds), the scale-22 bench
set -o pipefail
out=gpurun_out/m
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_local.py -x -q --timeout 300 --timeout-method thread -k "esc or galerkin or thin or local_digest or restriction" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for r in 1 2; do
  for f in 1 0; do
    CBG_AINL=$f timeout -k 10 200 python tools/galerkin.py --scale 22 --iters 5 --only-full > $out/gal_${f}_$r.json 2>>$out/err.log || exit 1
    python3 -c "import json;d=json.load(open('$out/gal_${f}_$r.json'));print('galerkin round $r ainl=$f', round(d['full_restriction_s']*1e3,3), 'ms')"
  done
done
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 1 > $out/b.json 2>>$out/err.log || exit 1
python3 -c "import json;d=json.load(open('$out/b.json'));print('s22', round(d['ms_per_step'],2), 'ms')"
