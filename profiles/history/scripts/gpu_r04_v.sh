#!/bin/bash
# Round 4: inline A records in the block numeric hash of the column bins
# (CBG_AINL_NUM) -- Galerkin parity tests, GalerkinNew scale 22 on / off (3 rounds)
set -o pipefail
out=gpurun_out/v
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_local.py -x -q --timeout 300 --timeout-method thread -k "galerkin or restriction or esc" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for r in 1 2 3; do
  for f in 1 0; do
    CBG_AINL_NUM=$f timeout -k 10 200 python tools/galerkin.py --scale 22 --iters 5 --only-full > $out/gal_${f}_$r.json 2>>$out/err.log || exit 1
    python3 -c "import json;d=json.load(open('$out/gal_${f}_$r.json'));print('galerkin round $r ainl_num=$f', round(d['full_restriction_s']*1e3,3), 'ms')"
  done
done
