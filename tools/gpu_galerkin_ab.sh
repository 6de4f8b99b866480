#!/bin/bash
# Same-box A/B of GalerkinNew (scale ${SCALE:-22}, full restriction, 5 iterations) under
# several env settings, ROUNDS interleaved rounds:
#   ENVS="name1:VAR=x,VAR2=y name2:" [ROUNDS=2] tools/gpu_galerkin_ab.sh
set -o pipefail
out=gpurun_out/${OUT:-galab}
mkdir -p $out
for r in $(seq 1 ${ROUNDS:-2}); do
  for e in $ENVS; do
    name=${e%%:*}; vars=${e#*:}
    env $(echo $vars | tr ',' ' ') timeout -k 10 200 python tools/galerkin.py --scale ${SCALE:-22} --iters 5 --only-full \
      > $out/${name}_$r.json 2>>$out/err.log || { tail -20 $out/err.log; exit 1; }
    python3 -c "import json;d=json.load(open('$out/${name}_$r.json'));print('round $r $name', round(d['full_restriction_s']*1e3,3), 'ms', 'correct', d['splitting_correct'])"
  done
done
