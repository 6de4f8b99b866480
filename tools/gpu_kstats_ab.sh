#!/bin/bash
# kernel-time tables of the bench under several env settings, same box:
#   KSETS="name1:VAR=x,VAR2=y name2:" [STEPS=2] tools/gpu_kstats_ab.sh
set -o pipefail
for e in $KSETS; do
  name=${e%%:*}; vars=${e#*:}
  echo "== $name ($vars)"
  OUT=ab_$name ENVS="$vars" STEPS=${STEPS:-2} TOP=${TOP:-12} bash tools/gpu_kstats.sh || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/ks_ab_$name/bench.json'));print('bench', round(d['ms_per_step'],2), 'ms')"
done
