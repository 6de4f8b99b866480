#!/bin/bash
# Round 4: hash-slab classes on the side stream at scale 24 and 22 (CBG_SIDE_HASH bit mask)
set -o pipefail
out=gpurun_out/r
mkdir -p $out
run() {  # name scale steps env...
  local name=$1 sc=$2 st=$3; shift 3
  env "$@" timeout -k 10 400 python bench.py --no-cpu-baseline --scale $sc --steps $st --warmup 1 > $out/$name.json 2>>$out/err.log || exit 1
  python3 -c "import json;d=json.load(open('$out/$name.json'));print('$name', round(d['ms_per_step'],1), 'ms')"
}
for r in 1 2; do
  run s24_base_$r 24 2 X=1
  run s24_side_all_$r 24 2 CBG_SIDE_HASH=511
  run s24_side_big_$r 24 2 CBG_SIDE_HASH=448
done
