#!/bin/bash
# Round 4 knob re-sweep on the current kernels (scale 22, 5 steps): env knobs
# and build variants, 2 interleaved rounds
set -o pipefail
out=gpurun_out/n
mkdir -p $out
run() {  # name, lib, env...
  local name=$1 lib=$2; shift 2
  env "$@" CBG_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 1 > $out/$name.json 2>>$out/err.log || exit 1
  python3 -c "import json;d=json.load(open('$out/$name.json'));print('$name', round(d['ms_per_step'],2), 'ms')"
}
T=combblas-spmm-test_amd/libcbg.so
for r in 1 2; do
  run base_$r $T X=1
  run gp2560_$r $T CBG_GROUP_PRODUCTS=2560
  run gp3584_$r $T CBG_GROUP_PRODUCTS=3584
  run big3072_$r $T CBG_BIG_FLOPS=3072
  run bud64_$r $T CBG_BITMAP_BUDGET_GB=64
  run wu8_$r build/variants/wu8/libcbg.so X=1
  run wu128_$r build/variants/wu128/libcbg.so X=1
done
