#!/bin/bash
# Round 4: adaptive stream of the small symbolic bins (default) vs CBG_SIDE=3 (always side)
set -o pipefail
out=gpurun_out/aa
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_local.py -x -q --timeout 300 --timeout-method thread -k "local_digest or phased_scale22 or galerkin or single" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
run() {  # name, args, env...
  local name=$1 args=$2; shift 2
  env "$@" timeout -k 10 400 python bench.py --no-cpu-baseline $args > $out/$name.json 2>>$out/err.log || exit 1
  python3 -c "import json;d=json.load(open('$out/$name.json'));print('$name', round(d['ms_per_step'],3), 'ms')"
}
for r in 1 2; do
  run s22_adapt_$r "--steps 5 --warmup 1" X=1
  run s22_side3_$r "--steps 5 --warmup 1" CBG_SIDE=3
done
run s18_adapt "--scale 18 --steps 30 --warmup 3" X=1
run s18_side3 "--scale 18 --steps 30 --warmup 3" CBG_SIDE=3
for f in adapt side3; do
  e=X=1; [ $f = side3 ] && e=CBG_SIDE=3
  env $e timeout -k 10 200 python tools/galerkin.py --scale 22 --iters 5 --only-full > $out/gal_$f.json 2>>$out/err.log || exit 1
  python3 -c "import json;d=json.load(open('$out/gal_$f.json'));print('galerkin $f', round(d['full_restriction_s']*1e3,3), 'ms')"
done
run s24_adapt "--scale 24 --steps 2 --warmup 1" X=1
