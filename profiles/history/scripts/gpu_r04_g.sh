#!/bin/bash
# Round 4: VALU cross-lane sorts (CBG_XOR_DPP) -- helper check, the small-column /
# Galerkin parity tests, then GalerkinNew scale 22 and the scale-22 bench, A/B
# against the ds_bpermute build (build/variants/nodpp)
set -o pipefail
out=gpurun_out/g
mkdir -p $out
timeout -k 10 60 ./build/xor_check || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_local.py -x -q --timeout 300 --timeout-method thread \
  -k "esc or galerkin or thin or restriction or wave or local_digest or random_values_scale20" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for r in 1 2; do
  for v in tree nodpp; do
    lib=build/variants/$v/libcbg.so; [ $v = tree ] && lib=combblas-spmm-test_amd/libcbg.so
    CBG_LIB=$lib timeout -k 10 200 python tools/galerkin.py --scale 22 --iters 5 --only-full > $out/gal_${v}_$r.json 2>>$out/err.log || exit 1
    python3 -c "import json;d=json.load(open('$out/gal_${v}_$r.json'));print('galerkin round $r $v', round(d['full_restriction_s']*1e3,3), 'ms')"
  done
done
for v in tree nodpp; do
  lib=build/variants/$v/libcbg.so; [ $v = tree ] && lib=combblas-spmm-test_amd/libcbg.so
  CBG_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 1 > $out/b_$v.json 2>>$out/err.log || exit 1
  python3 -c "import json;d=json.load(open('$out/b_$v.json'));print('s22', '$v', round(d['ms_per_step'],2), 'ms')"
done
