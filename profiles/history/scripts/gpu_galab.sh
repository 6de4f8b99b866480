#!/bin/bash
# Same-box A/B of libcbg builds on GalerkinNew (full restriction, scale ${SCALE:-22}):
# $VARIANTS (build/variants/<name>/libcbg.so; "tree" = in-tree), ${ROUNDS:-3} rounds
set -o pipefail
out=gpurun_out/galab
mkdir -p $out
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in $VARIANTS; do
    lib=build/variants/$v/libcbg.so; [ $v = tree ] && lib=combblas-spmm-test_amd/libcbg.so
    CBG_LIB=$lib timeout -k 10 200 python tools/galerkin.py --scale ${SCALE:-22} --iters 5 --only-full > $out/${v}_$r.json 2>>$out/err.log || exit 1
    python3 -c "import json;d=json.load(open('$out/${v}_$r.json'));print('round $r $v', round(d['full_restriction_s']*1e3,3), 'ms')"
  done
done
