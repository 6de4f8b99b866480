#!/bin/bash
# Round 4: flops block starts, scan totals in-kernel, thin sort after the big
# launches, ESC bins at 2 products per lane (CBG_ESC_NPL=2): parity subset
# (both ESC settings), GalerkinNew scale 22 and the scale-22 bench vs the
# previous commit's build (build/variants/prev)
set -o pipefail
out=gpurun_out/h
mkdir -p $out
K="esc or galerkin or thin or restriction or wave or local_digest or random_values_scale20 or phased_scale22 or auto_phases or flops"
timeout -k 10 900 python -u -m pytest tests/test_gpu_local.py -x -q --timeout 300 --timeout-method thread -k "$K" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
CBG_ESC_NPL=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_local.py -x -q --timeout 300 --timeout-method thread -k "esc or galerkin or thin or local_digest" > $out/tests2.log 2>&1 || { tail -30 $out/tests2.log; exit 1; }
tail -1 $out/tests2.log
for r in 1 2; do
  for v in prev tree npl2; do
    lib=combblas-spmm-test_amd/libcbg.so; [ $v = prev ] && lib=build/variants/prev/libcbg.so
    e=1; [ $v = npl2 ] && e=2
    CBG_ESC_NPL=$e CBG_LIB=$lib timeout -k 10 200 python tools/galerkin.py --scale 22 --iters 5 --only-full > $out/gal_${v}_$r.json 2>>$out/err.log || exit 1
    python3 -c "import json;d=json.load(open('$out/gal_${v}_$r.json'));print('galerkin round $r $v', round(d['full_restriction_s']*1e3,3), 'ms')"
  done
done
for v in prev tree npl2; do
  lib=combblas-spmm-test_amd/libcbg.so; [ $v = prev ] && lib=build/variants/prev/libcbg.so
  e=1; [ $v = npl2 ] && e=2
  CBG_ESC_NPL=$e CBG_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 1 > $out/b_$v.json 2>>$out/err.log || exit 1
  python3 -c "import json;d=json.load(open('$out/b_$v.json'));print('s22', '$v', round(d['ms_per_step'],2), 'ms')"
done
