#!/bin/bash
# Same-box A/B of libcbg builds (tools/gpu_libab.sh): bench.py (scale ${SCALE:-22}, ${STEPS:-5} steps) for every name in
# $VARIANTS (build/variants/<name>/libcbg.so; "tree" = the in-tree build), ${ROUNDS:-2} rounds interleaved.
# Optional: TESTS_K="expr" runs that GPU test selection (pytest -k) on the in-tree build first.
set -o pipefail
out=gpurun_out/ab
mkdir -p $out
if [ -n "$TESTS_K" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_local.py -x -q --timeout 300 --timeout-method thread -k "$TESTS_K" \
    > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
  tail -1 $out/tests.log
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    lib=build/variants/$v/libcbg.so; [ $v = tree ] && lib=combblas-spmm-test_amd/libcbg.so
    CBG_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-5} --warmup 1 \
      ${SCALE:+--scale $SCALE} ${BENCH_ARGS} > $out/${v}_$r.json 2>>$out/err.log || exit 1
    python3 -c "import json;d=json.load(open('$out/${v}_$r.json'));print('round $r $v', round(d['value']/1e9,2), 'G nnz/s', round(d['ms_per_step'],2), 'ms')"
  done
done
