#!/bin/bash
# Same-box A/B of environment settings on ONE build (the in-tree libcbg.so):
#   TESTS_K="expr" (optional) runs that pytest -k selection of test_gpu_local.py first
#   (under TESTS_ENV="VAR=x,VAR2=y" when given);
#   ENVS="name1:VAR=x,VAR2=y name2:VAR=z base:" benches each setting ROUNDS times (interleaved),
#   bench.py --scale ${SCALE:-22} --steps ${STEPS:-5} ${BENCH_ARGS}; DBG_ENV (optional) = the
#   setting whose CBG_DBG=48 phase/stat lines are printed at the end.
set -o pipefail
out=gpurun_out/${OUT:-abenv}
mkdir -p $out
if [ -n "$TESTS_K" ]; then
  env $(echo $TESTS_ENV | tr ',' ' ') timeout -k 10 ${TESTS_TIMEOUT:-600} python -u -m pytest tests/test_gpu_local.py -x -q --timeout 300 --timeout-method thread \
    -k "$TESTS_K" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
  tail -1 $out/tests.log
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for e in $ENVS; do
    name=${e%%:*}; vars=${e#*:}
    env $(echo $vars | tr ',' ' ') timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-5} --warmup 1 \
      --scale ${SCALE:-22} ${BENCH_ARGS} > $out/${name}_$r.json 2>>$out/err.log || { tail -20 $out/err.log; exit 1; }
    python3 -c "import json;d=json.load(open('$out/${name}_$r.json'));print('round $r $name', round(d['value']/1e9,2), 'G nnz/s', round(d['ms_per_step'],2), 'ms', 'frac', round(d['roofline']['frac'],4))"
  done
done
if [ -n "$DBG_ENV" ]; then
  env $(echo $DBG_ENV | tr ',' ' ') CBG_DBG=48 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 0 \
    --scale ${SCALE:-22} ${BENCH_ARGS} > $out/dbg.json 2> $out/dbg.err || { tail -20 $out/dbg.err; exit 1; }
  grep '\[cbg' $out/dbg.err | tail -4
fi
