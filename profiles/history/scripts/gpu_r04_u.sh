#!/bin/bash
# Round 4: dominant-run big columns by k_dom (CBG_DOM) -- parity subset, the
# scale-22 bench on / off (2 rounds), scale 24 on / off
set -o pipefail
out=gpurun_out/u
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_local.py -x -q --timeout 300 --timeout-method thread -k "local_digest or phased_scale22 or random_values_scale20 or golden or largeseq or single or tall or panel" > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for r in 1 2; do
  for f in 1 0; do
    CBG_DOM=$f timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 1 > $out/b_${f}_$r.json 2>>$out/err.log || exit 1
    python3 -c "import json;d=json.load(open('$out/b_${f}_$r.json'));print('s22 round $r dom=$f', round(d['ms_per_step'],2), 'ms')"
  done
done
for f in 1 0; do
  CBG_DOM=$f timeout -k 10 400 python bench.py --no-cpu-baseline --scale 24 --steps 2 --warmup 1 > $out/s24_$f.json 2>>$out/err.log || exit 1
  python3 -c "import json;d=json.load(open('$out/s24_$f.json'));print('s24 dom=$f', round(d['ms_per_step'],1), 'ms')"
done
