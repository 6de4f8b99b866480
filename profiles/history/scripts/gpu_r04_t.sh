#!/bin/bash
# Round 4: big single-entry columns copied too (CBG_COPY1=2) -- parity subset with it,
# the scale-22 bench at 2 / 1 (2 rounds), scale 18
set -o pipefail
out=gpurun_out/t
mkdir -p $out
CBG_COPY1=2 timeout -k 10 900 python -u -m pytest tests/test_gpu_local.py -x -q --timeout 300 --timeout-method thread -k "local_digest or phased_scale22 or random or golden or largeseq or edge or panel" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for r in 1 2; do
  for f in 2 1; do
    CBG_COPY1=$f timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 1 > $out/b_${f}_$r.json 2>>$out/err.log || exit 1
    python3 -c "import json;d=json.load(open('$out/b_${f}_$r.json'));print('s22 round $r copy1=$f', round(d['ms_per_step'],2), 'ms')"
  done
done
for f in 2 1; do
  CBG_COPY1=$f timeout -k 10 300 python bench.py --no-cpu-baseline --scale 18 --steps 30 --warmup 3 > $out/s18_$f.json 2>>$out/err.log || exit 1
  python3 -c "import json;d=json.load(open('$out/s18_$f.json'));print('s18 copy1=$f', round(d['ms_per_step'],3), 'ms')"
done
