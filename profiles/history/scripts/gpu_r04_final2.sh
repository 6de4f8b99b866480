#!/bin/bash
# Round-4 final refresh after the symbolic stream rule: default bench line,
# scale-22 kernel stats + traffic, scale 24, GalerkinNew (with min-plus and 2x4 tiles)
set -o pipefail
out=gpurun_out/f2
mkdir -p $out
timeout -k 10 600 python bench.py > $out/bench_default.json 2> $out/bench_default.err || { tail -20 $out/bench_default.err; exit 1; }
python3 -c "import json;d=json.loads(open('$out/bench_default.json').read().strip().splitlines()[-1]);print('default', round(d['ms_per_step'],2), 'ms', d['roofline']['frac'], d['roofline'].get('peak_measured'))"
STEPS=3 bash tools/profile_round.sh r04 22 2 || exit 1
timeout -k 10 900 python bench.py --scale 24 --steps 5 --warmup 1 --no-cpu-baseline > $out/bench_s24.json 2> $out/bench_s24.err || { tail -20 $out/bench_s24.err; exit 1; }
python3 -c "import json;d=json.load(open('$out/bench_s24.json'));print('s24', round(d['ms_per_step'],1), 'ms', d['roofline']['frac'])"
timeout -k 10 300 python tools/galerkin.py --scale 22 --iters 5 --rank-tiles 2x4 --minplus > $out/galerkin_s22.json 2> $out/galerkin.err || { tail -20 $out/galerkin.err; exit 1; }
python3 -c "import json;d=json.load(open('$out/galerkin_s22.json'));print('galerkin', d['full_restriction_s'], d['roofline_full']['frac'])"
