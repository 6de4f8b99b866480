#!/bin/bash
# Round 4 refresh: default bench line (N=1, scale 22, with the CPU baseline),
# scale 24 5-step line, GalerkinNew scale 22 with the 2x4 rank tiles
set -o pipefail
out=gpurun_out/l
mkdir -p $out
timeout -k 10 600 python bench.py > $out/bench_default.json 2> $out/bench_default.err || { tail -20 $out/bench_default.err; exit 1; }
python3 -c "import json;d=json.load(open('$out/bench_default.json'));print('default', round(d['ms_per_step'],2), 'ms', d['roofline']['frac'], d['roofline'].get('peak_measured'))"
timeout -k 10 300 python tools/galerkin.py --scale 22 --iters 5 --rank-tiles 2x4 --minplus > $out/galerkin_s22.json 2> $out/galerkin.err || { tail -20 $out/galerkin.err; exit 1; }
python3 -c "import json;d=json.load(open('$out/galerkin_s22.json'));print('galerkin', d['full_restriction_s'], d['roofline_full']['frac'], d['split_restriction_s'], d.get('full_restriction_minplus_s'))"
timeout -k 10 900 python bench.py --scale 24 --steps 5 --warmup 1 --no-cpu-baseline > $out/bench_s24.json 2> $out/bench_s24.err || { tail -20 $out/bench_s24.err; exit 1; }
python3 -c "import json;d=json.load(open('$out/bench_s24.json'));print('s24', round(d['ms_per_step'],1), 'ms', d['roofline']['frac'])"
