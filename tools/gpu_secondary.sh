#!/bin/bash
# Secondary configurations: scale 24 on one GPU (STEPS24 steps) and GalerkinNew at scale 22
# (full + split restriction, min-plus, config 5's 2x4 rank tiles); outputs under gpurun_out/${OUT:-sec}/
set -o pipefail
out=gpurun_out/${OUT:-sec}
mkdir -p $out
if [ -z "$NO_S24" ]; then
  timeout -k 10 900 python bench.py --scale 24 --steps ${STEPS24:-3} --warmup 1 --no-cpu-baseline --no-f64-leg \
    > $out/bench_s24.json 2> $out/bench_s24.err || { tail -20 $out/bench_s24.err; exit 1; }
  python3 -c "import json;d=json.load(open('$out/bench_s24.json'));print('s24', round(d['ms_per_step'],1), 'ms frac', round(d['roofline']['frac'],4))"
fi
timeout -k 10 300 python tools/galerkin.py --scale 22 --iters 5 --rank-tiles 2x4 --minplus > $out/galerkin_s22.json \
  2> $out/galerkin.err || { tail -20 $out/galerkin.err; exit 1; }
python3 -c "import json;d=json.load(open('$out/galerkin_s22.json'));print('galerkin full', round(d['full_restriction_s']*1e3,3), 'ms frac', round(d['roofline_full']['frac'],4), 'split', round(d['split_restriction_s']*1e3,3), 'minplus', round(d['full_restriction_minplus_s']*1e3,3))"
