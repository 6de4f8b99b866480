#!/bin/bash
# fused small columns: local GPU parity tests, Galerkin s22 timing and the s22 bench, fused vs not
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_local.py -x -q --timeout 300 --timeout-method thread > gpurun_out/e_tests.log 2>&1; rc=$?; tail -3 gpurun_out/e_tests.log; [ $rc -eq 0 ] || exit $rc
for f in 1 0; do
  CBG_FUSE_SMALL=$f timeout -k 10 200 python3 tools/galerkin.py --scale 22 --iters 5 --minplus > gpurun_out/e_gal_$f.json 2> gpurun_out/e_gal_$f.err || { tail -5 gpurun_out/e_gal_$f.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/e_gal_$f.json').read().strip().splitlines()[-1]);print('fuse=$f galerkin', round(d['full_restriction_s']*1e3,2), round(d['split_restriction_s']*1e3,2), round(d['full_restriction_minplus_s']*1e3,2), d['splitting_correct'])"
done
for f in 1 0; do
  CBG_FUSE_SMALL=$f timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 > gpurun_out/e_b$f.json 2> gpurun_out/e_b$f.err || { tail -5 gpurun_out/e_b$f.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/e_b$f.json'));print('fuse=$f s22', round(d['value']/1e9,2),'G',round(d['ms_per_step'],1),'ms', d['config']['phases'])"
  CBG_FUSE_SMALL=$f timeout -k 10 300 python bench.py --no-cpu-baseline --scale 18 --steps 20 > gpurun_out/e_b18_$f.json 2> gpurun_out/e_b18_$f.err || { tail -5 gpurun_out/e_b18_$f.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/e_b18_$f.json'));print('fuse=$f s18', round(d['value']/1e9,2),'G',round(d['ms_per_step'],3),'ms')"
done
