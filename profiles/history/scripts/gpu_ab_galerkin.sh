#!/bin/bash
# local parity tests, then for each variant (CBG_LIB) and the in-tree build: s18 bench and GalerkinNew s22, twice
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_local.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tm.log 2>&1 || { tail -30 gpurun_out/tm.log; exit 1; }
tail -1 gpurun_out/tm.log
for rep in 1 2; do
  for v in ${VARIANTS} base; do
    lib=build/variants/$v/libcbg.so; [ $v = base ] && lib=combblas-spmm-test_amd/libcbg.so
    CBG_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --scale 18 > gpurun_out/g_$v.json 2>>gpurun_out/g.err || exit 1
    CBG_LIB=$lib timeout -k 10 200 python tools/galerkin.py --scale 22 > gpurun_out/gal_$v.json 2>>gpurun_out/g.err || exit 1
    python3 -c "
import json;d=json.load(open('gpurun_out/g_$v.json'));g=open('gpurun_out/gal_$v.json').read().strip().splitlines()[-1]
print('$v s18', round(d['ms_per_step'],3), 'ms | galerkin', g[:300])"
  done
done
