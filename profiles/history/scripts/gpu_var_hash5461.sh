#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
CBG_LIB=build/variants/hash5461/libcbg.so timeout -k 10 400 python -u -m pytest tests/test_gpu_local.py -x -q --timeout 300 --timeout-method thread -k "digest or bit_exact or panel_groups or random_fp or big_column or phased_scale22" > gpurun_out/tv.log 2>&1 || { tail -20 gpurun_out/tv.log; exit 1; }
tail -1 gpurun_out/tv.log
tools/run_variants_s22.sh hash5461 && tools/run_variants_s22.sh hash5461 && SCALE=18 tools/run_variants_s22.sh hash5461 || exit 1
for v in hash5461 base; do
  lib=build/variants/$v/libcbg.so; [ $v = base ] && lib=combblas-spmm-test_amd/libcbg.so
  CBG_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --scale 24 --steps 3 > gpurun_out/v24_$v.json 2>>gpurun_out/v.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/v24_$v.json'));print('s24 $v', round(d['value']/1e9,2), 'G nnz/s', round(d['ms_per_step'],1), 'ms')"
done
