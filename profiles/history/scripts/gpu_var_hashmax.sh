#!/bin/bash
# A/B of the hash-pair product limit (CBG_SPARSE_SLAB_MAX variants) at scales 22, 18 and 24
set -o pipefail
mkdir -p gpurun_out
CBG_LIB=build/variants/hash3072/libcbg.so timeout -k 10 400 python -u -m pytest tests/test_gpu_local.py -x -q --timeout 300 --timeout-method thread -k "digest or bit_exact or panel_groups or random_fp or big_column" > gpurun_out/tv.log 2>&1 || { tail -20 gpurun_out/tv.log; exit 1; }
tail -1 gpurun_out/tv.log
tools/run_variants_s22.sh hash3072 hash2048 && tools/run_variants_s22.sh hash3072 hash2048 && SCALE=18 tools/run_variants_s22.sh hash3072 hash2048 || exit 1
for v in hash3072 base; do
  lib=build/variants/$v/libcbg.so; [ $v = base ] && lib=combblas-spmm-test_amd/libcbg.so
  CBG_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --scale 24 --steps 3 > gpurun_out/v24_$v.json 2>>gpurun_out/v.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/v24_$v.json'));print('s24 $v', round(d['value']/1e9,2), 'G nnz/s', round(d['ms_per_step'],1), 'ms')"
done
