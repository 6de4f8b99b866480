#!/bin/bash
# bench at scale 22 for each build/variants/<name>/libcbg.so given, then the in-tree build
set -o pipefail
mkdir -p gpurun_out
for v in "$@" base; do
  lib=build/variants/$v/libcbg.so; [ $v = base ] && lib=combblas-spmm-test_amd/libcbg.so
  CBG_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline ${SCALE:+--scale $SCALE} > gpurun_out/v_$v.json 2>>gpurun_out/v.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/v_$v.json'));print('$v', round(d['value']/1e9,2), 'G nnz/s', round(d['ms_per_step'],2), 'ms')"
done
