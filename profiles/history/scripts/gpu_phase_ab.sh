#!/bin/bash
# per-phase slab block time (CBG_DBG=16 marks, + 32 counters) at scale 22, one step, for variants and the in-tree build
set -o pipefail
mkdir -p gpurun_out
for v in ${VARIANTS} base; do
  lib=build/variants/$v/libcbg.so; [ $v = base ] && lib=combblas-spmm-test_amd/libcbg.so
  CBG_DBG=${DBG:-16} CBG_LIB=$lib timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS} \
    > gpurun_out/ph_$v.json 2> gpurun_out/ph_$v.err || exit 1
  echo "== $v"; grep "cbg phases" gpurun_out/ph_$v.err | tail -1
done
