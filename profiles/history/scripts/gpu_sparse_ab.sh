#!/bin/bash
# sparse-pair threshold A/B (hash vs bitmap slabs) at scale 22, default and larger kept-bitmap budgets
set -o pipefail
mkdir -p gpurun_out
tools/run_variants_s22.sh sp2048 sp1024 || exit 1
CBG_BITMAP_BUDGET_GB=100 tools/run_variants_s22.sh sp2048 sp1024 || exit 1
CBG_DBG=48 CBG_LIB=build/variants/sp1024/libcbg.so timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pm48b.json 2> gpurun_out/pm48b.err || exit 1
grep "cbg" gpurun_out/pm48b.err | tail -3
