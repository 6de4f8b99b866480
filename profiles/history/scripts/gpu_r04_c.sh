#!/bin/bash
# round 4: symbolic occupancy / overflow A/B, the expand-sort-compress hash classes (esc) checked
# and timed, then LDS counters of the hash slabs (CBG_LIB=base: HEAD of round 3; tree: in-tree build)
set -o pipefail
mkdir -p gpurun_out/r04c
CBG_LIB=build/variants/esc/libcbg.so timeout -k 10 600 python -u -m pytest tests/test_gpu_local.py -x -q --timeout 300 \
  --timeout-method thread -k "digest or bit_exact or panel_groups or random or big_column" > gpurun_out/r04c/esc_tests.log 2>&1 \
  || { tail -30 gpurun_out/r04c/esc_tests.log; exit 1; }
tail -1 gpurun_out/r04c/esc_tests.log
VARIANTS="tree symw8 s8 s8n s8o1 esc" ROUNDS=2 bash tools/gpu_libab.sh || exit 1
CBG_DBG=48 CBG_LIB=build/variants/esc/libcbg.so timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline \
  > gpurun_out/r04c/esc_marks.json 2> gpurun_out/r04c/esc_marks.err || exit 1
C="SQ_INSTS_LDS_ATOMIC SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"
CBG_LIB=build/variants/base/libcbg.so tools/pmc_sq.sh gpurun_out/r04c/base 22 2 "$C" || exit 1
tools/pmc_sq.sh gpurun_out/r04c/tree 22 2 "$C" || exit 1
CBG_LIB=build/variants/esc/libcbg.so tools/pmc_sq.sh gpurun_out/r04c/esc 22 2 "$C" || exit 1
echo done
