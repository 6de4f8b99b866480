#!/bin/bash
# per-phase block time of the slab kernels (CBG_DBG=16: wall-clock marks; results are still exact,
# the marks only add a timer read and an atomic per block phase) at scale 22, one step
set -o pipefail
mkdir -p gpurun_out
CBG_DBG=16 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS} \
  > gpurun_out/phase_marks.json 2> gpurun_out/phase_marks.err
rc=$?
grep "cbg phases" gpurun_out/phase_marks.err | tail -12
exit $rc
