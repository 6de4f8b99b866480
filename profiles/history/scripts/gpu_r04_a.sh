#!/bin/bash
# Round-4 first look: default bench on this box, then SQ counter passes over one
# scale-22 MemEfficientSpGEMM (2 phases; tools/traffic.py run marks its second
# multiply), then the slab kernels' phase marks + product/nnz counters.
set -o pipefail
out=gpurun_out/r04a
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $out/bench.json 2> $out/bench.err || exit 1
tools/pmc_sq.sh $out/sq1 22 2 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU" || exit 1
tools/pmc_sq.sh $out/sq2 22 2 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_ATOMIC_RETURN SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INST_LEVEL_VMEM SQ_WAVE_CYCLES" || exit 1
tools/pmc_sq.sh $out/sq3 22 2 "SQ_INSTS_LDS_ATOMIC SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES" || exit 1
CBG_DBG=48 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline > $out/marks.json 2> $out/marks.err || exit 1
echo done
