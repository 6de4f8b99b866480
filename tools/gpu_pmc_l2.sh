#!/bin/bash
# L2 hit rate and request counts per kernel of one scale-${SCALE:-22} multiply (tools/traffic.py run, 2nd
# multiply), two separate --pmc passes (rocprofv3 cannot split counters over passes):
#   OUT=tag [ENVS="VAR=x,..."] tools/gpu_pmc_l2.sh
set -o pipefail
out=gpurun_out/pmc_${OUT:-x}
mkdir -p $out
export TMPDIR=/tmp
ph=${PHASES:-2}
env $(echo $ENVS | tr ',' ' ') bash tools/pmc_sq.sh $out/a ${SCALE:-22} $ph "TCC_HIT_sum TCC_MISS_sum" || exit 1
env $(echo $ENVS | tr ',' ' ') bash tools/pmc_sq.sh $out/b ${SCALE:-22} $ph "TCC_REQ_sum TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum" || exit 1
python3 tools/pmc_kernels.py $(find $out/a $out/b -name '*counter_collection.csv') > $out/table.txt || exit 1
cat $out/table.txt
