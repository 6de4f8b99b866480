#!/bin/bash
# Kernel trace of the driver's N=2 bench command rehearsed on one GPU (both ranks on
# the card, RCCL socket transport, CBG_RANK_HOSTIDS=1): do the RCCL broadcast
# kernels of the pipelined PANEL SUMMA run while k_num_slab / k_sym_panel hold the
# CUs?  tools/overlap.py summarizes per process.  usage: tools/gpu_overlap_trace.sh [scale] [extra env]
set -o pipefail
mkdir -p gpurun_out/overlap
export TMPDIR=/tmp
sc=${1:-20}
env ${2:-CBG_X=0} CBG_RANK_HOSTIDS=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/overlap/trace -o %pid%_k -- \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29610 \
  bench.py --gpus 2 --scale $sc --steps 3 --warmup 1 > gpurun_out/overlap/bench.json 2> gpurun_out/overlap/bench.err \
  || { tail -20 gpurun_out/overlap/bench.err; exit 1; }
tail -1 gpurun_out/overlap/bench.json | head -c 600; echo
python3 tools/overlap.py gpurun_out/overlap/trace --json gpurun_out/overlap/summary.json
