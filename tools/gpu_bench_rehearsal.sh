#!/bin/bash
# The driver's N>1 bench command, rehearsed on a one-GPU box: every rank on the
# same GPU, RCCL over its socket transport (CBG_RANK_HOSTIDS=1, see bench.py).
# Checks the code path end to end; the times say nothing about xGMI.
#   tools/gpu_bench_rehearsal.sh [scale] [N...]
set -o pipefail
mkdir -p gpurun_out
sc=${1:-18}; shift
for n in ${@:-2 4}; do
  port=$((29500 + 2 * n))
  CBG_RANK_HOSTIDS=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n --scale $sc --steps 3 --warmup 1 \
    > gpurun_out/rehearsal_n$n.json 2> gpurun_out/rehearsal_n$n.err || { tail -20 gpurun_out/rehearsal_n$n.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('gpurun_out/rehearsal_n$n.json').read().strip().splitlines()[-1])
c = d['config']
db = c['double_buffering']
print('N=$n', c['grid'], c['transport'], 'nnz_C', c['nnz_C'], 'phases', c['phases'], 'ms', round(d['ms_per_step'], 2),
      'pieces', db['pieces'], 'decision', db.get('decision'), 'exposed_comm_ms', db.get('exposed_comm_ms'),
      'bytes_bcast_rank0', db.get('bytes_bcast_rank0'))"
done
