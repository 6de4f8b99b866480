#!/bin/bash
# bench.py's N>1 path on the one-GPU box: torchrun with 2 and 4 ranks on the same GPU
# (RCCL rejects duplicate devices, so the ranks fall back to the TCP host transport);
# checks that the driver's multi-GPU invocation produces its JSON line
set -o pipefail
mkdir -p gpurun_out
for n in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29600 + n * 10)) bench.py --gpus $n --scale ${SCALE:-18} --steps 3 --warmup 1 \
    > gpurun_out/bench_n$n.json 2> gpurun_out/bench_n$n.err || { tail -20 gpurun_out/bench_n$n.err; exit 1; }
  grep '^{' gpurun_out/bench_n$n.json | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print($n, d['value']/1e9, d['ms_per_step'], d['config']['grid'], d['config']['transport'], d['config']['double_buffering'])"
done
