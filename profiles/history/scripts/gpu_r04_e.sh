#!/bin/bash
# round 4: product-loop segment cursor variants (CBG_CURSOR 1/2) checked and timed against the tree,
# scale 22 and scale 18
set -o pipefail
mkdir -p gpurun_out/r04e
for v in cur1 cur2; do
  CBG_LIB=build/variants/$v/libcbg.so timeout -k 10 600 python -u -m pytest tests/test_gpu_local.py -x -q --timeout 300 \
    --timeout-method thread -k "digest or bit_exact or panel_groups or random_fp or big_column or esc or thin" \
    > gpurun_out/r04e/tests_$v.log 2>&1 || { tail -30 gpurun_out/r04e/tests_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r04e/tests_$v.log)"
done
VARIANTS="tree cur1 cur2" ROUNDS=2 bash tools/gpu_libab.sh || exit 1
SCALE=18 STEPS=30 VARIANTS="tree cur1 cur2" ROUNDS=1 bash tools/gpu_libab.sh || exit 1
bash tools/gpu_bench_rehearsal.sh 18 2 4 || exit 1
# a 3x1 grid: two remote B tiles per grid column, the RCCL rule that pipelines without measuring
CBG_RANK_HOSTIDS=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 \
  --master-port 29530 bench.py --gpus 3 --grid 3x1 --scale 18 --steps 3 --warmup 1 > gpurun_out/rehearsal_n3.json \
  2> gpurun_out/rehearsal_n3.err || { tail -20 gpurun_out/rehearsal_n3.err; exit 1; }
python3 -c "import json; d = json.loads(open('gpurun_out/rehearsal_n3.json').read().strip().splitlines()[-1]); print('N=3', d['config']['grid'], d['config']['double_buffering'])"
echo done
