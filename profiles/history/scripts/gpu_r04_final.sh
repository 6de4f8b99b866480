#!/bin/bash
# Round-4 final profiles: scale-22 kernel summary + HBM traffic (PMC passes),
# then the driver's N = 2 / 4 bench command rehearsed over RCCL's socket transport
set -o pipefail
STEPS=3 bash tools/profile_round.sh r04 22 2 || exit 1
bash tools/gpu_bench_rehearsal.sh 18 2 4 || exit 1
