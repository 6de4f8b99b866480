#!/bin/bash
# per-phase block time of the slab kernels (CBG_DBG=16 wall-clock marks) at one scale:
#   tools/gpu_phases.sh [scale] [phases]
set -o pipefail
mkdir -p gpurun_out
sc=${1:-22}; ph=${2:-3}
CBG_DBG=16 timeout -k 10 300 python bench.py --no-cpu-baseline --scale $sc --phases $ph --steps 1 --warmup 1 \
  > gpurun_out/phases_s$sc.json 2> gpurun_out/phases_s$sc.err || exit 1
grep -E "cbg (phases|slabs)" gpurun_out/phases_s$sc.err | tail -8
