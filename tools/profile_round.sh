#!/bin/bash
# Round profile bundle (run on the GPU box from the repo root):
#   tools/profile_round.sh r01 [scale] [phases]
# 1. rocprofv3 --kernel-trace --stats of the default bench (kernel summary)
# 2. two PMC passes (FETCH_SIZE, WRITE_SIZE) over tools/traffic.py run (2nd multiply)
# Raw outputs go to gpurun_out/prof_<tag>/; parse with tools/profile_collect.sh.
set -e -o pipefail
tag=$1; sc=${2:-18}; ph=${3:-1}
out=gpurun_out/prof_${tag}_s$sc
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/ks -o k -- python3 bench.py --scale $sc --phases $ph --steps ${STEPS:-10} --warmup 1 --no-cpu-baseline --no-f64-leg > $out/bench.json 2> $out/bench.err
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/pf -o f -- python3 tools/traffic.py run --scale $sc --phases $ph > $out/meta.log 2>&1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $out/pw -o w -- python3 tools/traffic.py run --scale $sc --phases $ph > $out/metaw.log 2>&1
echo done
