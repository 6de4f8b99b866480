#!/bin/bash
# round-2 profile bundle at the bench default (scale 22, 3 phases) + the default bench line
set -o pipefail
bash tools/profile_round.sh r02 22 3 || exit 1
timeout -k 10 900 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { tail -5 gpurun_out/bench_full.err; exit 1; }
cat gpurun_out/bench_full.json
