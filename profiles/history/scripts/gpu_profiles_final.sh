#!/bin/bash
# profile bundle at scale 22 (3 phases) and 18, then the default bench line
set -o pipefail
bash tools/profile_round.sh r02 22 3 || exit 1
bash tools/profile_round.sh r02 18 1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { tail -5 gpurun_out/bench_full.err; exit 1; }
cat gpurun_out/bench_full.json
