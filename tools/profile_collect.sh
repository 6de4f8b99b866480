#!/bin/bash
# Copy the judged summaries of tools/profile_round.sh into profiles/ (run here after gpurun).
set -e
tag=$1; sc=${2:-18}
src=gpurun_out/prof_${tag}_s$sc
cp $src/ks/k_kernel_stats.csv profiles/${tag}_s${sc}_kernel_stats.csv
grep '^{' $src/bench.json > profiles/${tag}_s${sc}_bench_under_rocprof.json
python3 tools/traffic.py parse --fetch $src/pf/f_counter_collection.csv --write $src/pw/w_counter_collection.csv \
  --meta $src/meta.log --out profiles/${tag}_traffic_s${sc}.json
