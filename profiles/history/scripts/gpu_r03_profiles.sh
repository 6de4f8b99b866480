#!/bin/bash
# round-3 profile bundle + secondary configuration lines (GPU box, repo root)
set -o pipefail
mkdir -p gpurun_out
STEPS=5 timeout -k 10 600 bash tools/profile_round.sh r03 22 2 || exit 1
STEPS=20 timeout -k 10 400 bash tools/profile_round.sh r03 18 1 || exit 1
timeout -k 10 400 python bench.py --scale 24 --steps 5 --no-cpu-baseline > gpurun_out/r03_bench_s24_1gpu.json 2> gpurun_out/r03_s24.err || { tail -5 gpurun_out/r03_s24.err; exit 1; }
timeout -k 10 300 python3 tools/galerkin.py --scale 22 --iters 5 --minplus --rank-tiles 2x4 > gpurun_out/r03_galerkin_s22.json 2> gpurun_out/r03_gal.err || { tail -5 gpurun_out/r03_gal.err; exit 1; }
timeout -k 10 300 python3 tools/tile_totals.py --scale 24 --grid 2x4 --reps 2 --pieces 2 > gpurun_out/r03_tiles_s24_2x4.jsonl 2> gpurun_out/r03_tiles.err || { tail -5 gpurun_out/r03_tiles.err; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/r03_bench_default.json 2> gpurun_out/r03_bench_default.err || { tail -5 gpurun_out/r03_bench_default.err; exit 1; }
echo PROFILES DONE
