#!/bin/bash
# new-surface GPU tests, Galerkin s22 (+ per-rank 2x4 tiles), default bench with the CPU baseline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${K:-plugin or adapter or galerkin or phased_scale22}" > gpurun_out/batch_tests.log 2>&1
rc=$?; tail -3 gpurun_out/batch_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/galerkin.py --scale 22 --minplus --rank-tiles 2x4 --iters 2 > gpurun_out/galerkin_s22.json 2> gpurun_out/galerkin_s22.err || { tail -5 gpurun_out/galerkin_s22.err; exit 1; }
timeout -k 10 900 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { tail -5 gpurun_out/bench_full.err; exit 1; }
cat gpurun_out/bench_full.json
