#!/bin/bash
# GalerkinNew scale-22 full restriction on one GPU under a kernel trace: per-kernel stats
# and the timeline (busy vs host gaps) of the last full restriction's two multiplies
set -o pipefail
mkdir -p gpurun_out/galt
export TMPDIR=/tmp
S=${SCALE:-22}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/galt/prof -o k -- python3 tools/galerkin.py --scale $S --iters 3 --only-full > gpurun_out/galt/run.json 2> gpurun_out/galt/run.err || { tail -5 gpurun_out/galt/run.err; exit 1; }
tail -1 gpurun_out/galt/run.json | head -c 300; echo
f=$(find gpurun_out/galt/prof -name "k_kernel_trace.csv" | head -1)
python3 tools/gal_timeline.py $f 2 > gpurun_out/galt/timeline.txt
tail -14 gpurun_out/galt/timeline.txt
timeout -k 10 120 python3 tools/galerkin.py --scale $S --iters 5 --only-full > gpurun_out/galt/plain.json 2>/dev/null && python3 -c "import json;d=json.load(open('gpurun_out/galt/plain.json'));print('full_restriction_s',d['full_restriction_s'])"
