#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/gals
export TMPDIR=/tmp
CBG_SIDE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gals/prof -o k -- python3 tools/galerkin.py --scale 22 --iters 3 --only-full > gpurun_out/gals/run.json 2> gpurun_out/gals/run.err || { tail -5 gpurun_out/gals/run.err; exit 1; }
f=$(find gpurun_out/gals/prof -name "k_kernel_trace.csv" | head -1)
python3 tools/gal_timeline.py $f 2 > gpurun_out/gals/timeline.txt
tail -3 gpurun_out/gals/timeline.txt
CBG_SIDE=0 timeout -k 10 120 python3 tools/galerkin.py --scale 22 --iters 5 --only-full > gpurun_out/gals/plain.json 2>/dev/null && python3 -c "import json;d=json.load(open('gpurun_out/gals/plain.json'));print('side0 full_restriction_s',d['full_restriction_s'])"
