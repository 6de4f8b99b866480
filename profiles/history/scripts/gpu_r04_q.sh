#!/bin/bash
# Round 4: scale-24 kernel summary (one timed step of 14 phases under rocprofv3)
set -o pipefail
out=gpurun_out/q
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/ks -o k -- python3 bench.py --scale 24 --steps 1 --warmup 1 --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
grep '^{' $out/bench.json | head -c 300; echo
