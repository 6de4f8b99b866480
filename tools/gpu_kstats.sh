#!/bin/bash
# Kernel time table of the bench (rocprofv3 --kernel-trace --stats), ms per step:
#   OUT=tag [STEPS=3] [SCALE=22] [ENVS="VAR=x,VAR2=y"] tools/gpu_kstats.sh
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/ks_${OUT:-x}
mkdir -p $out
st=${STEPS:-3}
# warmup 1 + st steps: the table counts warmup+steps multiplies
env $(echo $ENVS | tr ',' ' ') timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/ks -o k -- \
  python3 bench.py --scale ${SCALE:-22} --steps $st --warmup 1 --no-cpu-baseline --no-f64-leg ${BENCH_ARGS} \
  > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
f=$(find $out/ks -name '*kernel_stats.csv' | head -1)
cp $f $out/kernel_stats.csv
python3 tools/kstats_top.py $out/kernel_stats.csv $((st + 1)) ${TOP:-22}
