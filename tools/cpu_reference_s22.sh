#!/bin/bash
# One-off CPU baseline at the metric's own scale (run on the GPU box's host):
# the reference's Mult_AnXBn_Synch on R-MAT scale-22 ef16 A*A at 1x1, B cut into
# 16 column phases (SpDCCols::ColSplit; the whole C, 24.8 G nonzeros, exceeds
# the job's host memory), one process per phase (the reference's heap grows
# across calls: 5 phases in one process passed the box's 270 GB cap), on every
# CPU the job may use.  -> gpurun_out/cpu_ref_s22.log; tools/cpu_reference_s22.py
# sums it into profiles/<round>_cpu_reference_s22.json.
set -e -o pipefail
mkdir -p gpurun_out
T=$(python3 -c "import os;n=len(os.sched_getaffinity(0));q=open('/sys/fs/cgroup/cpu.max').read().split();print(min(n,int(q[0])//int(q[1])) if q[0]!='max' else n)")
echo "threads $T" > gpurun_out/cpu_ref_s22.log
lscpu | grep -E "Model name|Socket|Core\(s\)|Thread\(s\)" >> gpurun_out/cpu_ref_s22.log
export OMP_NUM_THREADS=$T
timeout -k 10 300 oracle/_ref/ref_driver gen 22 16 /tmp/cbg_A22.cbgt >> gpurun_out/cpu_ref_s22.log
for p in $(seq 0 15); do
  timeout -k 10 300 oracle/_ref/ref_driver multphased synch plus /tmp/cbg_A22.cbgt /tmp/cbg_A22.cbgt 16 $p 1 >> gpurun_out/cpu_ref_s22.log
done
rm -f /tmp/cbg_A22.cbgt
