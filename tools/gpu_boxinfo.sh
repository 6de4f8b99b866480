#!/bin/bash
# Host facts for the CPU baseline (cores actually available to this job).
mkdir -p gpurun_out
{ lscpu; echo "--- nproc"; nproc; echo "--- affinity"; python3 -c "import os;print(len(os.sched_getaffinity(0)))";
  echo "--- cgroup cpu.max"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /sys/fs/cgroup/cpu/cpu.cfs_quota_us 2>/dev/null;
  echo "--- mem"; free -g; } > gpurun_out/boxinfo.txt 2>&1
