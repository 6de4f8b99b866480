#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_local.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tm.log 2>&1 || { tail -30 gpurun_out/tm.log; exit 1; }
tail -1 gpurun_out/tm.log
tools/run_variants_s22.sh rowsnt norowsdirect && tools/run_variants_s22.sh rowsnt norowsdirect || exit 1
export TMPDIR=/tmp
out=gpurun_out/prof_rows
mkdir -p $out
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $out/pw -o w -- python3 tools/traffic.py run --scale 22 --phases 3 > $out/metaw.log 2>&1 || exit 1
echo done
