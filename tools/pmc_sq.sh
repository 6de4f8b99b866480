#!/bin/bash
# SQ counter pass over tools/traffic.py run (2nd multiply = dispatches between the 2nd and 3rd k_digest):
#   tools/pmc_sq.sh <out_dir> <scale> <phases> "<counters>"
set -e -o pipefail
out=$1; sc=$2; ph=$3; ctr=$4
mkdir -p $out
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $out -o s -- python3 tools/traffic.py run --scale $sc --phases $ph > $out/run.log 2>&1
