#!/bin/bash
# SQ counters of the local multiply under CBG_DBG ablation masks (diagnostics only).
# usage: tools/pmc_ablate.sh out_dir scale mask...
set -e -o pipefail
out=$1; sc=$2; shift 2
mkdir -p $out
for m in "$@"; do
  CBG_DBG=$m timeout -k 10 200 rocprofv3 --pmc ${PMC:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS} --kernel-trace --output-format csv -d $out/m$m -o s -- python3 tools/traffic.py run --scale $sc > $out/m$m.log 2>&1
done
