#!/bin/bash
# The round's GPU checks in one call: the full pytest -m gpu pass and smoke (no bench),
# then the scale-22 kernel table and the L2 table
set -o pipefail
NO_BENCH=1 bash tools/gpu_tests.sh || exit 1
OUT=${R:-r05}a bash tools/gpu_kstats.sh || exit 1
OUT=${R:-r05}a bash tools/gpu_pmc_l2.sh || exit 1
