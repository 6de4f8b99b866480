#!/bin/bash
# same-box A/B of libcbg variants at scale 22 (and 18): tools/gpu_variants.sh v1 v2 ...
set -o pipefail
tools/run_variants_s22.sh "$@" && tools/run_variants_s22.sh "$@" && SCALE=18 tools/run_variants_s22.sh "$@"
