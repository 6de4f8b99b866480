#!/bin/bash
# Round-5 profile bundle on the GPU box (then tools/profile_collect.sh r05 22 / 18 here):
# scale-22 and scale-18 kernel stats + traffic, the L2 table at 22, scale 24 (5 steps) and GalerkinNew
set -o pipefail
STEPS=5 bash tools/profile_round.sh r05 22 2 || exit 1
STEPS=10 bash tools/profile_round.sh r05 18 1 || exit 1
OUT=r05_s22 SCALE=22 PHASES=2 bash tools/gpu_pmc_l2.sh > /dev/null || exit 1
OUT=r05sec STEPS24=5 bash tools/gpu_secondary.sh || exit 1
