#!/bin/bash
# Round profile bundle on the GPU box (then, here: tools/profile_collect.sh $R 22 and $R 18,
# and copy gpurun_out/pmc_${R}_s22/table.txt, gpurun_out/${R}sec/* into profiles/):
# scale-22 and scale-18 kernel stats + traffic (the bench's phase plans), the L2 table at 22,
# scale 24 (5 steps) and GalerkinNew.  The default bench line is run after the collection,
# so that its roofline.traffic reads this round's traffic file.
#   R=r05 tools/gpu_profiles_round.sh
set -o pipefail
R=${R:-r05}
STEPS=5 bash tools/profile_round.sh $R 22 2 || exit 1
STEPS=10 bash tools/profile_round.sh $R 18 1 || exit 1
OUT=${R}_s22 SCALE=22 PHASES=2 bash tools/gpu_pmc_l2.sh > /dev/null || exit 1
OUT=${R}sec STEPS24=5 bash tools/gpu_secondary.sh || exit 1
