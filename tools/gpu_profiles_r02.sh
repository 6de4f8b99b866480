#!/bin/bash
# round-2 profile bundle: s22 (4 phases) and s18 kernel stats + traces + PMC traffic
set -o pipefail
bash tools/profile_round.sh r02 22 4 || exit 1
STEPS=20 bash tools/profile_round.sh r02 18 1 || exit 1
