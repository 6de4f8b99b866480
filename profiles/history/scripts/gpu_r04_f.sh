#!/bin/bash
# round-4 profile bundle: kernel stats + FETCH/WRITE passes at scale 22 (2 phases) and 18
set -o pipefail
STEPS=5 bash tools/profile_round.sh r04 22 2 || exit 1
STEPS=10 bash tools/profile_round.sh r04 18 1 || exit 1
echo done
