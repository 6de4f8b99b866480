#!/bin/bash
# round-2 profile bundle at scale 22 (4 phases): kernel stats + trace + PMC traffic
set -o pipefail
bash tools/profile_round.sh r02 22 4 || exit 1
