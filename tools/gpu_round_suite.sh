set -o pipefail
NO_BENCH=1 bash tools/gpu_tests.sh || exit 1
OUT=r05a bash tools/gpu_kstats.sh || exit 1
OUT=r05a bash tools/gpu_pmc_l2.sh || exit 1
