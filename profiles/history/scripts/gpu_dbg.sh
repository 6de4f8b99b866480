set -o pipefail
mkdir -p gpurun_out
export CBG_DEBUG_ERRORS=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 250 --timeout-method thread -k "${K:-scale18}" > gpurun_out/mp.log 2>&1
tail -3 gpurun_out/mp.log
