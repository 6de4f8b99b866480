set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_local.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tm.log 2>&1 || { tail -30 gpurun_out/tm.log; exit 1; }
tail -1 gpurun_out/tm.log
tools/run_variants_s22.sh ${VARIANTS} && tools/run_variants_s22.sh ${VARIANTS} && SCALE=18 tools/run_variants_s22.sh ${VARIANTS}
