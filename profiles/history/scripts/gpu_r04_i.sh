set -o pipefail
timeout -k 10 900 python -u -m pytest tests/test_gpu_local.py -x -q --timeout 300 --timeout-method thread -k "esc or galerkin or thin or local_digest or phased_scale22 or auto_phases or flops" > gpurun_out/i_tests.log 2>&1 || { tail -30 gpurun_out/i_tests.log; exit 1; }
tail -1 gpurun_out/i_tests.log
bash tools/gpu_galerkin_trace.sh
