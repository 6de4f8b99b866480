mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_local.py -x -v --timeout 200 --timeout-method thread -k "panel_groups or tall or variants or digest_vs" > gpurun_out/t2.log 2>&1 || { echo TESTFAIL; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/b22.json 2> gpurun_out/b22.err || exit 1
CBG_GROUPS=0 timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/b22_nog.json 2>> gpurun_out/b22.err || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --scale 20 > gpurun_out/b20.json 2>> gpurun_out/b22.err || exit 1
CBG_GROUPS=0 timeout -k 10 200 python bench.py --no-cpu-baseline --scale 20 > gpurun_out/b20_nog.json 2>> gpurun_out/b22.err || exit 1
echo ok
