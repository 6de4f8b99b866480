#!/bin/bash
# The whole GPU suite, one process, per-test timeouts; a heartbeat line every
# 60 s under gpurun_out/ (the long scale-24 tests print nothing for minutes)
set -o pipefail
mkdir -p gpurun_out
(while sleep 60; do date +%T >> gpurun_out/suite_heartbeat.log; done) &
hb=$!
timeout -k 10 1400 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/full_gpu_tests.log 2>&1
rc=$?
kill $hb
tail -5 gpurun_out/full_gpu_tests.log
exit $rc
