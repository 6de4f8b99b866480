#!/bin/bash
# round-3 GPU check: VMM reproducer, the new/changed GPU tests, default bench (auto phases)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 tools/vmm_repro > gpurun_out/vmm_repro.log 2>&1; echo "vmm_repro rc=$?"; tail -3 gpurun_out/vmm_repro.log
K=${PYTEST_K:-"auto_phases or phase_split or phased_scale22 or rank_tiles or galerkin_scale22 or multtiming_unmodified or adapter_runs or narrow or mismatch or redist_fault or (summa_multiprocess and largeseq) or rccl_multirank"}
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread -k "$K" > gpurun_out/r03_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/r03_tests.log | tail -60
tail -3 gpurun_out/r03_tests.log
[ $rc -eq 0 ] || exit $rc
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err || { tail -20 gpurun_out/r03_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r03_bench.json'));print(round(d['value']/1e9,2),'G',round(d['ms_per_step'],1),'ms',d['config']['phases'],d['config']['phase_plan'])"
