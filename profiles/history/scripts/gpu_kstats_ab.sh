#!/bin/bash
# per-kernel time (rocprofv3 kernel stats) of a 1-step scale-22 bench for variants and the in-tree build
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in ${VARIANTS} base; do
  lib=build/variants/$v/libcbg.so; [ $v = base ] && lib=combblas-spmm-test_amd/libcbg.so
  rm -rf gpurun_out/ks_$v
  CBG_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ks_$v -o k -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ks_$v.json 2> gpurun_out/ks_$v.err || exit 1
  echo "== $v"
  python3 - "$v" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/ks_{sys.argv[1]}/**/k_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {r['Calls']:>4} {r['Name'][:90]}")
PY
done
