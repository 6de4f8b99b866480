#!/bin/bash
# hash-slab kernel time with parts ablated (CBG_DBG 512: no products, 1024: no emit; results wrong) and with
# the numeric small bins on the main stream (CBG_SIDE=1), kernel stats per run; scale 22, 1 step
set -o pipefail
mkdir -p gpurun_out/hab
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for d in 0 512 1024 1536 side1; do
  envs="CBG_DBG=$d"; [ $d = side1 ] && envs="CBG_SIDE=1"
  rm -rf gpurun_out/hab/$d
  env $envs timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/hab/$d -o k -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/hab/$d.json 2> gpurun_out/hab/$d.err || exit 1
  python3 - "$d" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/hab/{sys.argv[1]}/**/k_kernel_stats.csv", recursive=True)[0]
tot = 0
for r in csv.DictReader(open(f)):
    if 'k_num_slab_hash' in r['Name'] or 'k_num_slab<' in r['Name'] or 'k_sym_panel' in r['Name']:
        print(f"dbg={sys.argv[1]} {float(r['TotalDurationNs'])/1e6:8.2f} ms {r['Name'][:52]}")
PY
done
