set -o pipefail
mkdir -p gpurun_out/dbg
for sc in 22 24; do
CBG_DBG=48 timeout -k 10 300 python bench.py --scale $sc --steps 1 --warmup 0 --no-cpu-baseline --no-f64-leg > gpurun_out/dbg/b$sc.json 2> gpurun_out/dbg/b$sc.err || exit 1
grep -E "k_num_slab\]|phases" gpurun_out/dbg/b$sc.err | tail -4
done
