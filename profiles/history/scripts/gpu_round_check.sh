set -o pipefail
bash tools/gpu_boxinfo.sh
bash tools/gpu_final_check.sh || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_r02a
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r02a/ks -o k -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r02a/bench.json 2> gpurun_out/prof_r02a/bench.err
