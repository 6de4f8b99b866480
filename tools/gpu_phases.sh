set -o pipefail
mkdir -p gpurun_out
for ph in 3 4 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --scale 22 --phases $ph > gpurun_out/ph_$ph.json 2>> gpurun_out/ph.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/ph_$ph.json'));print('phases $ph', round(d['value']/1e9,2), 'G nnz/s', round(d['ms_per_step'],2), 'ms', round(d['roofline']['frac'],3))"
done
