#!/bin/bash
# round 4 validation + secondary lines: the whole GPU suite, the default bench line, the random-valued
# scale-22 line, scale 24 on one GPU, GalerkinNew at scale 22 on the genrestrict-shaped restriction
set -o pipefail
out=gpurun_out/r04d
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 \
  || { tail -40 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > $out/bench_default.json 2> $out/bench_default.err || exit 1
timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --values random > $out/bench_random.json 2>> $out/err.log || exit 1
timeout -k 10 300 python bench.py --scale 24 --steps 3 --warmup 1 --no-cpu-baseline > $out/bench_s24.json 2>> $out/err.log || exit 1
timeout -k 10 400 python tools/galerkin.py --scale 22 --minplus --rank-tiles 2x4 --iters 2 > $out/galerkin_s22.json 2>> $out/err.log || exit 1
python3 - <<'PY'
import json
for f in ("bench_default", "bench_random", "bench_s24"):
    d = json.load(open("gpurun_out/r04d/%s.json" % f))
    r = d["roofline"]
    print(f, round(d["value"] / 1e9, 2), "G nnz/s", round(d["ms_per_step"], 1), "ms frac", round(r["frac"], 3),
          "peak_measured", round(r["peak_measured"]), "cpu", d.get("cpu_baseline", {}).get("value"))
g = json.load(open("gpurun_out/r04d/galerkin_s22.json"))
print("galerkin", g["full_restriction_s"], g["split_restriction_s"], g["roofline_full"]["frac"], g.get("full_restriction_minplus_s"))
PY
