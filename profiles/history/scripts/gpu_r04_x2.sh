set -o pipefail
out=gpurun_out/x2
mkdir -p $out
for r in 1 2 3; do
  for f in 8 0; do
    CBG_FEW_FRAC=0.2 CBG_FEW=$f timeout -k 10 200 python tools/galerkin.py --scale 22 --iters 5 --only-full > $out/gal_${f}_$r.json 2>>$out/err.log || exit 1
    python3 -c "import json;d=json.load(open('$out/gal_${f}_$r.json'));print('galerkin round $r few=$f', round(d['full_restriction_s']*1e3,3), 'ms')"
  done
done
CBG_FEW_FRAC=0.2 CBG_DBG=16 timeout -k 10 200 python tools/galerkin.py --scale 22 --iters 1 --only-full 2>&1 >/dev/null | grep "cbg bins" | tail -2
