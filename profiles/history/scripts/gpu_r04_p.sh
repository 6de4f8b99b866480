#!/bin/bash
# Round 4 secondary lines: scale-24 2x4 and scale-22 4x2 per-rank tile products
# on one GPU (no communication), GalerkinNew scale 22 plus-times with the 2x4
# rank tiles and min-plus
set -o pipefail
out=gpurun_out/p
mkdir -p $out
timeout -k 10 400 python3 tools/tile_totals.py --scale 24 --grid 2x4 --reps 2 --pieces 2 > $out/tiles_s24_2x4.jsonl 2> $out/tiles.err || { tail -5 $out/tiles.err; exit 1; }
tail -1 $out/tiles_s24_2x4.jsonl
timeout -k 10 300 python3 tools/tile_totals.py --scale 22 --grid 4x2 --reps 2 > $out/tiles_s22_4x2.jsonl 2>> $out/tiles.err || { tail -5 $out/tiles.err; exit 1; }
tail -1 $out/tiles_s22_4x2.jsonl
timeout -k 10 300 python tools/galerkin.py --scale 22 --iters 5 --rank-tiles 2x4 --minplus > $out/galerkin_s22.json 2> $out/galerkin.err || { tail -20 $out/galerkin.err; exit 1; }
python3 -c "import json;d=json.load(open('$out/galerkin_s22.json'));print('galerkin', d['full_restriction_s'], d['roofline_full']['frac'], d['split_restriction_s'], d.get('full_restriction_minplus_s'))"
