#!/usr/bin/env python3
"""Per-rank local products of a pr x pc SUMMA grid, run one after another on ONE GPU.

For rank (r, c) the PANEL execution multiplies the A block row r (rows block r
of pr, all columns) by the B block column c; here both panels are generated
directly on device.  Prints per-rank JSON lines and checks the totals (flops,
nnz(C)) against the reference's symbolic totals in tests/golden/golden.json.

  python tools/tile_totals.py --scale 22 --grid 1x2 [--ranks 0,1]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import load_cbg  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--scale", type=int, default=22)
    p.add_argument("--ef", type=int, default=16)
    p.add_argument("--grid", default="1x2")
    p.add_argument("--ranks", default=None)
    p.add_argument("--reps", type=int, default=1)
    p.add_argument("--pieces", type=int, default=1, help="multiply B's tile in this many column pieces")
    p.add_argument("--summa", action="store_true",
                   help="run the rank's multiply through the PANEL SUMMA on a one-rank grid (the pipelined "
                        "pieces of CBG_PIPELINE, the growable arena, A's maps kept across pieces)")
    a = p.parse_args()
    pr, pc = (int(x) for x in a.grid.split("x"))
    ranks = [int(x) for x in a.ranks.split(",")] if a.ranks else list(range(pr * pc))
    cbg = load_cbg()
    cbg.lib().cbg_set_device(0)
    tot_f = tot_n = 0
    for rk in ranks:
        r, c = rk // pc, rk % pc
        Ap = cbg.rmat_tile(a.scale, a.ef, grid=(pr, 1), pos=(r, 0))
        Bp = cbg.rmat_tile(a.scale, a.ef, grid=(1, pc), pos=(0, c))
        if a.summa:
            class Self:
                def bcast(self, comm, arr, root):
                    pass

                def allgather(self, comm, data):
                    return data
            g1 = cbg.CommGrid(0, 1, transport="host", host_comm=Self())
            nv = 1 << a.scale
            A1 = cbg.SpParMat(Ap, g1, Ap.m, nv)
            B1 = cbg.SpParMat(Bp, g1, nv, Bp.n)
            best = None
            for _ in range(a.reps + 1):  # the first is a warm-up
                cbg.synchronize()
                t0 = time.perf_counter()
                C = cbg.Mult_AnXBn_DoubleBuff(A1, B1)
                cbg.synchronize()
                dt = time.perf_counter() - t0
                nnz = C.tile.nnz
                C.tile.free()
                best = dt if best is None or _ == 0 else min(best, dt)
            print(json.dumps({"rank": rk, "grid": a.grid, "scale": a.scale, "s": best, "nnz_C": nnz,
                              "nnzC_per_s": nnz / best, "pipeline": os.environ.get("CBG_PIPELINE", "default")}),
                  flush=True)
            g1.destroy()
            Ap.free()
            Bp.free()
            tot_n += nnz
            continue
        pieces = []
        rest = Bp
        for q in range(a.pieces - 1):
            left, rest2 = rest.split_cols(rest.n // (a.pieces - q))
            pieces.append(left)
            rest = rest2
        pieces.append(rest)
        cbg.synchronize()
        best = None
        for _ in range(a.reps):
            dt = 0.0
            st = dict(flops=0, nnz=0, ms_symbolic=0.0, ms_numeric=0.0, n_big=0, n_slabs=0)
            nnz = 0
            for Bq in pieces:
                t0 = time.perf_counter()
                C = cbg.LocalHybridSpGEMM(Ap, Bq)
                cbg.synchronize()
                dt += time.perf_counter() - t0
                for k, v in cbg.last_stats().items():
                    st[k] += v
                nnz += C.nnz
                C.free()
                del C
            best = dt if best is None else min(best, dt)
        bytes_alg = 16 * st["flops"] + 12 * st["nnz"] + 32 * Bp.nnz + 8 * Bp.n
        ms = st["ms_symbolic"] + st["ms_numeric"]
        print(json.dumps({"rank": rk, "grid": a.grid, "scale": a.scale, "s": best, "nnz_C": nnz, "flops": st["flops"],
                          "nnzC_per_s": nnz / best, "big": st["n_big"], "slabs": st["n_slabs"],
                          "roofline_frac": bytes_alg / (ms * 1e-3) / 8e12}), flush=True)
        tot_f += st["flops"]
        tot_n += nnz
        Ap.free()
        for Bq in pieces:
            if Bq is not Bp:
                Bq.free()
        Bp.free()
    g = json.load(open(os.path.join(REPO, "tests", "golden", "golden.json")))["rmat"].get(f"s{a.scale}_ef{a.ef}")
    if g and len(ranks) == pr * pc:
        ok = (a.summa or g["symbolic"]["flops"] == tot_f) and g["symbolic"]["nnzC"] == tot_n
        print(json.dumps({"total_flops": tot_f, "total_nnzC": tot_n, "reference": g["symbolic"], "match": ok}))
        sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
