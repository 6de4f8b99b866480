#!/usr/bin/env python3
"""GalerkinNew (reference ReleaseTests/GalerkinNew.cpp:96-153) on the MI355X path.

  python tools/galerkin.py [--scale S] [--order K] [--iters N] [--minplus]      (one rank: 1x1 grid)
  torchrun ... tools/galerkin.py --scale 22                                     (square grids: 4, 9, 16 ranks)
  python tools/galerkin.py --scale 22 --minplus --rank-tiles 2x4               (per-rank work of a grid, one GPU)

A = Graph500 R-MAT (loops removed, so A is its own off-diagonal part L) plus a
seeded positive diagonal D (the driver's dvec); T = restriction operator
(cbg_restriction_tile, n x n/order); S = T^T (SpParMat::Transpose).
Checks the splitting approach S*(L*T) + (S*D)*T == S*(A*T) (SpParMat::operator==)
and times the full restriction (AT = PSpGEMM(A,T); SAT = PSpGEMM(S,AT)) and the
split one, like the reference; --minplus also times the full restriction on
MinPlusSRing.  Prints one JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def load():
    import importlib.util
    name = "combblas_spmm_test_amd"
    if name in sys.modules:
        return sys.modules[name]
    spec = importlib.util.spec_from_file_location(name, os.path.join(REPO, "combblas-spmm-test_amd", "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def diag_matrix(cbg, grid, d):
    """diagonal SpParMat with values d (host), block-distributed"""
    n = len(d)
    idx = np.arange(n)
    g = dict(m=n, n=n, cp=np.arange(n + 1, dtype=np.int64), jc=idx.astype(np.int32), ir=idx.astype(np.int32),
             val=np.asarray(d, np.float64))
    return cbg.SpParMat.from_global(grid, g)


def grid_of(cbg):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world == 1:
        class Self:
            def bcast(self, comm, arr, root):
                pass

            def allgather(self, comm, data):
                return data

        return cbg.CommGrid(0, 1, transport="host", host_comm=Self()), rank, world
    side = int(round(world ** 0.5))
    hc = cbg.TcpHostComm(rank, world, side, side, os.environ.get("MASTER_ADDR", "127.0.0.1"),
                         int(os.environ.get("MASTER_PORT", "29500")) + 1)
    uid = hc.bcast_object(cbg.CommGrid.unique_id() if rank == 0 else None, root=0)
    try:
        return cbg.CommGrid(rank, world, side, side, unique_id=uid, transport="rccl"), rank, world
    except cbg.CbgError:
        hc.allgather(0, b"0")
        return cbg.CommGrid(rank, world, side, side, transport="host", host_comm=hc), rank, world


def rank_tiles(cbg, a, A, T, S):
    """Every rank's local work of the full restriction on a pr x pc grid, timed on this
    one GPU: rank (r,c) multiplies A's block row r by T's block column c (AT(r,c)),
    then S's block row r by AT's block column c (SAT(r,c)), as the PANEL SUMMA does
    after its broadcasts (SpParMat::Owner blocks).  Communication is not included:
    these are the per-GPU compute times of a pr x pc run."""
    pr, pc = (int(x) for x in a.rank_tiles.lower().split("x"))

    def rows(t, lo, hi):
        top, bot = t.split_rows(hi)
        bot.free()
        _, mid = top.split_rows(lo)
        _.free()
        top.free()
        return mid

    def cols(t, lo, hi):
        left, right = t.split_cols(hi)
        right.free()
        _, mid = left.split_cols(lo)
        _.free()
        left.free()
        return mid

    def run(sr):
        per = []
        for c in range(pc):
            c0, c1 = cbg.block_range(T.gn, pc, c)
            Tc = cols(T.tile, c0, c1)
            ATc = cbg.LocalHybridSpGEMM(A.tile, Tc, sr)  # AT's block column c (all its rows)
            for r in range(pr):
                r0, r1 = cbg.block_range(A.gm, pr, r)
                s0, s1 = cbg.block_range(S.gm, pr, r)
                Ar, Sr = rows(A.tile, r0, r1), rows(S.tile, s0, s1)
                cbg.synchronize()
                t0 = time.perf_counter()
                X = cbg.LocalHybridSpGEMM(Ar, Tc, sr)
                Y = cbg.LocalHybridSpGEMM(Sr, ATc, sr)
                cbg.synchronize()
                per.append(dict(rank=[r, c], seconds=time.perf_counter() - t0, nnz_AT=X.nnz, nnz_SAT=Y.nnz))
                for t in (X, Y, Ar, Sr):
                    t.free()
            ATc.free()
            Tc.free()
        return per

    out = {"grid": "%dx%d" % (pr, pc), "note": "per-rank local products on one GPU, no communication"}
    for name, sr in (("plus", cbg.PlusTimesSRing), ("minplus", cbg.MinPlusSRing)):
        run(sr)  # warm-up
        per = run(sr)
        out[name] = {"max_rank_s": max(x["seconds"] for x in per), "mean_rank_s": sum(x["seconds"] for x in per) / len(per),
                     "nnz_SAT": sum(x["nnz_SAT"] for x in per), "ranks": per}
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--scale", type=int, default=18)
    p.add_argument("--order", type=int, default=2)
    p.add_argument("--iters", type=int, default=3)
    p.add_argument("--minplus", action="store_true")
    p.add_argument("--only-full", action="store_true",
                   help="time the full restriction only (kernel traces: its multiplies are the last dispatches)")
    p.add_argument("--rank-tiles", default=None,
                   help="RxC: time every rank's local products of a RxC grid on this one GPU (no communication)")
    a = p.parse_args()
    cbg = load()
    cbg.lib().cbg_set_device(int(os.environ.get("LOCAL_RANK", "0")) % max(1, cbg.device_count()))
    grid, rank, world = grid_of(cbg)
    n = 1 << a.scale
    L = cbg.SpParMat.rmat(grid, a.scale)                  # loops removed: off-diagonal
    d = np.random.default_rng(7).uniform(0.5, 1.5, n)     # the driver's dvec
    A = L.copy()
    A += diag_matrix(cbg, grid, d)                        # A = L + D
    T = cbg.SpParMat.restriction(grid, a.scale, a.order)
    S = T.copy()
    S.Transpose()                                         # S = T^T
    # splitting check (GalerkinNew.cpp:105-128)
    AT = cbg.PSpGEMM(A, T)
    SAT = cbg.PSpGEMM(S, AT)
    LT = cbg.PSpGEMM(L, T)
    SLT = cbg.PSpGEMM(S, LT)
    SD = S.copy()
    SD.DimApply(cbg.Column, d)                            # scale columns of S
    SDT = cbg.PSpGEMM(SD, T)
    SLT += SDT
    split_ok = SLT == SAT
    if rank == 0:
        print("Splitting approach is correct" if split_ok else "Error in splitting, go fix it", file=sys.stderr)
    nnz_sat = SAT.getnnz()

    def timed(fn):
        grid.barrier()
        cbg.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            fn()
        cbg.synchronize()
        grid.barrier()
        return grid.allreduce_max((time.perf_counter() - t0) / a.iters)

    def full(sr=cbg.PlusTimesSRing):
        X = cbg.PSpGEMM(A, T, sr)
        Y = cbg.PSpGEMM(S, X, sr)
        X.tile.free()
        Y.tile.free()

    def split():
        X = cbg.PSpGEMM(L, T)
        Y = cbg.PSpGEMM(S, X)
        W = cbg.PSpGEMM(SD, T)
        Y += W
        for M in (X, Y, W):
            M.tile.free()

    # algorithmic bytes of the full restriction (per local multiply:
    # 16 F + 12 nnz(C) + 32 nnz(B) + 8 ncol(B)), from the two products' statistics
    def alg_bytes():
        X = cbg.PSpGEMM(A, T)
        s1 = cbg.last_stats()
        Y = cbg.PSpGEMM(S, X)
        s2 = cbg.last_stats()
        b = (16 * s1["flops"] + 12 * s1["nnz"] + 32 * T.tile.nnz + 8 * T.tile.n +
             16 * s2["flops"] + 12 * s2["nnz"] + 32 * X.tile.nnz + 8 * X.tile.n)
        X.tile.free()
        Y.tile.free()
        return b, s1["flops"] + s2["flops"]

    bytes_alg, flops_full = alg_bytes()
    t_full = timed(full)
    t_split = None if a.only_full else timed(split)
    out = {"workload": "GalerkinNew R*A*R^T (R-MAT scale %d, restriction order %d)" % (a.scale, a.order),
           "grid": "%dx%d" % (grid.grid_rows, grid.grid_cols), "n_gpus": world, "nnz_A": A.getnnz(),
           "nnz_T": T.getnnz(), "nnz_SAT": nnz_sat, "splitting_correct": bool(split_ok),
           "full_restriction_s": t_full, "split_restriction_s": t_split,
           "roofline_full": {"bytes_alg_rank0": bytes_alg, "flops_rank0": flops_full,
                             "achieved_GBps": bytes_alg / t_full / 1e9, "peak_GBps": 8000.0,
                             "frac": bytes_alg / t_full / 8e12,
                             "note": "both products' algorithmic bytes over the full restriction's wall time "
                                     "(host-timed, max over ranks)"}}
    if a.minplus:
        out["full_restriction_minplus_s"] = timed(lambda: full(cbg.MinPlusSRing))
    if a.rank_tiles and world == 1:
        out["rank_tiles"] = rank_tiles(cbg, a, A, T, S)
    if rank == 0:
        print(json.dumps(out), flush=True)
    grid.destroy()
    if not split_ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
