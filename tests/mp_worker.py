"""Worker for multi-process SUMMA tests (launched by torch.distributed.run).

usage: mp_worker.py <mode> <grid_rows> <grid_cols> <case>
  mode "gpu": every rank runs the HIP SUMMA over the host (gloo) transport on the
              shared GPU and checks the global digest against the reference's.
  mode "cpu": transport plumbing only (no device work): bcast/allgather through
              GlooHostComm and the block distribution of the golden matrix.
  mode "rccl": as "gpu", but the grid's collectives run over RCCL with several
              ranks.  The ranks share the one GPU of a development box, which
              RCCL refuses for ranks it sees on one host ("Duplicate GPU"), so
              every rank gets its own NCCL_HOSTID: RCCL then treats them as
              separate hosts and moves data with its socket transport over
              loopback.  Every RCCL call of the SUMMA (communicator split,
              grouped broadcasts, send/recv of Transpose, allgathers, the error
              agreement and abort) runs with more than one rank this way.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from conftest import load_cbg  # noqa: E402
from helpers import digest, golden, load_npz  # noqa: E402


def add_digests(ds):
    hs = sum(int(d["hs"], 16) for d in ds) % (1 << 64)
    hv = sum(int(d["hv"], 16) for d in ds) % (1 << 64)
    return dict(nnz=sum(d["nnz"] for d in ds), hs="%016x" % hs, hv="%016x" % hv, vsum=sum(d["vsum"] for d in ds))


def main():
    mode, pr, pc, case = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    cbg = load_cbg()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    assert world == pr * pc
    port = int(os.environ["MASTER_PORT"]) + 1
    if case == "fault" and rank == world - 1:
        # its 2nd (PANEL) and 3rd (STAGED) SUMMA call, or the first two (CBG_FAULT_FIRST=1)
        os.environ["CBG_FAULT_INJECT"] = "%d:%s" % (rank, "0,1" if os.environ.get("CBG_FAULT_FIRST") == "1" else "1,2")
    if case == "redist_fault" and rank == world - 1:
        os.environ["CBG_FAULT_INJECT_REDIST"] = "%d:0,1" % rank  # its first Transpose and first BlockSplit
    if mode == "rccl":
        os.environ["NCCL_HOSTID"] = "cbg-test-rank-%d" % rank
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ.setdefault("NCCL_IB_DISABLE", "1")
    if mode in ("gpu", "cputcp", "rccl"):
        # GPU processes never import torch (a second HIP runtime corrupts the heap)
        if mode != "cputcp":
            cbg.lib()
        hc = cbg.TcpHostComm(rank, world, pr, pc, "127.0.0.1", port)

        class _D:
            @staticmethod
            def barrier():
                hc.allgather(0, b"x")
        dist = _D
    else:
        import torch.distributed as dist
        dist.init_process_group("gloo")
        hc = cbg.GlooHostComm(pr, pc)
    G = golden()

    def make_grid():
        if mode != "rccl":
            return cbg.CommGrid(rank, world, pr, pc, transport="host", host_comm=hc)
        uid = hc.bcast_object(cbg.CommGrid.unique_id() if rank == 0 else None, root=0)
        g = cbg.CommGrid(rank, world, pr, pc, unique_id=uid, transport="rccl")
        if rank == 0:
            print("transport rccl, %d ranks" % world, flush=True)
        return g

    if case == "agree":
        # collective error agreement without a device: a code raised on one rank
        # reaches every rank; then a rank that leaves makes its peers' next
        # collective fail (CBG_ERR_RCCL) instead of hanging
        grid = make_grid()
        ok = grid.agree(3102 if rank == world - 1 else 0) == 3102 and grid.agree(0) == 0
        dist.barrier()
        if rank == world - 1:
            print("MPOK" if ok else "AGREE FAILED", flush=True)
            os._exit(0)  # leave without a goodbye: the peers must not hang
        try:
            grid.agree(0)
            ok = False
        except cbg.CbgError as e:
            ok = ok and e.code == 3101
        print("MPOK" if ok else "PEER-LOSS NOT DETECTED", flush=True)
        os._exit(0)
    if case == "fault":
        # CBG_FAULT_INJECT makes the last rank's first local multiply fail like
        # an OOM: every rank must return 3102 (no hang), then the grid still works
        Ah = load_npz("rmat_s10_ef16_A.npz")
        gd = G["rmat"]["s10_ef16"]["C_local_plus"]
        grid = make_grid()
        Ad = cbg.SpParMat.from_global(grid, Ah)
        Bd = cbg.SpParMat.from_global(grid, Ah)
        ok = True
        r0, _ = cbg.block_range(Ah["m"], pr, grid.prow)
        c0, _ = cbg.block_range(Ah["n"], pc, grid.pcol)
        r1, _ = cbg.block_range(Ah["m"], pr, grid.prow)[1], 0
        c1 = cbg.block_range(Ah["n"], pc, grid.pcol)[1]
        Cg = load_npz("rmat_s10_ef16_C_local_plus.npz")
        d0 = digest(cbg.sub_tile(Cg, r0, r1, c0, c1), r0, c0)  # this rank's tile of the golden C
        first = os.environ.get("CBG_FAULT_FIRST") == "1"
        if not first:
            C0 = cbg.Mult_AnXBn_DoubleBuff(Ad, Bd, exec_mode=1)  # call 0: a good STAGED multiply
            dd = C0.tile.digest(r0, c0)
            if dd != d0:
                print(rank, "first multiply differs", dd, d0, flush=True)
            C0.tile.free()
        for ex in (0, 1):
            try:
                cbg.Mult_AnXBn_DoubleBuff(Ad, Bd, exec_mode=ex)
                ok = False
                print(rank, "no error raised", flush=True)
            except cbg.CbgError as e:
                ok = ok and e.code == 3102
                if e.code != 3102:
                    print(rank, "wrong code", e, flush=True)
        C = cbg.Mult_AnXBn_DoubleBuff(Ad, Bd)  # the next call succeeds on the same grid
        d1 = C.tile.digest(r0, c0)
        if d1 != d0:
            print(rank, "final tile differs from the golden tile", d1, d0, flush=True)
            ok = False
        import pickle
        alld = [pickle.loads(b) for b in _chunks(hc.allgather(0, _pad(pickle.dumps(C.tile.digest(r0, c0)))))]
        tot = add_digests(alld)
        ok = ok and tot["nnz"] == gd["nnz"] and tot["hs"] == gd["hs"] and tot["hv"] == gd["hv"]
        grid.destroy()
        dist.barrier()
        if rank == 0:
            print("MPOK" if ok else f"FAULT TEST FAILED {tot}", flush=True)
        return
    if case == "rmat18":
        # scale-18 R-MAT A*A on the grid, generated per tile on device: PANEL and
        # STAGED (DoubleBuff + Synch) against the reference's digest, rows ordered
        import pickle
        grid = make_grid()
        Ad = cbg.SpParMat.rmat(grid, 18)
        Bd = cbg.SpParMat.rmat(grid, 18)
        gd = G["rmat"]["s18_ef16"]["C_local_plus"]
        r0, _ = cbg.block_range(Ad.gm, pr, grid.prow)
        c0, _ = cbg.block_range(Bd.gn, pc, grid.pcol)
        ok = True
        for algo, ex in (("doublebuff", 1), ("synch", 1), ("doublebuff", 0)):
            f = cbg.Mult_AnXBn_DoubleBuff if algo == "doublebuff" else cbg.Mult_AnXBn_Synch
            C = f(Ad, Bd, exec_mode=ex)
            d = C.tile.digest(r0, c0)
            C.tile.free()
            alld = [pickle.loads(b) for b in _chunks(hc.allgather(0, _pad(pickle.dumps(d))))]
            tot = add_digests(alld)
            uns = sum(x["unsorted"] for x in alld)
            good = tot["nnz"] == gd["nnz"] and tot["hs"] == gd["hs"] and tot["hv"] == gd["hv"] and uns == 0
            if rank == 0:
                print(algo, ex, "OK" if good else f"BAD {tot} unsorted={uns} vs {gd}", flush=True)
            ok = ok and good
        # the grid branch of MemEfficientSpGEMM's phase planner (ParFriends.h:482-535):
        # perProcessMemory = 1 GB asks for several phases on every rank of this
        # grid (C = 5.1 GB); the count is agreed (equal on every rank), the plan's
        # flops are this rank's product flops, and the streamed phases add up to
        # the reference's digest
        parts = []
        cbg.MemEfficientSpGEMM(Ad, Bd, cbg.PHASES_AUTO, perProcessMemory=1,
                               on_phase=lambda ph, off, t: parts.append(t.digest(r0, c0 + off)))
        plan, st = cbg.phase_plan(), cbg.last_stats()
        mine = add_digests(parts)
        mine["phases"], mine["flops_ok"] = plan["phases"], plan["flops"] == st["flops"]
        alld = [pickle.loads(b) for b in _chunks(hc.allgather(0, _pad(pickle.dumps(mine))))]
        tot = add_digests(alld)
        good = (tot["nnz"] == gd["nnz"] and tot["hs"] == gd["hs"] and tot["hv"] == gd["hv"]
                and len({x["phases"] for x in alld}) == 1 and alld[0]["phases"] > 1 and all(x["flops_ok"] for x in alld)
                and plan["automatic"] == 1)
        if rank == 0:
            print("planned phases", alld[0]["phases"], "OK" if good else f"BAD {alld} vs {gd}", flush=True)
        ok = ok and good
        grid.destroy()
        dist.barrier()
        if rank == 0 and ok:
            print("MPOK", flush=True)
        return
    if case == "multtest":
        # ReleaseTests/MultTest.cpp SpGEMM part on a pr x pc grid: ParallelReadMM of
        # A, B, CControl; Synch / DoubleBuff / phased products == CControl
        grid = make_grid()
        mm = os.path.join(HERE, "golden", "sevenvertex.mtx")
        A = cbg.SpParMat.ParallelReadMM(grid, mm)
        B = cbg.SpParMat.ParallelReadMM(grid, mm)
        CC = cbg.SpParMat.ParallelReadMM(grid, os.path.join(HERE, "golden", "sevenvertex_C.mtx"))
        ok = (cbg.Mult_AnXBn_Synch(A, B) == CC) and (cbg.Mult_AnXBn_DoubleBuff(A, B) == CC)
        ok = ok and (cbg.MemEfficientSpGEMM(A, B, 2) == CC)
        grid.destroy()
        dist.barrier()
        if rank == 0:
            print("MPOK" if ok else "MULTTEST FAILED", flush=True)
        return
    if case == "galerkin":
        # GalerkinNew on a square grid: distributed Transpose (complement-rank
        # exchange), PSpGEMMs, DimApply, +=, operator==; SAT digest vs the oracle
        from helpers import add_diag_host, oracle_local, restriction_host, transpose_host
        import pickle
        grid = make_grid()
        scale, n = 10, 1 << 10
        dv = np.random.default_rng(7).uniform(0.5, 1.5, n)
        Lh = load_npz("rmat_s10_ef16_A.npz")
        Ah = add_diag_host(Lh, dv)
        L = cbg.SpParMat.from_global(grid, Lh)
        A = cbg.SpParMat.from_global(grid, Ah)
        T = cbg.SpParMat.restriction(grid, scale, 2)
        S = T.copy()
        S.Transpose()
        SAT = cbg.PSpGEMM(S, cbg.PSpGEMM(A, T))
        SLT = cbg.PSpGEMM(S, cbg.PSpGEMM(L, T))
        SD = S.copy()
        SD.DimApply(cbg.Column, dv)
        SLT += cbg.PSpGEMM(SD, T)
        ok = SLT == SAT
        r0, _ = cbg.block_range(SAT.gm, pr, grid.prow)
        c0, _ = cbg.block_range(SAT.gn, pc, grid.pcol)
        d = SAT.tile.digest(r0, c0)
        alld = [pickle.loads(b) for b in _chunks(hc.allgather(0, _pad(pickle.dumps(d))))]
        tot = add_digests(alld)
        Th = restriction_host(scale, 2)
        ref = digest(oracle_local(transpose_host(Th), oracle_local(Ah, Th)))
        ok = ok and tot["nnz"] == ref["nnz"] and tot["hs"] == ref["hs"]
        ok = ok and abs(tot["vsum"] - ref["vsum"]) < 1e-9 * abs(ref["vsum"])
        # min-plus S*A*T on the grid (config 5's semiring): exact, digest == oracle
        mp = cbg.MinPlusSRing
        SATm = cbg.PSpGEMM(S, cbg.PSpGEMM(A, T, mp), mp)
        dm = SATm.tile.digest(r0, c0)
        alld = [pickle.loads(b) for b in _chunks(hc.allgather(0, _pad(pickle.dumps(dm))))]
        totm = add_digests(alld)
        refm = digest(oracle_local(transpose_host(Th), oracle_local(Ah, Th, sr="minplus"), sr="minplus"))
        okm = totm["nnz"] == refm["nnz"] and totm["hs"] == refm["hs"] and totm["hv"] == refm["hv"]
        if not okm and rank == 0:
            print("GALERKIN MINPLUS", totm, refm, flush=True)
        ok = ok and okm
        grid.destroy()
        dist.barrier()
        if rank == 0:
            print("MPOK" if ok else f"GALERKIN FAILED {tot} vs {ref}", flush=True)
        return
    if case == "blockspgemm":
        # ReleaseTests/BlockedSpGEMM.cpp on a pr x pc grid: BlockSplit redistributes
        # every block over the whole grid (standard layout), the C blocks at their
        # offsets add up to the golden A*A digest
        import pickle
        grid = make_grid()
        Ah = load_npz("rmat_s10_ef16_A.npz")
        A = cbg.SpParMat.from_global(grid, Ah)
        B = cbg.SpParMat.from_global(grid, Ah)
        ok = True
        blocks = A.BlockSplit(3, 2)
        roff, coff = cbg._block_offsets(Ah["m"], 3), cbg._block_offsets(Ah["n"], 2)
        for i in range(3):
            for j in range(2):
                X = blocks[i][j]
                r0, r1 = cbg.block_range(X.gm, pr, grid.prow)
                c0, c1 = cbg.block_range(X.gn, pc, grid.pcol)
                want = cbg.sub_tile(Ah, roff[i] + r0, roff[i] + r1, coff[j] + c0, coff[j] + c1)
                h = X.tile.to_host()
                ok = ok and all(np.array_equal(np.asarray(h[k]), np.asarray(want[k])) for k in ("cp", "jc", "ir", "val"))
        bs = cbg.BlockSpGEMM(A, B, 3, 2)
        ds = []
        while bs.hasNext():
            C, ro, co = bs.getNextBlock()
            r0, _ = cbg.block_range(C.gm, pr, grid.prow)
            c0, _ = cbg.block_range(C.gn, pc, grid.pcol)
            ds.append(C.tile.digest(ro + r0, co + c0))
        alld = [pickle.loads(b) for b in _chunks(hc.allgather(0, _pad(pickle.dumps(add_digests(ds)))))]
        tot = add_digests(alld)
        gd = G["rmat"]["s10_ef16"]["C_local_plus"]
        ok = ok and tot["nnz"] == gd["nnz"] and tot["hs"] == gd["hs"] and tot["hv"] == gd["hv"]
        grid.destroy()
        dist.barrier()
        if rank == 0:
            print("MPOK" if ok else f"BLOCKSPGEMM FAILED {tot} vs {gd}", flush=True)
        return
    if case == "narrow":
        # B tiles of uneven, narrow widths (31 columns on a 1 x 2 grid: 15 and 16):
        # the pipeline's piece count is agreed from the narrowest tile, so every
        # rank makes the same collectives (CBG_PIPELINE from the test: unset, 2, 1/4)
        from helpers import oracle_local
        rng = np.random.default_rng(5)
        n = 31
        dense = (rng.random((n, n)) < 0.3) * rng.uniform(-1, 1, (n, n))
        cols, rows = np.nonzero(dense.T)
        H = dict(m=n, n=n, cp=np.searchsorted(cols, np.arange(n + 1)).astype(np.int64), jc=np.arange(n, dtype=np.int32),
                 ir=rows.astype(np.int32), val=dense.T[cols, rows].astype(np.float64))
        keep = np.diff(H["cp"]) > 0
        H["jc"] = H["jc"][keep]
        H["cp"] = np.append(H["cp"][:-1][keep], H["cp"][-1]).astype(np.int64)
        from helpers import abs_tile, assert_tiles_equal
        ref = oracle_local(H, H)
        bound = oracle_local(abs_tile(H), abs_tile(H))
        grid = make_grid()
        Ad = cbg.SpParMat.from_global(grid, H)
        Bd = cbg.SpParMat.from_global(grid, H)
        r0, r1 = cbg.block_range(n, pr, grid.prow)
        c0, c1 = cbg.block_range(n, pc, grid.pcol)
        want, wb = cbg.sub_tile(ref, r0, r1, c0, c1), cbg.sub_tile(bound, r0, r1, c0, c1)
        ok = True
        for ex in (0, 1):
            for f in (cbg.Mult_AnXBn_DoubleBuff, cbg.Mult_AnXBn_Synch):
                C = f(Ad, Bd, exec_mode=ex)
                try:
                    assert_tiles_equal(C.tile.to_host(), want, rtol=1e-12, bound=wb["val"])
                except AssertionError as e:
                    print(rank, "narrow", ex, f.__name__, e, flush=True)
                    ok = False
                C.tile.free()
        Cp = cbg.MemEfficientSpGEMM(Ad, Bd, 3)
        try:
            assert_tiles_equal(Cp.tile.to_host(), want, rtol=1e-12, bound=wb["val"])
        except AssertionError as e:
            print(rank, "narrow phased", e, flush=True)
            ok = False
        oks = hc.allgather(0, b"1" if ok else b"0")
        grid.destroy()
        dist.barrier()
        if rank == 0:
            print("MPOK" if oks == b"1" * world else "NARROW FAILED %r" % oks, flush=True)
        return
    if case == "mismatch":
        # a tile off the block layout (the last rank's A tile one column short):
        # PANEL and STAGED both return CBG_ERR_DIMMISMATCH on every rank, and the
        # grid still multiplies afterwards
        Ah = load_npz("rmat_s10_ef16_A.npz")
        gd = G["rmat"]["s10_ef16"]["C_local_plus"]
        grid = make_grid()
        Ad = cbg.SpParMat.from_global(grid, Ah)
        Bd = cbg.SpParMat.from_global(grid, Ah)
        bad = Ad
        if rank == world - 1:
            left, right = Ad.tile.split_cols(Ad.tile.n - 1)
            right.free()
            bad = cbg.SpParMat(left, grid, Ad.gm, Ad.gn)
        ok = True
        for ex in (0, 1):
            try:
                cbg.Mult_AnXBn_DoubleBuff(bad, Bd, exec_mode=ex)
                ok = False
                print(rank, "no error", ex, flush=True)
            except cbg.CbgError as e:
                if e.code != cbg.DIMMISMATCH:
                    ok = False
                    print(rank, "wrong code", ex, e, flush=True)
        C = cbg.Mult_AnXBn_DoubleBuff(Ad, Bd)
        r0, _ = cbg.block_range(Ah["m"], pr, grid.prow)
        c0, _ = cbg.block_range(Ah["n"], pc, grid.pcol)
        import pickle
        alld = [pickle.loads(b) for b in _chunks(hc.allgather(0, _pad(pickle.dumps(C.tile.digest(r0, c0)))))]
        tot = add_digests(alld)
        ok = ok and tot["nnz"] == gd["nnz"] and tot["hs"] == gd["hs"] and tot["hv"] == gd["hv"]
        oks = hc.allgather(0, b"1" if ok else b"0")
        grid.destroy()
        dist.barrier()
        if rank == 0:
            print("MPOK" if oks == b"1" * world else "MISMATCH FAILED %r" % oks, flush=True)
        return
    if case == "redist_fault":
        # CBG_FAULT_INJECT_REDIST makes the last rank's first Transpose and first
        # BlockSplit fail their receive-buffer allocation: every rank returns
        # CBG_ERR_OOM (no rank left in a send/recv or broadcast), then both work
        from helpers import transpose_host
        Ah = load_npz("rmat_s10_ef16_A.npz")
        grid = make_grid()
        ok = True
        for what in ("transpose", "blocksplit"):
            X = cbg.SpParMat.from_global(grid, Ah)
            try:
                X.Transpose() if what == "transpose" else X.BlockSplit(3, 1)
                ok = False
                print(rank, what, "no error", flush=True)
            except cbg.CbgError as e:
                if e.code != cbg.OOM:
                    ok = False
                    print(rank, what, "wrong code", e, flush=True)
            X.tile.free()
        X = cbg.SpParMat.from_global(grid, Ah)
        X.Transpose()
        Th = transpose_host(Ah)
        r0, r1 = cbg.block_range(Th["m"], pr, grid.prow)
        c0, c1 = cbg.block_range(Th["n"], pc, grid.pcol)
        from helpers import assert_tiles_equal
        try:
            assert_tiles_equal(X.tile.to_host(), cbg.sub_tile(Th, r0, r1, c0, c1))
        except AssertionError as e:
            ok = False
            print(rank, "transpose after the fault", e, flush=True)
        blocks = cbg.SpParMat.from_global(grid, Ah).BlockSplit(3, 1)
        roff = cbg._block_offsets(Ah["m"], 3)
        for i in range(3):
            Xb = blocks[i][0]
            a0, a1 = cbg.block_range(Xb.gm, pr, grid.prow)
            b0, b1 = cbg.block_range(Xb.gn, pc, grid.pcol)
            h = Xb.tile.to_host()
            want = cbg.sub_tile(Ah, roff[i] + a0, roff[i] + a1, b0, b1)
            ok = ok and all(np.array_equal(np.asarray(h[k]), np.asarray(want[k])) for k in ("cp", "jc", "ir", "val"))
        oks = hc.allgather(0, b"1" if ok else b"0")
        grid.destroy()
        dist.barrier()
        if rank == 0:
            print("MPOK" if oks == b"1" * world else "REDIST FAULT FAILED %r" % oks, flush=True)
        return
    if case.startswith("rmat"):
        A = load_npz("rmat_s10_ef16_A.npz")
        B = A
        gd = G["rmat"]["s10_ef16"]["C_local_plus"]
    else:
        A = load_npz("largeseq_A.npz")
        B = load_npz("largeseq_B.npz")
        gd = G["files"]["largeseq"]["C_local_plus"]
    if mode in ("cpu", "cputcp"):
        # tiles of the block distribution cover A exactly once
        r0, r1 = cbg.block_range(A["m"], pr, hc.prow)
        c0, c1 = cbg.block_range(A["n"], pc, hc.pcol)
        t = cbg.sub_tile(A, r0, r1, c0, c1)
        d = digest(t, r0, c0)
        import pickle
        alld = [pickle.loads(b) for b in _chunks(hc.allgather(0, _pad(pickle.dumps(d))))]
        tot = add_digests(alld)
        ga = G["rmat"]["s10_ef16"]["A"] if case.startswith("rmat") else G["files"]["largeseq"]["A"]
        assert tot["nnz"] == ga["nnz"] and tot["hs"] == ga["hs"] and tot["hv"] == ga["hv"], (tot, ga)
        # row / column broadcasts reach exactly the grid row / column
        buf = np.full(16, 255, np.uint8)
        if hc.pcol == 0:
            buf[:] = hc.prow
        hc.bcast(1, buf, 0)
        assert np.all(buf == hc.prow)
        buf[:] = 255
        if hc.prow == pr - 1:
            buf[:] = 100 + hc.pcol
        hc.bcast(2, buf, pr - 1)
        assert np.all(buf == 100 + hc.pcol)
        got = hc.allgather(1, bytes([hc.rank]))
        assert list(got) == [hc.prow * pc + c for c in range(pc)]
        got = hc.allgather(2, bytes([hc.rank]))
        assert list(got) == [r * pc + hc.pcol for r in range(pr)]
        dist.barrier()
        if rank == 0:
            print("MPOK", flush=True)
        return
    grid = make_grid()
    Ad = cbg.SpParMat.from_global(grid, A)
    Bd = cbg.SpParMat.from_global(grid, B)
    ok = True
    for algo in ("doublebuff", "synch"):
        for ex in (0, 1):  # PANEL (pipelined) and STAGED (any grid shape)
            f = cbg.Mult_AnXBn_DoubleBuff if algo == "doublebuff" else cbg.Mult_AnXBn_Synch
            C = f(Ad, Bd, exec_mode=ex)
            if ex == 0 and rank == 0:
                print("pieces %d" % cbg.summa_info()["pieces"], flush=True)
            r0, _ = cbg.block_range(A["m"], pr, grid.prow)
            c0, _ = cbg.block_range(B["n"], pc, grid.pcol)
            d = C.tile.digest(r0, c0)
            import pickle
            alld = [pickle.loads(b) for b in _chunks(hc.allgather(0, _pad(pickle.dumps(d))))]
            tot = add_digests(alld)
            good = tot["nnz"] == gd["nnz"] and tot["hs"] == gd["hs"] and all(x["unsorted"] == 0 for x in alld)
            if case.startswith("rmat"):
                good = good and tot["hv"] == gd["hv"]
            else:
                # every entry of this rank's tile within 1e-12 (|A||B|)_ij of the
                # reference's product (the single-rank tests' bound)
                from helpers import abs_tile, assert_tiles_equal, oracle_local
                r1_ = cbg.block_range(A["m"], pr, grid.prow)[1]
                c1_ = cbg.block_range(B["n"], pc, grid.pcol)[1]
                if "bound" not in locals():
                    bound = oracle_local(abs_tile(A), abs_tile(B))
                    Cg = load_npz("largeseq_C_local_plus.npz")
                try:
                    assert_tiles_equal(C.tile.to_host(), cbg.sub_tile(Cg, r0, r1_, c0, c1_), rtol=1e-12,
                                       bound=cbg.sub_tile(bound, r0, r1_, c0, c1_)["val"])
                    mine_ok = b"1"
                except AssertionError as e:
                    print(rank, algo, ex, "per-entry", e, flush=True)
                    mine_ok = b"0"
                good = good and hc.allgather(0, mine_ok) == b"1" * world
            if rank == 0:
                print(algo, ex, "OK" if good else f"BAD {tot} vs {gd}", flush=True)
            ok = ok and good
            C.tile.free()
    # MemEfficientSpGEMM phases: concatenated result equals the unphased one
    # (SpParMat::operator==, AND over the grid), streamed phases add up to it
    import pickle
    C1 = cbg.Mult_AnXBn_DoubleBuff(Ad, Bd)
    Cp = cbg.MemEfficientSpGEMM(Ad, Bd, 3)
    same = (Cp == C1)
    r0, _ = cbg.block_range(A["m"], pr, grid.prow)
    c0, _ = cbg.block_range(B["n"], pc, grid.pcol)
    parts = []
    cbg.MemEfficientSpGEMM(Ad, Bd, 3, on_phase=lambda ph, off, t: parts.append(t.digest(r0, c0 + off)))
    mine = add_digests(parts)
    alld = [pickle.loads(b) for b in _chunks(hc.allgather(0, _pad(pickle.dumps(mine))))]
    tot = add_digests(alld)
    good = same and tot["nnz"] == gd["nnz"] and tot["hs"] == gd["hs"]
    if rank == 0:
        print("phased", "OK" if good else f"BAD same={same} {tot} vs {gd}", flush=True)
    ok = ok and good
    # phases = 1 with a consumer: the SUMMA's pipeline pieces (2 on a grid when the
    # adaptive pipeline keeps them) are all handed over as phase 0, at their offsets
    seen = []
    cbg.MemEfficientSpGEMM(Ad, Bd, 1, on_phase=lambda ph, off, t: seen.append((ph, t.digest(r0, c0 + off))))
    mine = add_digests([d for _, d in seen])
    mine["ph"] = sorted({ph for ph, _ in seen})
    alld = [pickle.loads(b) for b in _chunks(hc.allgather(0, _pad(pickle.dumps(mine))))]
    tot = add_digests(alld)
    good = tot["nnz"] == gd["nnz"] and tot["hs"] == gd["hs"] and all(x["ph"] == [0] for x in alld)
    if rank == 0:
        print("phases=1 consumer pieces", len(seen), "OK" if good else f"BAD {alld}", flush=True)
    ok = ok and good
    C1.tile.free()
    Cp.tile.free()
    grid.destroy()
    dist.barrier()
    if rank == 0 and ok:
        print("MPOK", flush=True)


PAD = 512


def _pad(b):
    assert len(b) <= PAD
    return b + b" " * (PAD - len(b))


def _chunks(b):
    return [b[i:i + PAD].rstrip(b" ") for i in range(0, len(b), PAD)]


if __name__ == "__main__":
    main()
