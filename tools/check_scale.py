#!/usr/bin/env python3
"""One-off parity check at scales beyond the golden digests: the HIP C = A*A
digest against the CPU oracle's (test infrastructure) for R-MAT `--scale`.

  python tools/check_scale.py --scale 20 [--sr minplus]      # local multiply
  python tools/check_scale.py --scale 22 --phases 4          # MemEfficientSpGEMM, digests streamed
  python tools/check_scale.py --scale 22 --ef 8 --oracle-pieces 4   # one resident C on the GPU (109 GB)

Digests (tests/helpers.py digest) add over column pieces, so the phased GPU
run and the oracle (one B column piece at a time) are compared on the whole C
without holding it.  Host memory: ~150 GB at scale 20-21, ~100 GB per piece
at scale 22 with 4 pieces; run on the GPU box.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))


def chunked_digest(t, coff=0, chunk=1 << 27):
    """helpers.digest(t, 0, coff) over column blocks (bounded temporaries)."""
    from helpers import _mix64
    cp, jc, ir, val = t["cp"], t["jc"], t["ir"], t["val"]
    hs = np.uint64(0)
    hv = np.uint64(0)
    vsum = 0.0
    nzc = len(jc)
    c0 = 0
    unsorted = 0
    while c0 < nzc:
        c1 = int(np.searchsorted(cp, cp[c0] + chunk, side="right")) - 1
        c1 = min(max(c1, c0 + 1), nzc)
        a, b = int(cp[c0]), int(cp[c1])
        col = np.repeat(jc[c0:c1].astype(np.uint64) + np.uint64(coff), np.diff(cp[c0:c1 + 1]))
        row = ir[a:b].astype(np.uint64)
        h = _mix64((col << np.uint64(32)) | row)
        vb = _mix64(np.ascontiguousarray(val[a:b], dtype=np.float64).view(np.uint64))
        with np.errstate(over="ignore"):
            hs = hs + np.sum(h, dtype=np.uint64)
            hv = hv + np.sum(h * vb, dtype=np.uint64)
        vsum += float(np.sum(val[a:b]))
        d = np.diff(ir[a:b].astype(np.int64))
        same = np.diff(col.astype(np.int64)) == 0
        unsorted += int(np.sum((d <= 0) & same))
        del col, row, h, vb, d, same
        c0 = c1
    return dict(nnz=int(len(ir)), nzc=int(nzc), hs="%016x" % int(hs), hv="%016x" % int(hv), vsum=vsum,
                unsorted=unsorted)


def add(ds):
    return dict(nnz=sum(d["nnz"] for d in ds), nzc=sum(d["nzc"] for d in ds),
                hs="%016x" % (sum(int(d["hs"], 16) for d in ds) % (1 << 64)),
                hv="%016x" % (sum(int(d["hv"], 16) for d in ds) % (1 << 64)),
                vsum=sum(d["vsum"] for d in ds), unsorted=sum(d.get("unsorted", 0) for d in ds))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--scale", type=int, default=20)
    p.add_argument("--threads", type=int, default=16)
    p.add_argument("--sr", choices=["plus", "minplus"], default="plus")
    p.add_argument("--phases", type=int, default=1)
    p.add_argument("--ef", type=int, default=16)
    p.add_argument("--oracle-pieces", type=int, default=None,
                   help="B column pieces of the oracle run (default: --phases); bounds host memory")
    a = p.parse_args()
    if a.oracle_pieces is None:
        a.oracle_pieces = a.phases
    from conftest import load_cbg
    cbg = load_cbg()
    cbg.lib().cbg_set_device(0)
    t0 = time.time()
    A = cbg.rmat_tile(a.scale, a.ef)
    B = cbg.rmat_tile(a.scale, a.ef)
    if a.phases <= 1:
        C = cbg.LocalHybridSpGEMM(A, B, a.sr)
        gd = C.digest()
        C.free()
    else:
        class Self:
            def bcast(self, comm, arr, root):
                pass

            def allgather(self, comm, data):
                return data

        g = cbg.CommGrid(0, 1, transport="host", host_comm=Self())
        nv = 1 << a.scale
        parts = []
        sr = cbg.MinPlusSRing if a.sr == "minplus" else cbg.PlusTimesSRing
        cbg.MemEfficientSpGEMM(cbg.SpParMat(A, g, nv, nv), cbg.SpParMat(B, g, nv, nv), a.phases, sr=sr,
                               on_phase=lambda ph, off, t: parts.append(dict(t.digest(0, off), nzc=t.nzc)))
        gd = add(parts)
    A.free()
    B.free()
    print(json.dumps({"gpu": gd, "s": round(time.time() - t0, 1)}), flush=True)
    from helpers import oracle_local, oracle_rmat  # the checker
    t0 = time.time()
    Ah = oracle_rmat(a.scale, a.ef, nthreads=a.threads)
    if a.oracle_pieces <= 1:
        Ch = oracle_local(Ah, dict(Ah), a.sr, nthreads=a.threads)
        od = chunked_digest(Ch)
        del Ch
    else:
        sys.path.insert(0, REPO)
        sub_tile = cbg.sub_tile
        n = Ah["n"]
        parts = []
        np_ = a.oracle_pieces
        for ph in range(np_):
            c0, c1 = ph * (n // np_), (n if ph == np_ - 1 else (ph + 1) * (n // np_))
            Ch = oracle_local(Ah, sub_tile(Ah, 0, Ah["m"], c0, c1), a.sr, nthreads=a.threads)
            parts.append(chunked_digest(Ch, c0))
            del Ch
            print(json.dumps({"piece": ph, "oracle_s": round(time.time() - t0, 1)}), flush=True)
        od = add(parts)
    print(json.dumps({"oracle_s": round(time.time() - t0, 1)}), flush=True)
    ok = od["nnz"] == gd["nnz"] and od["hs"] == gd["hs"] and od["hv"] == gd["hv"] and od["unsorted"] == 0
    print(json.dumps({"oracle": od, "match": ok}), flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
