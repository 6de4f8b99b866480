#!/usr/bin/env python3
"""One-off parity check at a scale beyond the golden digests: the HIP local
multiply's C = A*A digest against the CPU oracle's (test infrastructure), for
R-MAT `--scale` (default 20: 4 row panels, panel groups, multi-slab pairs).
Needs ~150 GB of host memory at scale 20 (the oracle's C); run on the GPU box:

  python tools/check_scale.py --scale 20 --threads 16
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))


def chunked_digest(t, chunk=1 << 27):
    """helpers.digest over column blocks (bounded temporaries)."""
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
        c1 = max(c1, c0 + 1)
        c1 = min(c1, nzc)
        a, b = int(cp[c0]), int(cp[c1])
        col = np.repeat(jc[c0:c1].astype(np.uint64), np.diff(cp[c0:c1 + 1]))
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


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--scale", type=int, default=20)
    p.add_argument("--threads", type=int, default=16)
    p.add_argument("--sr", choices=["plus", "minplus"], default="plus")
    a = p.parse_args()
    from conftest import load_cbg
    cbg = load_cbg()
    cbg.lib().cbg_set_device(0)
    t0 = time.time()
    A = cbg.rmat_tile(a.scale, 16)
    B = cbg.rmat_tile(a.scale, 16)
    C = cbg.LocalHybridSpGEMM(A, B, a.sr)
    gd = C.digest()
    C.free()
    A.free()
    B.free()
    print(json.dumps({"gpu": gd, "s": round(time.time() - t0, 1)}), flush=True)
    from helpers import oracle_local, oracle_rmat  # the checker
    t0 = time.time()
    Ah = oracle_rmat(a.scale, 16, nthreads=a.threads)
    Ch = oracle_local(Ah, dict(Ah), a.sr, nthreads=a.threads)
    print(json.dumps({"oracle_s": round(time.time() - t0, 1), "nnz": int(len(Ch["ir"]))}), flush=True)
    od = chunked_digest(Ch)
    ok = od["nnz"] == gd["nnz"] and od["hs"] == gd["hs"] and od["hv"] == gd["hv"] and od["unsorted"] == 0
    print(json.dumps({"oracle": od, "match": ok}), flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
