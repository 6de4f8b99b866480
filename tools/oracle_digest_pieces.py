#!/usr/bin/env python3
"""The CPU oracle's digest of C = A*A for R-MAT `--scale`, computed one B-column
piece at a time (host memory bounded by the piece), resumable: every finished
piece is appended to `--state` (JSON lines), a rerun skips them.  TEST
INFRASTRUCTURE: it pins digests (tests/golden/oracle_large.json) beyond the
reference-generated golden vectors; no GPU is used.

  nice -n 19 python tools/oracle_digest_pieces.py --scale 24 --pieces 256 --threads 6 \
      --state /tmp/s24_pieces.jsonl
  # a strided sample (config 4's 2x4 grid: 128 pieces per grid column, 8 from each)
  python tools/oracle_digest_pieces.py --scale 24 --pieces 512 --only 0:512:16 --state ...

Prints the summed digest (tools/check_scale.py's definition: hs, hv mod 2^64,
vsum, unsorted) when all pieces are done.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "tools"))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--scale", type=int, required=True)
    p.add_argument("--ef", type=int, default=16)
    p.add_argument("--sr", choices=["plus", "minplus"], default="plus")
    p.add_argument("--pieces", type=int, default=64)
    p.add_argument("--threads", type=int, default=6)
    p.add_argument("--state", required=True)
    p.add_argument("--only", default=None, help="start:stop:step of the pieces to compute (default: all)")
    a = p.parse_args()
    want = range(a.pieces) if a.only is None else range(*[int(x) for x in a.only.split(":")])
    from check_scale import add, chunked_digest
    from helpers import oracle_local, oracle_rmat
    import numpy as np

    done = {}
    if os.path.exists(a.state):
        with open(a.state) as f:
            for line in f:
                d = json.loads(line)
                done[d["piece"]] = d
    t0 = time.time()
    A = oracle_rmat(a.scale, a.ef, nthreads=a.threads)
    print(json.dumps({"A_nnz": int(len(A["ir"])), "gen_s": round(time.time() - t0, 1)}), flush=True)
    n = A["n"]
    cp, jc = A["cp"], A["jc"]
    for ph in want:
        if ph in done:
            continue
        c0, c1 = ph * (n // a.pieces), (n if ph == a.pieces - 1 else (ph + 1) * (n // a.pieces))
        lo, hi = int(np.searchsorted(jc, c0)), int(np.searchsorted(jc, c1))
        Bp = dict(m=A["m"], n=c1 - c0, cp=(cp[lo:hi + 1] - cp[lo]).astype(np.int64),
                  jc=(jc[lo:hi] - c0).astype(np.int32), ir=A["ir"][cp[lo]:cp[hi]], val=A["val"][cp[lo]:cp[hi]])
        t1 = time.time()
        C = oracle_local(A, Bp, a.sr, nthreads=a.threads)
        d = chunked_digest(C, c0)
        del C
        d.update(piece=ph, s=round(time.time() - t1, 1))
        with open(a.state, "a") as f:
            f.write(json.dumps(d) + "\n")
        done[ph] = d
        print(json.dumps(d), flush=True)
    if a.only is not None:
        print(json.dumps({"scale": a.scale, "ef": a.ef, "sr": a.sr, "pieces": a.pieces,
                          "digests": {str(k): done[k] for k in want}}), flush=True)
        return
    tot = add([done[k] for k in range(a.pieces)])
    tot["unsorted"] = sum(done[k]["unsorted"] for k in range(a.pieces))
    print(json.dumps({"scale": a.scale, "ef": a.ef, "sr": a.sr, "pieces": a.pieces, "digest": tot}), flush=True)


if __name__ == "__main__":
    main()
