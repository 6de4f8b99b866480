#!/usr/bin/env python3
"""Generate tests/golden/ fixtures by running the REFERENCE CombBLAS code.

TEST INFRASTRUCTURE ONLY -- runs in the build container (where /root/reference
exists), never on the GPU box.  Requires `make -C oracle ref` first, which
builds oracle/_ref/ref_driver from oracle/ref_driver.cpp + the reference's own
sources (see oracle/Makefile).

Outputs (all data, no reference source):
  tests/golden/golden.json      digests / totals produced by the reference
  tests/golden/*.npz            full matrices (inputs and products) for small cases

Digest definition (mirrored by tests/digest.py):
  nnz, nzc, hs = sum_e mix64(col<<32|row) mod 2^64,
  hv = sum_e mix64(col<<32|row) * mix64(bits(val)) mod 2^64, vsum = sum_e val.
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
DRIVER = os.path.join(REPO, "oracle", "_ref", "ref_driver")
MPIRUN = "/opt/conda/bin/mpirun"
REF = "/root/reference"


def read_cbgt(path):
    with open(path, "rb") as f:
        magic = f.read(8)
        assert magic == b"CBGT0001", magic
        hdr = np.frombuffer(f.read(80), dtype=np.int64)
        m, n, nnz, nzc = (int(x) for x in hdr[:4])
        cp = np.frombuffer(f.read(8 * (nzc + 1)), dtype=np.int64)
        jc = np.frombuffer(f.read(4 * nzc), dtype=np.int32)
        ir = np.frombuffer(f.read(4 * nnz), dtype=np.int32)
        val = np.frombuffer(f.read(8 * nnz), dtype=np.float64)
    return dict(m=m, n=n, cp=cp, jc=jc, ir=ir, val=val, grid=hdr[4:8].tolist(), off=hdr[8:10].tolist())


def save_npz(name, t):
    np.savez_compressed(os.path.join(HERE, name), m=t["m"], n=t["n"], cp=t["cp"], jc=t["jc"], ir=t["ir"], val=t["val"])


def run(args, nprocs=1, env=None):
    cmd = [DRIVER] + args
    if nprocs > 1:
        cmd = [MPIRUN, "-n", str(nprocs)] + cmd
    e = dict(os.environ)
    e.setdefault("OMP_NUM_THREADS", "8")
    if env:
        e.update(env)
    out = subprocess.run(cmd, check=True, capture_output=True, text=True, env=e).stdout
    recs = []
    for line in out.splitlines():
        line = line.strip()
        if line.startswith("{"):
            recs.append(json.loads(line))
    return recs


def tagged(recs, tag):
    for r in recs:
        if r.get("tag") == tag:
            d = dict(r)
            d.pop("tag")
            return d
    raise KeyError(tag)


def main():
    if not os.path.exists(DRIVER):
        sys.exit("build the reference driver first: make -C oracle ref")
    gold = {"_doc": __doc__.strip().splitlines()[0], "rmat": {}, "files": {}}
    tmp = tempfile.mkdtemp(prefix="cbg_golden_")

    # ---- bundled small inputs (configs[0]: MultTest plumbing, fp-tolerance KAT) ----
    files = {
        "sevenvertex": ("readmm", f"{REF}/ReleaseTests/sevenvertex.mtx", None),
        "small_nonsym": ("readtriples", f"{REF}/ReleaseTests/small_nonsym.mtx", None),
        "largeseq": ("readtriples", f"{REF}/largeseq/input1_0", f"{REF}/largeseq/input2_0"),
    }
    for name, (mode, fa, fb) in files.items():
        entry = {}
        pa = os.path.join(tmp, name + "_A.cbgt")
        entry["A"] = tagged(run([mode, fa, pa]), "A")
        A = read_cbgt(pa)
        save_npz(f"{name}_A.npz", A)
        pb = pa
        if fb is not None:
            pb = os.path.join(tmp, name + "_B.cbgt")
            entry["B"] = tagged(run([mode, fb, pb]), "A")
            save_npz(f"{name}_B.npz", read_cbgt(pb))
        else:
            # A*A with B a deep copy of A (aliasing is forbidden, ParFriends.h:172-178)
            pb = os.path.join(tmp, name + "_B.cbgt")
            with open(pa, "rb") as s, open(pb, "wb") as d:
                d.write(s.read())
        for sr in ("plus", "minplus"):
            for algo in ("local", "heap", "doublebuff", "synch"):
                pc = os.path.join(tmp, f"{name}_C_{algo}_{sr}.cbgt")
                recs = run(["mult", algo, sr, pa, pb, pc])
                entry[f"C_{algo}_{sr}"] = tagged(recs, f"C_{algo}_{sr}")
                if algo in ("local", "doublebuff"):
                    save_npz(f"{name}_C_{algo}_{sr}.npz", read_cbgt(pc))
            # distributed 2x2 grid, same product (reference's square-grid SUMMA)
            if name != "sevenvertex":  # 7x7 with 4 ranks is fine for GEMM; keep the set small
                for algo in ("doublebuff", "synch"):
                    recs = run(["mult", algo, sr, pa, pb, "-"], nprocs=4)
                    entry[f"C_{algo}_{sr}_p4"] = tagged(recs, f"C_{algo}_{sr}")
        gold["files"][name] = entry
        print(name, "done", flush=True)

    # ---- R-MAT A*A (Graph500 Kronecker, SEED default 0xDECAFBAD) ----
    scales = [int(s) for s in os.environ.get("GOLD_SCALES", "8,10,12,14,16,18").split(",")]
    for scale in scales:
        ef = 16
        key = f"s{scale}_ef{ef}"
        entry = {}
        pa = os.path.join(tmp, key + "_A.cbgt")
        recs = run(["gen", str(scale), str(ef), pa])
        entry["A"] = tagged(recs, "A")
        entry["loops_removed"] = tagged(recs, "gen_loops_removed")["value"]
        A = read_cbgt(pa)
        pb = os.path.join(tmp, key + "_B.cbgt")
        with open(pa, "rb") as s, open(pb, "wb") as d:
            d.write(s.read())
        if scale <= 10:
            save_npz(f"rmat_{key}_A.npz", A)
        algos = ("local", "heap", "doublebuff", "synch") if scale <= 16 else ("local", "synch", "doublebuff")
        for algo in algos:
            for sr in (("plus", "minplus") if algo == "local" else ("plus",)):
                pc = os.path.join(tmp, f"{key}_C_{algo}_{sr}.cbgt") if (scale <= 10 and algo == "local") else "-"
                recs = run(["mult", algo, sr, pa, pb, pc])
                entry[f"C_{algo}_{sr}"] = tagged(recs, f"C_{algo}_{sr}")
                entry[f"time_{algo}_{sr}"] = tagged(recs, f"time_{algo}")["seconds"]
                if pc != "-":
                    save_npz(f"rmat_{key}_C_{algo}_{sr}.npz", read_cbgt(pc))
        if scale <= 14:
            recs = run(["mult", "doublebuff", "plus", pa, pb, "-"], nprocs=4)
            entry["C_doublebuff_plus_p4"] = tagged(recs, "C_doublebuff_plus")
        entry["symbolic"] = tagged(run(["symbolic", pa, pb]), "symbolic")
        gold["rmat"][key] = entry
        print(key, "done", flush=True)
        with open(os.path.join(HERE, "golden.json"), "w") as f:
            json.dump(gold, f, indent=1, sort_keys=True)

    big_scales(gold, tmp, os.environ.get("GOLD_BIG", "20x16,20x8,22x16,22x8"))
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(gold, f, indent=1, sort_keys=True)
    multtest_fixture()


def big_scales(gold, tmp, spec):
    """large scales: inputs + symbolic totals only (C does not fit this host)"""
    big = [tuple(int(x) for x in s.split("x")) for s in spec.split(",") if s]
    for scale, ef in big:
        key = f"s{scale}_ef{ef}"
        entry = {}
        pa = os.path.join(tmp, key + "_A.cbgt")
        recs = run(["gen", str(scale), str(ef), pa])
        entry["A"] = tagged(recs, "A")
        entry["loops_removed"] = tagged(recs, "gen_loops_removed")["value"]
        entry["symbolic"] = tagged(run(["symbolic", pa, pa]), "symbolic")
        os.remove(pa)
        gold["rmat"][key] = entry
        print(key, "done", flush=True)
        with open(os.path.join(HERE, "golden.json"), "w") as f:
            json.dump(gold, f, indent=1, sort_keys=True)


def multtest_fixture():
    """ReleaseTests/MultTest inputs: the reference's bundled sevenvertex.mtx (data
    file, copied) and CControl = the reference's product of it with itself
    (sevenvertex_C_local_plus.npz above), written as Matrix Market."""
    import shutil
    shutil.copyfile(f"{REF}/ReleaseTests/sevenvertex.mtx", os.path.join(HERE, "sevenvertex.mtx"))
    d = np.load(os.path.join(HERE, "sevenvertex_C_local_plus.npz"))
    cols = np.repeat(d["jc"].astype(np.int64), np.diff(d["cp"]))
    with open(os.path.join(HERE, "sevenvertex_C.mtx"), "w") as f:
        f.write("%%MatrixMarket matrix coordinate real general\n")
        f.write(f"{int(d['m'])} {int(d['n'])} {len(d['ir'])}\n")
        for r, c, v in zip(d["ir"], cols, d["val"]):
            f.write(f"{int(r) + 1} {int(c) + 1} {float(v)!r}\n")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "big":
        # add large-scale symbolic totals to the existing golden.json, e.g. `big 24x16`
        with open(os.path.join(HERE, "golden.json")) as f:
            g = json.load(f)
        big_scales(g, tempfile.mkdtemp(prefix="cbg_golden_"), sys.argv[2])
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "multtest":
        multtest_fixture()
    else:
        main()
