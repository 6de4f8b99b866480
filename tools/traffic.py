#!/usr/bin/env python3
"""HBM traffic of one local SpGEMM (the bench's dominant pipeline) from rocprofv3 PMC passes.

  # on the GPU box, one pass per counter group (FETCH_SIZE and WRITE_SIZE do not fit one pass):
  rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pf -o f -- python3 tools/traffic.py run --scale 18
  rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pw -o w -- python3 tools/traffic.py run --scale 18
  # anywhere:
  python3 tools/traffic.py parse --fetch <f_counter_collection.csv> --write <w_counter_collection.csv> \
      --meta <run json> --out profiles/r01_traffic_s18.json

`run` issues: digest(A), multiply, digest(A), multiply, digest(C).  The second
multiply is every dispatch strictly between the 2nd and 3rd k_digest.  The
digests are the calibration: k_digest reads A's DCSC arrays once, wave per
column, 4-8 B per lane -- the same access widths as the SpGEMM kernels -- so
known_bytes / FETCH bytes of digest(A) corrects the gfx950 FETCH_SIZE
under-count (MI355X_MICROARCH.md, HBM section: FETCH_SIZE reports 1/2 of a wide
coalesced read; other widths uncalibrated).  WRITE_SIZE: after the last digest
`run` stores known byte counts with 4- and 8-byte stores per lane (k_store_probe,
the widths of C's row ids and values; the kept bitmaps are 16-byte stores, which
the guide finds exact) and a wave-per-column 8-byte store of A's values
(k_random_values: C's per-column runs), so the parse reports WRITE_SIZE's factor
for each width; the write total is corrected with the 4-/8-byte factors applied to
C's known row-id and value bytes (the rest taken as read).
The algorithmic bytes split as SURVEY 8(d): symbolic 4 F + 12 N_B (A's rows per
product, B's entries and map hops), numeric 12 F + 12 N_C + 20 N_B + 8 n; the
per-phase ratios compare the symbolic and numeric kernels' traffic with them.
"""
import argparse
import csv
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def tile_bytes(t):
    return 8 * (t["nzc"] + 1) + 4 * t["nzc"] + 12 * t["nnz"]


def run(a):
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from conftest import load_cbg
    cbg = load_cbg()
    cbg.lib().cbg_set_device(0)
    A = cbg.rmat_tile(a.scale, a.ef)
    B = cbg.rmat_tile(a.scale, a.ef)
    cbg.synchronize()
    if a.phases > 1:
        # C larger than HBM: MemEfficientSpGEMM phases on a one-rank grid, C
        # materialized per phase (as bench.py --phases); digests of A mark the
        # second multiply's dispatches
        class Self:
            def bcast(self, comm, arr, root):
                pass

            def allgather(self, comm, data):
                return data

        g = cbg.CommGrid(0, 1, transport="host", host_comm=Self())
        nv = 1 << a.scale
        PA, PB = cbg.SpParMat(A, g, nv, nv), cbg.SpParMat(B, g, nv, nv)
        seen = [0, 0]

        def consume(p, off, t):
            seen[0] += t.nnz
            seen[1] += t.nzc

        A.digest()
        cbg.MemEfficientSpGEMM(PA, PB, a.phases, on_phase=consume)
        A.digest()
        seen[:] = [0, 0]
        cbg.MemEfficientSpGEMM(PA, PB, a.phases, on_phase=consume)
        st = cbg.last_stats()
        A.digest()
        cnnz, cnzc = seen
    else:
        A.digest()
        C = cbg.LocalHybridSpGEMM(A, B)
        cbg.synchronize()
        C.free()
        A.digest()
        C = cbg.LocalHybridSpGEMM(A, B)
        cbg.synchronize()
        st = cbg.last_stats()
        C.digest()
        cnnz, cnzc = C.nnz, C.nzc
    # WRITE_SIZE calibration (after the 3rd digest): known bytes at 4 and 8 B per lane,
    # and 8-byte values written wave per column (A's values, 8 nnz(A) bytes)
    probe = 1 << 30
    cbg.store_probe(probe, 4)
    cbg.store_probe(probe, 8)
    A.set_random_values()
    cbg.synchronize()
    meta = {"store_probe_bytes": probe, "scale": a.scale, "ef": a.ef, "phases": a.phases,
            "A": {"nnz": A.nnz, "nzc": A.nzc}, "B": {"nnz": B.nnz, "nzc": B.nzc, "n": B.n},
            "C": {"nnz": cnnz, "nzc": cnzc}, "flops": st["flops"]}
    print(json.dumps(meta), flush=True)


def read_pmc(path, counter):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter:
                rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    rows.sort()
    # one value per dispatch (some counters are reported per XCD/instance: sum them)
    out = {}
    for d, n, v in rows:
        if d in out:
            out[d] = (n, out[d][1] + v)
        else:
            out[d] = (n, v)
    return [(d, n, v) for d, (n, v) in sorted(out.items())]


def split(rows):
    dig = [i for i, (_, n, _) in enumerate(rows) if "k_digest" in n]
    if len(dig) < 3:
        raise SystemExit("expected 3 k_digest dispatches, found %d" % len(dig))
    return rows[dig[0]], rows[dig[1]], rows[dig[2]], rows[dig[1] + 1:dig[2]]


def parse(a):
    meta = None
    for line in open(a.meta):
        line = line.strip()
        if line.startswith("{"):
            meta = json.loads(line)
    fr = read_pmc(a.fetch, "FETCH_SIZE")
    wr = read_pmc(a.write, "WRITE_SIZE")
    kb = 1024.0  # rocprofv3 FETCH_SIZE / WRITE_SIZE unit: KiB
    wcal = {}
    if "store_probe_bytes" in meta:
        pb = meta["store_probe_bytes"]
        for w in (4, 8):
            v = [x for _, n, x in wr if "k_store_probe<%d>" % w in n]
            if v:
                wcal["lane_%dB" % w] = pb / (v[-1] * kb)
        v = [x for _, n, x in wr if "k_random_values" in n]
        if v:
            wcal["column_runs_8B"] = 8 * meta["A"]["nnz"] / (v[-1] * kb)
    d0, d1, _, mult_f = split(fr)
    _, _, _, mult_w = split(wr)
    known_a = tile_bytes(meta["A"])
    calib = known_a / (0.5 * (d0[2] + d1[2]) * kb)
    fetch_raw = sum(v for _, _, v in mult_f) * kb
    write_raw = sum(v for _, _, v in mult_w) * kb
    per_kernel = {}
    for _, n, v in mult_f:
        k = n.split("(")[0]
        per_kernel.setdefault(k, [0.0, 0.0])[0] += v * kb * calib
    for _, n, v in mult_w:
        k = n.split("(")[0]
        per_kernel.setdefault(k, [0.0, 0.0])[1] += v * kb
    F, nnzc, nnzb, n = meta["flops"], meta["C"]["nnz"], meta["B"]["nnz"], meta["B"]["n"]
    alg = 16 * F + 12 * nnzc + 32 * nnzb + 8 * n
    # the writes with a calibrated width: C's row ids (4 B) and values (8 B); the
    # rest (kept bitmaps in 16-byte stores, column pointers, temporaries) as read
    write = write_raw
    if "lane_4B" in wcal and "lane_8B" in wcal:
        c4, c8 = 4.0 * nnzc, 8.0 * nnzc
        write = write_raw - c4 / wcal["lane_4B"] - c8 / wcal["lane_8B"] + c4 + c8
    # per phase: symbolic (k_sym*) and the rest (numeric, copies, scans) against
    # SURVEY 8(d)'s split of the algorithmic bytes
    alg_sym = 4 * F + 12 * nnzb
    sym_t = sum(f + w for k, (f, w) in per_kernel.items() if "k_sym" in k)
    num_t = sum(f + w for k, (f, w) in per_kernel.items() if "k_sym" not in k)
    phases = {"symbolic": {"counter_bytes": sym_t, "algorithmic_bytes": alg_sym, "ratio": sym_t / alg_sym},
              "numeric": {"counter_bytes": num_t, "algorithmic_bytes": alg - alg_sym, "ratio": num_t / (alg - alg_sym)}}
    out = {"scale": meta["scale"], "ef": meta["ef"], "phases": meta.get("phases", 1), "dispatches": len(mult_f),
           "fetch_calibration": calib, "fetch_bytes_raw": fetch_raw, "fetch_bytes": fetch_raw * calib,
           "write_calibration": wcal, "write_bytes_raw": write_raw,
           "write_bytes": write, "traffic_bytes": fetch_raw * calib + write,
           "algorithmic_bytes": alg, "traffic_over_algorithmic": (fetch_raw * calib + write) / alg,
           "per_phase": phases,
           "per_kernel_fetch_write": {k: [round(x), round(y)] for k, (x, y) in
                                      sorted(per_kernel.items(), key=lambda kv: -(kv[1][0] + kv[1][1]))},
           "meta": meta}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: out[k] for k in ("fetch_calibration", "write_calibration", "fetch_bytes", "write_bytes",
                                          "traffic_bytes", "algorithmic_bytes", "traffic_over_algorithmic",
                                          "per_phase")}))


def main():
    p = argparse.ArgumentParser()
    sub = p.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("--scale", type=int, default=18)
    r.add_argument("--ef", type=int, default=16)
    r.add_argument("--phases", type=int, default=1)
    q = sub.add_parser("parse")
    q.add_argument("--fetch", required=True)
    q.add_argument("--write", required=True)
    q.add_argument("--meta", required=True)
    q.add_argument("--out", required=True)
    a = p.parse_args()
    run(a) if a.cmd == "run" else parse(a)


if __name__ == "__main__":
    main()
