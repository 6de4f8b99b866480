#!/usr/bin/env python3
"""Communication/compute overlap from rocprofv3 kernel traces of a multi-rank run
(tools/gpu_overlap_trace.sh): for every process, the RCCL kernels (broadcasts of
the pipelined PANEL SUMMA) and how much of their time runs while one of that
process's local-SpGEMM kernels (cbg::k_*) is executing.

  python tools/overlap.py <trace dir> [--json out.json]
"""
import csv
import glob
import json
import os
import sys


def intervals_union(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def overlap(a, b_union):
    s, e = a
    t = 0
    for bs, be in b_union:
        if be <= s:
            continue
        if bs >= e:
            break
        t += min(e, be) - max(s, bs)
    return t


def main():
    d = sys.argv[1]
    out_json = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    files = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))
    res = []
    for f in files:
        rows = list(csv.DictReader(open(f)))
        by_pid = {}
        for r in rows:
            # one host thread per rank process dispatches its kernels (rocprofv3 has no process column)
            by_pid.setdefault(r.get("Process_Id") or r.get("Thread_Id", "?"), []).append(r)
        for pid, rs in by_pid.items():
            comm = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rs
                    if "nccl" in r["Kernel_Name"].lower()]
            comp = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rs
                    if r["Kernel_Name"].startswith("cbg::k_") or r["Kernel_Name"].startswith("void cbg::k_")]
            slab = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rs if "k_num_slab<" in r["Kernel_Name"]
                    or "k_sym_panel" in r["Kernel_Name"]]
            cu, su = intervals_union(comp), intervals_union(slab)
            tot = sum(e - s for s, e, _ in comm)
            ov = sum(overlap((s, e), cu) for s, e, _ in comm)
            ovs = sum(overlap((s, e), su) for s, e, _ in comm)
            big = sorted(comm, key=lambda x: x[1] - x[0])[-3:]
            rec = dict(trace=os.path.relpath(f, d), thread=pid, rccl_kernels=len(comm), rccl_ms=tot / 1e6,
                       rccl_ms_overlapped_with_cbg=ov / 1e6, rccl_ms_overlapped_with_slab_or_symbolic=ovs / 1e6,
                       cbg_kernels=len(comp), longest_rccl=[(n[:60], (e - s) / 1e6) for s, e, n in big])
            res.append(rec)
            print(json.dumps(rec))
    if out_json:
        with open(out_json, "w") as fo:
            json.dump(res, fo, indent=1)


if __name__ == "__main__":
    main()
