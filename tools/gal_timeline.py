#!/usr/bin/env python3
"""Timeline of the last K local multiplies in a rocprofv3 kernel_trace.csv (from the K-th
last k_colmap dispatch to the end): per-kernel offsets, the busy union and the idle gaps
between dispatches (host work: synchronizations, allocations, Python).
usage: tools/gal_timeline.py k_kernel_trace.csv [K]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
K = int(sys.argv[2]) if len(sys.argv) > 2 else 2
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("cbg::k_colmap(")]
rows = rows[starts[-K]:]
t0 = int(rows[0]["Start_Timestamp"])
iv = []
for r in rows:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    iv.append((s, e))
    print(f"{s/1e3:9.1f} {e/1e3:9.1f} {(e-s)/1e3:8.1f}us q{r.get('Queue_Id','?'):>3} {r['Kernel_Name'][:80]}")
iv.sort()
busy, gaps, cs, ce = 0, [], None, None
for s, e in iv:
    if cs is None or s > ce:
        if cs is not None:
            busy += ce - cs
            gaps.append((ce, s))
        cs, ce = s, e
    else:
        ce = max(ce, e)
busy += ce - cs
span = ce
print(f"span {span/1e3:.1f} us, busy {busy/1e3:.1f} us, idle {(span-busy)/1e3:.1f} us in {len(gaps)} gaps")
for a, b in sorted(gaps, key=lambda g: g[0] - g[1])[:12]:
    print(f"  gap {a/1e3:9.1f} -> {b/1e3:9.1f}: {(b-a)/1e3:7.1f} us")
