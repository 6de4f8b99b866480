#!/usr/bin/env python3
"""Timeline of one local multiply from a rocprofv3 kernel_trace.csv (the LAST multiply:
dispatches from the last k_colmap launch to the last k_col_scatter): per kernel start/end offsets, stream, and
the busy union / gaps.  usage: tools/timeline.py k_kernel_trace.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("cbg::k_colmap(")]
rows = rows[starts[-1]:]
ends = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("cbg::k_col_scatter(")]
if ends:  # the multiply ends with its column scatter (later dispatches: e.g. the bench's copy-rate probe)
    rows = rows[:ends[-1] + 1]
t0 = int(rows[0]["Start_Timestamp"])
busy = []
for r in rows:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    busy.append((s, e))
    print(f"{s/1e3:9.1f} {e/1e3:9.1f} {(e-s)/1e3:8.1f}us q{r.get('Queue_Id','?'):>3} {r['Kernel_Name'][:70]}")
busy.sort()
u, cs, ce = 0, None, None
for s, e in busy:
    if cs is None or s > ce:
        if cs is not None:
            u += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
u += ce - cs
print(f"span {busy[-1][1]/1e3:.1f} us, busy union {u/1e3:.1f} us")
