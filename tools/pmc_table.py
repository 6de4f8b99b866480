#!/usr/bin/env python3
"""Per-kernel SQ counter table from rocprofv3 counter_collection CSVs (2nd multiply of tools/traffic.py run)."""
import collections
import csv
import sys


def table(path, top=8):
    rows = list(csv.DictReader(open(path)))
    dig = sorted({int(r["Dispatch_Id"]) for r in rows if "k_digest" in r["Kernel_Name"]})
    lo, hi = (dig[1], dig[2]) if len(dig) >= 3 else (0, 1 << 62)
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in rows:
        d = int(r["Dispatch_Id"])
        if lo < d < hi:
            agg[r["Kernel_Name"].split("(")[0][-40:]][r["Counter_Name"]] += float(r["Counter_Value"])
    for n, c in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:top]:
        wc = max(c["SQ_WAVE_CYCLES"], 1)
        print(f"{n:40s} wave_cyc {wc:9.3g} wait_any {c['SQ_WAIT_ANY']/wc:.2f} wait_inst {c['SQ_WAIT_INST_ANY']/wc:.2f} "
              f"active {c['SQ_ACTIVE_INST_ANY']/wc:.2f} lds_insts {c['SQ_INSTS_LDS']:9.3g} bankconf {c['SQ_LDS_BANK_CONFLICT']:9.3g}")


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print("==", p)
        table(p)
