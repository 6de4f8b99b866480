#!/usr/bin/env python3
"""Per-kernel counter sums of the 2nd multiply of tools/traffic.py run (dispatches between the
2nd and 3rd k_digest) from rocprofv3 counter_collection CSVs:  pmc_kernels.py <csv>..."""
import collections
import csv
import sys


def load(path):
    rows = list(csv.DictReader(open(path)))
    dig = sorted({int(r["Dispatch_Id"]) for r in rows if "k_digest" in r["Kernel_Name"]})
    lo, hi = (dig[1], dig[2]) if len(dig) >= 3 else (0, 1 << 62)
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in rows:
        d = int(r["Dispatch_Id"])
        if lo < d < hi:
            n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("cbg::", "")
            agg[n][r["Counter_Name"]] += float(r["Counter_Value"])
    return agg


if __name__ == "__main__":
    agg = collections.defaultdict(dict)
    for p in sys.argv[1:]:
        for k, c in load(p).items():
            agg[k].update(c)
    names = sorted({c for v in agg.values() for c in v})
    def weight(c):
        return c.get("SQ_WAVE_CYCLES", c.get("SQ_BUSY_CYCLES", c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0)))
    top = sorted(agg.items(), key=lambda kv: -weight(kv[1]))[:14]
    for k, c in top:
        wc = max(c.get("SQ_WAVE_CYCLES", 1), 1)
        hit = c.get("TCC_HIT_sum", 0.0)
        miss = c.get("TCC_MISS_sum", 0.0)
        print(f"== {k}" + (f"   L2 hit {hit / (hit + miss):.3f}" if hit + miss > 0 else ""))
        print("   " + "  ".join(f"{n}={c[n]:.3g}" + (f"({c[n]/wc:.2f}wc)" if n.startswith(("SQ_WAIT", "SQ_ACTIVE")) else "")
                               for n in names if n in c))
