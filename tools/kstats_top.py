#!/usr/bin/env python3
"""Top kernels of a rocprofv3 --stats CSV, ms per step: kstats_top.py <stats.csv> <steps> [n]."""
import csv
import sys

path, steps = sys.argv[1], float(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("total kernel ms/step %.1f" % (tot / 1e6 / steps))
for r in rows[:top]:
    name = r["Name"].split("(")[0][:90]
    print("%8.2f ms/step %6d calls  %s" % (float(r["TotalDurationNs"]) / 1e6 / steps, int(r["Calls"]), name))
