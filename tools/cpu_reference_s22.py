#!/usr/bin/env python3
"""Sum tools/cpu_reference_s22.sh's per-phase lines (gpurun_out/cpu_ref_s22.log) into
profiles/<round>_cpu_reference_s22.json: the reference's Mult_AnXBn_Synch on R-MAT
scale-22 ef16 A*A, 16 B-column phases, multiply time only, summed digest (checked
against the oracle's whole-C digest in tests/golden/oracle_large.json)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(log, out):
    secs, nnz, hs, hv, uns, threads, host, phases = 0.0, 0, 0, 0, 0, None, {}, 0
    for line in open(log):
        line = line.strip()
        if line.startswith("threads"):
            threads = int(line.split()[1])
        elif ":" in line and not line.startswith("{"):
            k, _, v = line.partition(":")
            host[k.strip()] = v.strip()
        elif line.startswith("{"):
            d = json.loads(line)
            if d["tag"].startswith("time_"):
                secs += d["seconds"]
            elif d["tag"].startswith("C_"):
                nnz += d["nnz"]
                hs = (hs + int(d["hs"], 16)) % (1 << 64)
                hv = (hv + int(d["hv"], 16)) % (1 << 64)
                uns += d["unsorted"]
                phases += 1
    gold = json.load(open(os.path.join(REPO, "tests", "golden", "oracle_large.json")))["s22_ef16"]
    res = {"value": nnz / secs, "unit": "nnz(C)/s", "cores": threads, "kind": "reference",
           "sample": "R-MAT scale-22 ef16 A*A (the metric's configuration), the reference's Mult_AnXBn_Synch 1x1 "
                     "(oracle/_ref/ref_driver multphased), B cut into %d column phases by SpDCCols::ColSplit because "
                     "the whole C (24.8 G nonzeros) exceeds the job's host memory; one process per phase; multiply "
                     "time only, summed: %.1f s" % (phases, secs),
           "seconds": secs, "nnz_C": nnz, "phases": phases, "host": host,
           "digest_matches_oracle": (nnz, "%016x" % hs, "%016x" % hv) == (gold["nnz"], gold["hs"], gold["hv"]),
           "unsorted": uns, "command": "tools/cpu_reference_s22.sh (on the GPU box) + tools/cpu_reference_s22.py"}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "gpurun_out", "cpu_ref_s22.log"),
         sys.argv[2] if len(sys.argv) > 2 else os.path.join(REPO, "profiles", "r02_cpu_reference_s22.json"))
