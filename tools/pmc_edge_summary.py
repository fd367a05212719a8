#!/usr/bin/env python3
"""Per-variant edge-kernel PMC summary of tools/gpu_edge_ab.sh passes:
median per-dispatch L2->fabric read bytes (128-B requests) and L2 hit rate.

    python tools/pmc_edge_summary.py gpurun_out/pmc_<tag>_v*
"""
import csv
import glob
import json
import os
import statistics
import sys

out = {}
for d in sys.argv[1:]:
    per = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if "k_edge" not in r["Kernel_Name"] or "merge" in r["Kernel_Name"]:
                continue
            c = per.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"][:60]})
            c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    if not per:
        continue
    rd = statistics.median(128 * c.get("TCC_EA0_RDREQ_128B_sum", 0) for c in per.values())
    hit = statistics.median(c.get("TCC_HIT_sum", 0) for c in per.values())
    miss = statistics.median(c.get("TCC_MISS_sum", 0) for c in per.values())
    out[os.path.basename(d)] = {"kernel": next(iter(per.values()))["name"],
                                "fabric_read_GB": rd / 1e9,
                                "l2_hit": hit / (hit + miss) if hit + miss else None,
                                "dispatches": len(per)}
print(json.dumps(out, indent=1))
