#!/usr/bin/env python3
"""Median per-dispatch SQ counters for our kernels from rocprofv3 --pmc CSVs."""
import csv
import glob
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import short_name  # noqa: E402

per = {}
for d in sys.argv[1:]:
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            n = r["Kernel_Name"]
            if not any(k in n for k in ("k_edge", "k_project", "k_bwd", "k_wgrad", "k_dx")):
                continue
            key = short_name(n)
            per.setdefault(key, {}).setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
            per[key][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
for k, ctrs in per.items():
    print(k)
    med = {c: statistics.median(v.values()) for c, v in ctrs.items()}
    for c, v in sorted(med.items()):
        print(f"   {c:24s} {v:16.1f}")
    if "SQ_WAVE_CYCLES" in med and "SQ_WAVES" in med and med["SQ_WAVES"]:
        print(f"   avg wave lifetime (cycles) {4 * med['SQ_WAVE_CYCLES'] / med['SQ_WAVES']:.0f}")
    if "GRBM_GUI_ACTIVE" in med:
        print(f"   GRBM_GUI_ACTIVE/8 (cycles) {med['GRBM_GUI_ACTIVE'] / 8:.0f}")
