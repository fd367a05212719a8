#!/usr/bin/env python3
"""Median per-dispatch value of every counter in rocprofv3 --pmc pass
directories, for the kernels whose name contains --match (default: the edge
kernel k_edge_grp), one JSON object per pass directory.

    python tools/pmc_kernel_summary.py --match k_edge_grp gpurun_out/r05r/pl_p*
"""
import argparse
import csv
import glob
import json
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--match", default="k_edge_grp")
    ap.add_argument("dirs", nargs="+")
    args = ap.parse_args()
    out = {}
    for d in args.dirs:
        per = {}
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(path)):
                if args.match not in r["Kernel_Name"]:
                    continue
                c = per.setdefault(int(r["Dispatch_Id"]), {})
                c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        if not per:
            continue
        names = sorted({k for c in per.values() for k in c})
        out[os.path.basename(d)] = {k: statistics.median(c.get(k, 0.0) for c in per.values())
                                    for k in names}
        out[os.path.basename(d)]["dispatches"] = len(per)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
