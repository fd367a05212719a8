#!/usr/bin/env python3
"""Parse rocprofv3 --pmc counter CSVs (one directory per pass) into
profiles/pmc_<workload>.json: per-launch counter means for the edge kernel,
the projection and the calibration copy.

HBM-traffic correction (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7):
FETCH_SIZE on gfx950 reads ½ of the bytes of a wide coalesced streaming read;
WRITE_SIZE is exact for 16-B streaming stores.  The calibration copy (known
bytes) measures that factor in THIS run; the edge kernel's gather pattern is
outside the guide's calibrated cases, so the JSON carries the raw counters, the
calibration ratios and the corrected estimate side by side.

    python tools/pmc_traffic.py ppi gpurun_out/pmc_ppi_fetch gpurun_out/pmc_ppi_write ...
"""
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CALIB_BYTES = 1 << 30


def classify(name: str) -> str:
    if "k_edge" in name:
        return "edge"
    if "k_project" in name:
        return "project"
    if "copy" in name.lower() and "elementwise" in name.lower() or "CopyKernel" in name:
        return "calib_copy"
    return "other"


def load(dirs):
    per = {}  # (kind, counter) -> [values per dispatch]
    names = {}
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(path)):
                kind = classify(r["Kernel_Name"])
                if kind == "other":
                    continue
                names[kind] = r["Kernel_Name"][:100]
                per.setdefault((kind, r["Counter_Name"]), {}).setdefault(
                    r["Dispatch_Id"], 0.0)
                per[(kind, r["Counter_Name"])][r["Dispatch_Id"]] += float(r["Counter_Value"])
    out = {}
    for (kind, ctr), by_dispatch in per.items():
        vals = list(by_dispatch.values())
        if kind == "calib_copy":
            vals = vals[-1:]  # the last (warm) copy
        out.setdefault(kind, {})[ctr] = statistics.median(vals)
    return out, names


def main():
    workload = sys.argv[1]
    counters, names = load(sys.argv[2:])
    res = {"workload": workload, "kernels": names, "counters_median_per_launch": counters}
    calib = counters.get("calib_copy", {})
    f_ratio = w_ratio = None
    if "FETCH_SIZE" in calib:
        f_ratio = CALIB_BYTES / (calib["FETCH_SIZE"] * 1024.0)
    if "WRITE_SIZE" in calib:
        w_ratio = CALIB_BYTES / (calib["WRITE_SIZE"] * 1024.0)
    res["calibration"] = {"copy_bytes_each_way": CALIB_BYTES,
                          "fetch_correction": f_ratio, "write_correction": w_ratio}
    edge = counters.get("edge", {})
    if "FETCH_SIZE" in edge and "WRITE_SIZE" in edge:
        raw = (edge["FETCH_SIZE"] + edge["WRITE_SIZE"]) * 1024.0
        corr = (edge["FETCH_SIZE"] * (f_ratio or 1.0) + edge["WRITE_SIZE"] * (w_ratio or 1.0)) * 1024.0
        res["edge_kernel_hbm_bytes_raw"] = raw
        res["edge_kernel_hbm_bytes_per_launch"] = corr
    if "TCC_HIT_sum" in edge and "TCC_MISS_sum" in edge:
        tot = edge["TCC_HIT_sum"] + edge["TCC_MISS_sum"]
        res["edge_kernel_l2_hit_rate"] = edge["TCC_HIT_sum"] / tot if tot else None
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    path = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    with open(path, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
