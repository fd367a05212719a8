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
    if "copyBuffer" in name:
        return "copy"
    return "other"


def load(dirs):
    """{kind: {counter: median per-dispatch value}}; for the copies only the
    calibration copy (the dispatch with the largest read count) is kept."""
    per = {}  # (kind, dispatch) -> {counter: value}
    names = {}
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(path)):
                kind = classify(r["Kernel_Name"])
                if kind == "other":
                    continue
                names[kind] = r["Kernel_Name"][:100]
                key = (kind, d, r["Dispatch_Id"])
                c = per.setdefault(key, {})
                c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    out = {}
    by_kind_ctr = {}
    for (kind, d, _), ctrs in per.items():
        for ctr, v in ctrs.items():
            by_kind_ctr.setdefault((kind, ctr, d), []).append(v)
    for (kind, ctr, d), vals in by_kind_ctr.items():
        if kind == "copy":
            val = max(vals)  # the 1 GiB calibration copy
        else:
            val = statistics.median(vals)
        out.setdefault(kind, {})[ctr] = val
    names["calib_copy"] = names.pop("copy", None)
    out["calib_copy"] = out.pop("copy", {})
    return out, names


def req_bytes(c):
    """Exact L2->fabric read bytes from the per-size request counters."""
    keys = ("TCC_EA0_RDREQ_128B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_32B_sum")
    if not all(k in c for k in keys):
        return None
    return 128 * c[keys[0]] + 64 * c[keys[1]] + 32 * c[keys[2]]


def main():
    workload = sys.argv[1]
    counters, names = load(sys.argv[2:])
    res = {"workload": workload, "kernels": names, "counters_median_per_launch": counters}
    calib = counters.get("calib_copy", {})
    f_ratio = w_ratio = r_ratio = None
    if calib.get("FETCH_SIZE"):
        f_ratio = CALIB_BYTES / (calib["FETCH_SIZE"] * 1024.0)
    if calib.get("WRITE_SIZE"):
        w_ratio = CALIB_BYTES / (calib["WRITE_SIZE"] * 1024.0)
    if req_bytes(calib):
        r_ratio = CALIB_BYTES / req_bytes(calib)
    res["calibration"] = {"copy_bytes_each_way": CALIB_BYTES,
                          "fetch_size_correction": f_ratio, "write_size_correction": w_ratio,
                          "request_bytes_correction": r_ratio}
    for kind in ("edge", "project"):
        c = counters.get(kind, {})
        rd = req_bytes(c)
        if rd is None and "FETCH_SIZE" in c:
            rd = c["FETCH_SIZE"] * 1024.0 * (f_ratio or 1.0)
        elif rd is not None and r_ratio:
            rd *= r_ratio
        wr = c["WRITE_SIZE"] * 1024.0 * (w_ratio or 1.0) if "WRITE_SIZE" in c else None
        res[f"{kind}_kernel_read_bytes"] = rd
        res[f"{kind}_kernel_write_bytes"] = wr
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
            tot = c["TCC_HIT_sum"] + c["TCC_MISS_sum"]
            res[f"{kind}_kernel_l2_hit_rate"] = c["TCC_HIT_sum"] / tot if tot else None
    if res.get("edge_kernel_read_bytes") is not None and res.get("edge_kernel_write_bytes") is not None:
        # L2 -> memory-fabric bytes per launch; Infinity Cache hits are included
        # (no MALL hit counter at the TCC), so this bounds the HBM bytes from above
        res["edge_kernel_hbm_bytes_per_launch"] = (res["edge_kernel_read_bytes"] +
                                                   res["edge_kernel_write_bytes"])
    path = os.environ.get("PMC_OUT") or os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
