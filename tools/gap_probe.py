#!/usr/bin/env python3
"""Where does a layer step's time go between kernels?

Run mode (under rocprofv3 --kernel-trace): eager layer forwards back to back,
exactly as bench.py's timed loop, after a marker kernel.

    rocprofv3 --kernel-trace --output-format csv -d D -o run -- \
        python3 tools/gap_probe.py run --workload ppi --steps 200

Parse mode: per-kernel durations and the idle gaps between consecutive
dispatches (end of one -> start of the next) of the timed loop.

    python3 tools/gap_probe.py parse D/run_kernel_trace.csv
"""
import argparse
import csv
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(args):
    import torch
    from atmlgraphattentionnetworks_amd import GraphAttentionLayer
    from atmlgraphattentionnetworks_amd.synthetic import WORKLOADS, make_inputs
    dev = torch.device("cuda", 0)
    w = WORKLOADS[args.workload]
    x, ei = make_inputs(w, dev)
    torch.manual_seed(0)
    layer = GraphAttentionLayer(w.in_channels, w.out_channels, num_heads=w.heads,
                                concat=w.concat).to(dev).eval()
    with torch.no_grad():
        for _ in range(10):
            layer(x, ei)
        torch.cuda.synchronize()
        torch.zeros(1, device=dev).add_(1)  # marker: the timed loop follows
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            layer(x, ei)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / args.steps
    print(json.dumps({"workload": args.workload, "host_clock_us_per_step": ms * 1e3}))


def classify(name):
    if "k_project" in name:
        return "project"
    if "k_edge_merge" in name:
        return "merge"
    if "k_edge" in name:
        return "edge"
    return "other"


def parse(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the timed loop starts after the last 'elementwise' marker
    start = 0
    for i, r in enumerate(rows):
        if classify(r["Kernel_Name"]) == "other":
            start = i + 1
    rows = rows[start:]
    dur = {}
    gaps = {}
    prev = None
    for r in rows:
        k = classify(r["Kernel_Name"])
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        dur.setdefault(k, []).append((e - s) / 1e3)
        if prev is not None:
            gaps.setdefault(f"{prev[0]}->{k}", []).append((s - prev[1]) / 1e3)
        prev = (k, e)
    span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
    n_steps = len(dur.get("project", [])) or 1
    out = {"dispatches": len(rows), "steps": n_steps, "us_per_step_trace": span / n_steps,
           "kernel_us": {k: {"median": statistics.median(v), "mean": statistics.mean(v)}
                         for k, v in dur.items()},
           "gap_us": {k: {"median": statistics.median(v), "mean": statistics.mean(v),
                          "min": min(v), "max": max(v)} for k, v in gaps.items()}}
    print(json.dumps(out, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["run", "parse"])
    ap.add_argument("path", nargs="?")
    ap.add_argument("--workload", default="ppi")
    ap.add_argument("--steps", type=int, default=200)
    args = ap.parse_args()
    if args.mode == "run":
        run(args)
    else:
        parse(args.path)


if __name__ == "__main__":
    main()
