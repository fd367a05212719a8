#!/usr/bin/env python3
"""In-sequence A/B of the layer step's two kernels: projection then edge
kernel, eager launches back to back as in bench.py, with HIP events between
them, so each kernel is timed in the cache state the step leaves it (the
projection runs right after the previous step's edge kernel).  Variants are
library env knobs, interleaved over rounds in one process.

    python tools/step_probe.py --workload ppi --variants 'base:;u8:GAT_EDGE_U=8'
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from atmlgraphattentionnetworks_amd import tuning  # noqa: E402


def parse_variants(spec):
    out = {}
    for part in spec.split(";"):
        name, _, envs = part.partition(":")
        env = {}
        for kv in filter(None, envs.split(",")):
            k, _, v = kv.partition("=")
            env[k] = v
        out[name] = env
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="ppi")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--variants", default="base:")
    ap.add_argument("--double-proj", action="store_true",
                    help="run the projection twice per step and time the second one too")
    args = ap.parse_args()
    from atmlgraphattentionnetworks_amd import GraphAttentionLayer, get_csr
    from atmlgraphattentionnetworks_amd.layer import (alloc_table, edge_aggregate, project,
                                                      wh_slices)
    from atmlgraphattentionnetworks_amd.synthetic import WORKLOADS, make_inputs

    dev = torch.device("cuda", 0)
    w = WORKLOADS[args.workload]
    x, ei = make_inputs(w, dev)
    n = x.size(0)
    torch.manual_seed(0)
    layer = GraphAttentionLayer(w.in_channels, w.out_channels, num_heads=w.heads,
                                concat=w.concat).to(dev).eval()
    csr = get_csr(ei, n)
    del ei
    pp = layer.packed()
    H, F = w.heads, w.out_channels
    variants = parse_variants(args.variants)
    # PRED (probe-only key): work inserted before each step's projection —
    # fill (an 11.5-MB store kernel), read (an 11.5-MB reduction), sleep (a
    # ~20 us busy-wait kernel, no memory traffic), tinyproj (the projection
    # kernel itself on 64 rows)
    preds = {name: env.pop("PRED", "") for name, env in variants.items()}
    knobs = sorted({k for env in variants.values() for k in env})
    scratch = torch.empty(n, H * F, device=dev)
    x64 = x[:64].clone()
    s_dst64 = torch.empty(64, H, device=dev)
    table64 = None
    res = {name: {"project": [], "project2": [], "edge": [], "step": []} for name in variants}
    stream = torch.cuda.current_stream()
    with torch.no_grad():
        for _ in range(args.rounds):
            for name, env in variants.items():
                for k in knobs:
                    os.environ.pop(k, None)
                os.environ.update(env)
                tuning.reload()
                slices = wh_slices(H, F, w.concat, layer.negative_slope, csr.num_edges // n)
                table = alloc_table(n, H, F, dev, slices=slices)
                table64 = alloc_table(64, H, F, dev, slices=slices)
                s_dst = torch.empty(n, H, device=dev)
                out = torch.empty(n, H * F if w.concat else F, device=dev)
                evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)]
                       for _ in range(args.steps)]
                for _ in range(5):
                    project(x, pp, H, F, table=table, s_dst=s_dst)
                    edge_aggregate(csr, table, s_dst, H, F, w.concat, layer.bias, out=out, pp=pp)
                torch.cuda.synchronize()
                for e in evs:
                    if preds[name] == "fill":
                        scratch.fill_(1.0)
                    elif preds[name] == "read":
                        scratch.sum()
                    elif preds[name] == "sleep":
                        torch.cuda._sleep(50_000)
                    elif preds[name] == "tinyproj":  # the same projection kernel, 64 rows
                        project(x64, pp, H, F, table=table64, s_dst=s_dst64)
                    e[0].record(stream)
                    project(x, pp, H, F, table=table, s_dst=s_dst)
                    e[3].record(stream)
                    if args.double_proj:
                        project(x, pp, H, F, table=table, s_dst=s_dst)
                    e[1].record(stream)
                    edge_aggregate(csr, table, s_dst, H, F, w.concat, layer.bias, out=out, pp=pp)
                    e[2].record(stream)
                torch.cuda.synchronize()
                res[name]["project"].append(statistics.median(e[0].elapsed_time(e[3]) for e in evs))
                res[name]["project2"].append(statistics.median(e[3].elapsed_time(e[1]) for e in evs))
                res[name]["edge"].append(statistics.median(e[1].elapsed_time(e[2]) for e in evs))
                res[name]["step"].append(statistics.median(e[0].elapsed_time(e[2]) for e in evs))
    for k in knobs:
        os.environ.pop(k, None)
    summary = {name: {part: round(statistics.median(v) * 1e3, 2) for part, v in d.items()}
               for name, d in res.items()}
    print(json.dumps({"workload": args.workload, "unit": "us (median of per-step medians)",
                      "results": summary}, indent=1))


if __name__ == "__main__":
    main()
