#!/usr/bin/env python3
"""Interleaved A/B of the layer's eager eval step (bench.py's headline loop:
``layer(x, ei)`` back to back, host clock around K synchronized steps) under
environment variants, in ONE process.  A variant is ``name:K=V,K=V`` (knobs,
or any variable the layer reads when it builds its cached plan); each round
builds a fresh layer per variant from the same parameters.

    python tools/step_ab.py --workload ppi --rounds 5 --variants "base:;plain:GAT_EDGE_SCHED=plain"
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="ppi")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--variants", default="base:")
    args = ap.parse_args()
    from atmlgraphattentionnetworks_amd import GraphAttentionLayer, tuning
    from atmlgraphattentionnetworks_amd.graph import get_csr
    from atmlgraphattentionnetworks_amd.synthetic import WORKLOADS, make_inputs
    w = WORKLOADS[args.workload]
    dev = torch.device("cuda", 0)
    x, ei = make_inputs(w, dev)
    get_csr(ei, x.size(0))
    torch.manual_seed(0)
    state = GraphAttentionLayer(w.in_channels, w.out_channels, num_heads=w.heads,
                                concat=w.concat).state_dict()
    variants = []
    for spec in args.variants.split(";"):
        name, _, kv = spec.partition(":")
        env = dict(p.split("=", 1) for p in kv.split(",") if p)
        variants.append((name, env))
    keys = {k for _, env in variants for k in env}
    res = {name: [] for name, _ in variants}
    outs = {}
    for _ in range(args.rounds):
        for name, env in variants:
            for k in keys:
                os.environ.pop(k, None)
            os.environ.update(env)
            tuning.reload()
            layer = GraphAttentionLayer(w.in_channels, w.out_channels, num_heads=w.heads,
                                        concat=w.concat)
            layer.load_state_dict(state)
            layer = layer.to(dev).eval()
            with torch.no_grad():
                for _ in range(10):
                    layer(x, ei)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(args.steps):
                    y = layer(x, ei)
                torch.cuda.synchronize()
                res[name].append((time.perf_counter() - t0) * 1e3 / args.steps)
                outs[name] = y.clone()
            del layer
    ref = outs[variants[0][0]]
    print(json.dumps({"workload": args.workload, "steps": args.steps, "results": {
        name: {"step_ms_median": statistics.median(v), "step_ms_min": min(v),
               "edges_per_s": get_csr(ei, x.size(0)).num_edges / statistics.median(v) * 1e3,
               "max_abs_diff_vs_first": float((outs[name] - ref).abs().max())}
        for name, v in res.items()}}, indent=1))


if __name__ == "__main__":
    main()
