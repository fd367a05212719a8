#!/usr/bin/env python3
"""Interleaved A/B of projection variants (the layer's own table layout) in
ONE process, with each variant's error against a float64 torch restatement of
Wh = x W^T + b and s_dst (GAT.py:42-52).  Variants are GAT_* knob sets.

    python tools/proj_ab.py --workload arxiv --variants "base"
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from edge_ab import apply, parse  # noqa: E402
from timing import time_fn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="arxiv")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--variants", default="base")
    args = ap.parse_args()
    from atmlgraphattentionnetworks_amd import GraphAttentionLayer, _lib, get_csr
    from atmlgraphattentionnetworks_amd.layer import ForwardPlan
    from atmlgraphattentionnetworks_amd.synthetic import WORKLOADS, make_inputs

    lib = _lib.load()
    dev = torch.device("cuda", 0)
    w = WORKLOADS[args.workload]
    x, ei = make_inputs(w, dev)
    n, fin = x.shape
    torch.manual_seed(0)
    layer = GraphAttentionLayer(w.in_channels, w.out_channels, num_heads=w.heads,
                                concat=w.concat).to(dev).eval()
    csr = get_csr(ei, n)
    del ei
    pp = layer.packed()
    H, F = w.heads, w.out_channels
    hf = H * F
    # float64 reference (GAT.py:42-45): Wh = x W^T + b; s_dst = Wh_h . a2_h + c2_h
    wh64 = x.double() @ pp.w.double().t() + pp.b.double()
    sd64 = (wh64.view(n, H, F) * pp.a_dst.double().view(1, H, F)).sum(-1) + \
        pp.c_dst.double().view(1, H)
    ss64 = (wh64.view(n, H, F) * pp.a_src.double().view(1, H, F)).sum(-1) + \
        pp.c_src.double().view(1, H)
    specs = [s.strip() for s in args.variants.split(";") if s.strip()]
    envs = [parse(s) for s in specs]
    plans = []
    with torch.no_grad():
        for e in envs:
            apply(e)
            plans.append(ForwardPlan(x, csr, H, F, w.concat, 0.2))
        res = {s: [] for s in specs}
        for _ in range(args.rounds):
            for s, e, plan in zip(specs, envs, plans):
                apply(e)
                res[s].append(time_fn(lambda: plan.project(lib, x, pp), args.iters))
        summary = {}
        flops = 2.0 * n * fin * hf
        for s, e, plan in zip(specs, envs, plans):
            apply(e)
            plan.project(lib, x, pp)
            torch.cuda.synchronize()
            nw = n * plan.hfp
            ws = plan.ws
            if plan.slices > 1:
                sw = hf // plan.slices
                planes = ws[:n * hf].view(plan.slices, n, sw)
                wh = torch.cat([planes[g] for g in range(plan.slices)], dim=1)
            else:
                wh = ws[:nw].view(n, plan.hfp)[:, :hf]
            sd = ws[nw + n * H:nw + 2 * n * H].view(n, H)
            ss = ws[nw:nw + n * H].view(n, H)
            med = statistics.median(res[s])
            err = (wh.double() - wh64).abs()
            summary[s] = {
                "median_ms": round(med, 5), "min_ms": round(min(res[s]), 5),
                "TFLOPs": flops / (med * 1e-3) / 1e12,
                "wh_max_abs_err_vs_f64": float(err.max()),
                "wh_max_rel_err_vs_f64": float((err / (wh64.abs() + 1e-6)).max()),
                "wh_max_abs_f64": float(wh64.abs().max()),
                "s_dst_max_abs_err_vs_f64": float((sd.double() - sd64).abs().max()),
                "slices": plan.slices}
            if plan.slices == 1:
                summary[s]["s_src_max_abs_err_vs_f64"] = float((ss.double() - ss64).abs().max())
                # rows where the three outputs disagree most (bug hunting)
                e_rows = err.max(1).values
                summary[s]["worst_rows"] = torch.topk(e_rows, 5).indices.tolist()
        apply({})
    print(json.dumps({"workload": args.workload, "N": n, "Fin": fin, "HF": hf,
                      "results": summary}, indent=1))


if __name__ == "__main__":
    main()
