#!/usr/bin/env python3
"""Interleaved A/B timing of kernel variants in ONE process (methodology rule:
perf deltas from interleaved rounds on one device).  Variants are selected by
the library's env knobs; outputs are cross-checked against the first variant.

    python tools/tune_edge.py --workload ppi --rounds 5
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

EDGE_VARIANTS = {
    "generic": {"GAT_EDGE_KERNEL": "generic"},
    "gather_v1": {"GAT_EDGE_SCORE": "gather"},
    "fused_v1": {},
    "fused_v1_natural": {"GAT_EDGE_ORDER": "natural"},
    "fused_v2": {"GAT_EDGE_V": "2"},
    "fused_v2_natural": {"GAT_EDGE_V": "2", "GAT_EDGE_ORDER": "natural"},
    "fused_v2_u4": {"GAT_EDGE_V": "2", "GAT_EDGE_U": "4"},
    "fused_v2_u8": {"GAT_EDGE_V": "2", "GAT_EDGE_U": "8"},
    "fused_v2_u16": {"GAT_EDGE_V": "2", "GAT_EDGE_U": "16"},
    "fused_v1_u4": {"GAT_EDGE_U": "4"},
    "fused_v1_u16": {"GAT_EDGE_U": "16"},
}
REF_MM = True  # also time torch.mm(x, W^T) (hipBLASLt) as a projection reference point
PROJ_VARIANTS = {"generic": {"GAT_PROJ_KERNEL": "lds"}, "tiled": {"GAT_PROJ_KERNEL": "tiled"},
                 "wk": {}}


def set_env(d):
    for k in ("GAT_EDGE_KERNEL", "GAT_PROJ_KERNEL", "GAT_EDGE_U", "GAT_EDGE_SCORE", "GAT_EDGE_V",
              "GAT_EDGE_ORDER"):
        os.environ.pop(k, None)
    os.environ.update(d)
    tuning.reload()


def time_fn(fn, iters, reps=3):
    """Average GPU time per call: `iters` calls captured in one HIP graph and
    replayed, so host launch overhead does not leak into short kernels."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        g.replay()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / (iters * reps)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="ppi")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    from atmlgraphattentionnetworks_amd import GraphAttentionLayer, get_csr
    from atmlgraphattentionnetworks_amd.layer import alloc_table, edge_aggregate, project
    from atmlgraphattentionnetworks_amd.synthetic import WORKLOADS, make_inputs
    from bench import edge_kernel_bytes

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
    with torch.no_grad():
        set_env({})
        table, s_dst = project(x, pp, H, F)
        outs, res = {}, {k: [] for k in EDGE_VARIANTS}
        for r in range(args.rounds):
            for name, env in EDGE_VARIANTS.items():
                set_env(env)
                out = torch.empty(n, H * F if w.concat else F, device=dev)
                res[name].append(time_fn(lambda: edge_aggregate(
                    csr, table, s_dst, H, F, w.concat, layer.bias, out=out, pp=pp), args.iters))
                outs[name] = out
        ref = outs["generic"]
        alg = edge_kernel_bytes(n, csr.num_edges, H, F, w.concat)
        summary = {}
        for name, ts in res.items():
            med = statistics.median(ts)
            summary[name] = {"median_ms": med, "min_ms": min(ts), "GBps_alg": alg / med / 1e6,
                             "max_abs_diff_vs_generic": float((outs[name] - ref).abs().max())}
        pres, pouts = {k: [] for k in PROJ_VARIANTS}, {}
        for r in range(args.rounds):
            for name, env in PROJ_VARIANTS.items():
                set_env(env)
                if name == "wk" and x.size(1) > 128:
                    continue
                t2 = alloc_table(n, H, F, dev); s2 = torch.empty_like(s_dst)
                pres[name].append(time_fn(lambda: project(x, pp, H, F, table=t2, s_dst=s2),
                                          args.iters))
                pouts[name] = (t2, s2)
        for name, ts in pres.items():
            if not ts:
                continue
            summary["proj_" + name] = {
                "median_ms": statistics.median(ts), "min_ms": min(ts),
                "max_abs_diff_vs_generic": max(
                    float((pouts[name][0].wh - pouts["generic"][0].wh).abs().max()),
                    float((pouts[name][1] - pouts["generic"][1]).abs().max()))}
        if REF_MM:
            wt = pp.w.t().contiguous()
            summary["ref_torch_mm"] = {"median_ms": time_fn(lambda: torch.mm(x, wt), args.iters),
                                       "max_abs_diff_vs_generic": 0.0}
    print(json.dumps({"workload": args.workload, "N": n, "E'": csr.num_edges,
                      "alg_bytes": alg, "results": summary}, indent=1))


if __name__ == "__main__":
    main()
