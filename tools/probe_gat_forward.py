#!/usr/bin/env python3
"""Why gat_forward (a ForwardPlan per call) runs arxiv at ~1 ms in the --dist
bench's one-GPU reference while the layer's cached plan takes ~0.1 ms: times
each piece of the per-call path (plan construction, projection, edge kernel)
with a host clock around synchronized calls, and torch.profiler's op list.

    python tools/probe_gat_forward.py --workload arxiv
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def clock(fn, iters):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="arxiv")
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    from atmlgraphattentionnetworks_amd import _lib
    from atmlgraphattentionnetworks_amd.graph import build_csr
    from atmlgraphattentionnetworks_amd.layer import ForwardPlan, gat_forward
    from atmlgraphattentionnetworks_amd.distributed import _make_layer
    from atmlgraphattentionnetworks_amd.synthetic import WORKLOADS, make_inputs
    dev = torch.device("cuda", 0)
    w = WORKLOADS[args.workload]
    x, ei = make_inputs(w, dev)
    csr = build_csr(ei, x.size(0))
    layer = _make_layer(w, dev)
    lib = _lib.load()
    res = {"workload": w.name}
    with torch.no_grad():
        pp = layer.packed()
        bias = layer.bias.detach()

        def fwd():
            return gat_forward(x, csr, pp, bias, w.heads, w.out_channels, w.concat, 0.2)

        for _ in range(3):
            fwd()
        res["gat_forward_ms"] = clock(fwd, args.iters)
        res["layer_cached_plan_ms"] = clock(lambda: layer(x, ei), args.iters)
        res["plan_ctor_ms"] = clock(lambda: ForwardPlan(x, csr, w.heads, w.out_channels,
                                                        w.concat, 0.2), args.iters)
        plan = ForwardPlan(x, csr, w.heads, w.out_channels, w.concat, 0.2)
        out = torch.empty(x.size(0), w.heads * w.out_channels, device=dev)
        res["project_ms"] = clock(lambda: plan.project(lib, x, pp), args.iters)
        res["edge_ms"] = clock(lambda: plan.edge(lib, csr, pp, bias, out), args.iters)
        res["kernel"] = plan.kernel_name()
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            for _ in range(3):
                fwd()
            torch.cuda.synchronize()
        res["profile"] = prof.key_averages().table(sort_by="cpu_time_total", row_limit=15)
    print(json.dumps({k: v for k, v in res.items() if k != "profile"}))
    print(res["profile"])


if __name__ == "__main__":
    main()
