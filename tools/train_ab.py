#!/usr/bin/env python3
"""Interleaved A/B of library env knobs on the layer's training step
(forward with dropout + HIP backward), timed with events in one process.
The gradient cross-check is meaningful only with --dropout 0: the dropout
seed comes from a device counter that torch.manual_seed does not reset.

    python tools/train_ab.py --workload reddit --variants 'base:;nokink:GAT_BWD_KINK=0'
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

from atmlgraphattentionnetworks_amd import tuning  # noqa: E402

from step_probe import parse_variants  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="ppi")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--dropout", type=float, default=0.6)
    ap.add_argument("--variants", default="base:")
    args = ap.parse_args()
    from atmlgraphattentionnetworks_amd import GraphAttentionLayer
    from atmlgraphattentionnetworks_amd.synthetic import WORKLOADS, make_inputs

    dev = torch.device("cuda", 0)
    w = WORKLOADS[args.workload]
    x, ei = make_inputs(w, dev)
    torch.manual_seed(0)
    layer = GraphAttentionLayer(w.in_channels, w.out_channels, num_heads=w.heads,
                                concat=w.concat, dropout=args.dropout).to(dev).train()
    gout = torch.randn(x.size(0), w.heads * w.out_channels if w.concat else w.out_channels,
                       device=dev)
    variants = parse_variants(args.variants)
    knobs = sorted({k for env in variants.values() for k in env})

    def step():
        layer.zero_grad(set_to_none=True)
        layer(x, ei).backward(gout)

    res = {name: [] for name in variants}
    grads = {}
    for _ in range(args.rounds):
        for name, env in variants.items():
            for k in knobs:
                os.environ.pop(k, None)
            os.environ.update(env)
            tuning.reload()
            torch.manual_seed(1)
            for _ in range(2):
                step()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.steps):
                step()
            e1.record()
            e1.synchronize()
            res[name].append(e0.elapsed_time(e1) / args.steps)
            grads[name] = layer.ws[0].weight.grad.detach().clone()
    for k in knobs:
        os.environ.pop(k, None)
    ref = next(iter(grads.values()))
    print(json.dumps({"workload": args.workload, "unit": "ms per training step",
                      "results": {n: {"median_ms": round(statistics.median(v), 4),
                                      "min_ms": round(min(v), 4),
                                      "max_abs_dW0_vs_first": float((grads[n] - ref).abs().max())}
                                  for n, v in res.items()}}, indent=1))


if __name__ == "__main__":
    main()
