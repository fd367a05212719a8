#!/usr/bin/env python3
"""Does the backward source pass (k_bwd_sources, rows in natural order) gain
from rows of equal out-degree running together, as the forward's rows run by
in-degree?  Relabels the nodes of a synthetic workload so that natural order
IS descending out-degree (x permuted alike: the same graph, other labels) and
times the training step; run it under rocprofv3 --kernel-trace --stats once
per order to read the per-kernel split.

    python tools/bwd_order_probe.py <workload> natural|outdeg [steps]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    from atmlgraphattentionnetworks_amd import GraphAttentionLayer
    from atmlgraphattentionnetworks_amd.synthetic import WORKLOADS, make_inputs
    name, mode = sys.argv[1], sys.argv[2]
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    w = WORKLOADS[name]
    dev = torch.device("cuda", 0)
    x, ei = make_inputs(w, dev)
    n = x.size(0)
    if mode == "outdeg":
        outdeg = torch.bincount(ei[0], minlength=n)
        perm = torch.sort(-outdeg, stable=True).indices      # new label k -> old node perm[k]
        new_id = torch.empty_like(perm)
        new_id[perm] = torch.arange(n, device=dev)
        ei = new_id[ei]
        x = x[perm].contiguous()
    elif mode != "natural":
        raise SystemExit("mode: natural | outdeg")
    torch.manual_seed(0)
    layer = GraphAttentionLayer(w.in_channels, w.out_channels, num_heads=w.heads,
                                concat=w.concat, dropout=0.6).to(dev).train()
    opt = torch.optim.Adam(layer.parameters(), lr=1e-3)
    gout = torch.randn(n, w.heads * w.out_channels if w.concat else w.out_channels, device=dev)

    def step():
        opt.zero_grad(set_to_none=True)
        layer(x, ei).backward(gout)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        step()
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"workload": name, "order": mode, "steps": steps,
                      "train_step_ms": round(e0.elapsed_time(e1) / steps, 4)}))


if __name__ == "__main__":
    main()
