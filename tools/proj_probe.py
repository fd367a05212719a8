#!/usr/bin/env python3
"""Projection kernel time by cache state: hot (back-to-back), after a 512 MB
streaming write (L2 + Infinity Cache flushed), and after the edge kernel
(the state it runs in inside a layer step).  Events bracket ONLY the
projection launch in each case."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    from atmlgraphattentionnetworks_amd import GraphAttentionLayer, get_csr
    from atmlgraphattentionnetworks_amd.layer import edge_aggregate, project
    from atmlgraphattentionnetworks_amd.synthetic import WORKLOADS, make_inputs
    w = WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "ppi"]
    dev = torch.device("cuda", 0)
    x, ei = make_inputs(w, dev)
    layer = GraphAttentionLayer(w.in_channels, w.out_channels, num_heads=w.heads,
                                concat=w.concat).to(dev).eval()
    csr = get_csr(ei, x.size(0))
    pp = layer.packed()
    H, F = w.heads, w.out_channels
    flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream()
    with torch.no_grad():
        table, s_dst = project(x, pp, H, F)
        out = edge_aggregate(csr, table, s_dst, H, F, w.concat, layer.bias, pp=pp)
        res = {"hot": [], "after_flush": [], "after_edge": []}
        for _ in range(30):
            for case in res:
                if case == "after_flush":
                    flush.fill_(1)
                elif case == "after_edge":
                    edge_aggregate(csr, table, s_dst, H, F, w.concat, layer.bias, out=out, pp=pp)
                else:
                    project(x, pp, H, F, table=table, s_dst=s_dst)
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(s)
                project(x, pp, H, F, table=table, s_dst=s_dst)
                e1.record(s)
                e1.synchronize()
                res[case].append(e0.elapsed_time(e1) * 1e3)
    for k, v in res.items():
        print(f"project {k:12s} median {statistics.median(v):7.2f} us  min {min(v):7.2f} us")


if __name__ == "__main__":
    main()
