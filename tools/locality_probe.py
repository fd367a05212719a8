#!/usr/bin/env python3
"""Does sorting each CSR row's sources improve the edge kernel's L2 locality?
Times gat_edge_aggregate on the module's CSR (input order within a row) and
on the same CSR with each row's sources ascending, graph-captured, interleaved."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    from atmlgraphattentionnetworks_amd import GraphAttentionLayer, get_csr
    from atmlgraphattentionnetworks_amd.graph import CSRGraph
    from atmlgraphattentionnetworks_amd.layer import edge_aggregate, project
    from atmlgraphattentionnetworks_amd.synthetic import WORKLOADS, make_inputs
    for name in sys.argv[1:] or ["ppi", "arxiv", "reddit"]:
        w = WORKLOADS[name]
        dev = torch.device("cuda", 0)
        x, ei = make_inputs(w, dev)
        n = x.size(0)
        torch.manual_seed(0)
        layer = GraphAttentionLayer(w.in_channels, w.out_channels, num_heads=w.heads,
                                    concat=w.concat).to(dev).eval()
        csr = get_csr(ei, n)
        rp = csr.rowptr.long()
        row = torch.repeat_interleave(torch.arange(n, device=dev), rp[1:] - rp[:-1])
        key = row * n + csr.col.long()
        col2 = csr.col[torch.argsort(key)].contiguous()
        csr2 = CSRGraph(csr.rowptr, col2, n, csr.num_edges, csr.order)
        pp = layer.packed()
        with torch.no_grad():
            table, s_dst = project(x, pp, w.heads, w.out_channels)
            out = torch.empty(n, w.heads * w.out_channels, device=dev)
            ref = edge_aggregate(csr, table, s_dst, w.heads, w.out_channels, w.concat, layer.bias,
                                 pp=pp).clone()
            got = edge_aggregate(csr2, table, s_dst, w.heads, w.out_channels, w.concat,
                                 layer.bias, pp=pp)
            err = float((got - ref).abs().max())
            iters = 50 if name != "reddit" else 5
            res = {}
            graphs = {}
            for tag, c in (("input_order", csr), ("sorted_sources", csr2)):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(iters):
                        edge_aggregate(c, table, s_dst, w.heads, w.out_channels, w.concat,
                                       layer.bias, out=out, pp=pp)
                graphs[tag] = g
                res[tag] = []
            for _ in range(5):
                for tag, g in graphs.items():
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record()
                    g.replay()
                    e1.record()
                    e1.synchronize()
                    res[tag].append(e0.elapsed_time(e1) / iters * 1e3)
        print(name, {k: round(min(v), 2) for k, v in res.items()}, "us; max diff", err,
              flush=True)


if __name__ == "__main__":
    main()
