#!/usr/bin/env python3
"""Workload runner for rocprofv3 --pmc passes (see tools/pmc_collect.sh).

Launches, on one GPU: a calibration streaming copy of a known byte count
(torch copy_, 1 GiB -> 1 GiB) and then `--iters` launches of the edge kernel
and the projection for the workload.  tools/pmc_traffic.py turns the counter
CSVs into profiles/pmc_<workload>.json.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

CALIB_BYTES = 1 << 30


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="ppi")
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    from atmlgraphattentionnetworks_amd import GraphAttentionLayer, get_csr
    from atmlgraphattentionnetworks_amd.layer import alloc_table, edge_aggregate, project, wh_slices
    from atmlgraphattentionnetworks_amd.synthetic import WORKLOADS, make_inputs

    dev = torch.device("cuda", 0)
    a = torch.empty(CALIB_BYTES // 4, dtype=torch.float32, device=dev).normal_()
    b = torch.empty_like(a)
    for _ in range(3):
        b.copy_(a)
    torch.cuda.synchronize()
    del a, b
    w = WORKLOADS[args.workload]
    x, ei = make_inputs(w, dev)
    torch.manual_seed(0)
    layer = GraphAttentionLayer(w.in_channels, w.out_channels, num_heads=w.heads,
                                concat=w.concat).to(dev).eval()
    csr = get_csr(ei, x.size(0))
    del ei
    with torch.no_grad():
        pp = layer.packed()
        slices = wh_slices(w.heads, w.out_channels, w.concat, layer.negative_slope,
                           csr.num_edges // x.size(0))  # the layout the layer uses
        table, s_dst = project(x, pp, w.heads, w.out_channels,
                               table=alloc_table(x.size(0), w.heads, w.out_channels, dev,
                                                 slices=slices))
        out = None
        for _ in range(args.iters):
            project(x, pp, w.heads, w.out_channels, table=table, s_dst=s_dst)
            out = edge_aggregate(csr, table, s_dst, w.heads, w.out_channels, w.concat,
                                 layer.bias, out=out, pp=pp)
        torch.cuda.synchronize()
    print(f"pmc_run done: {args.workload} N={x.size(0)} E'={csr.num_edges} slices={slices}")


if __name__ == "__main__":
    main()
