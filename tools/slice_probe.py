#!/usr/bin/env python3
"""Interleaved A/B of the sliced node table (gat_amd.h, gat_*_sliced) against
the row-major one, in ONE process: edge kernel alone, projection alone and the
whole layer forward, for slices in {1, 2, 4, 8} and V in {1, 2}.  Outputs are
checked bitwise against the row-major path.

    python tools/slice_probe.py --workload ppi --rounds 5
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

from tune_edge import time_fn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="ppi")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--slices", default="1,2,4,8")
    ap.add_argument("--vs", default="1,2")
    ap.add_argument("--us", default="")
    ap.add_argument("--pipes", default="0", help="GAT_EDGE_PIPE values (0 = default)")
    ap.add_argument("--lds", default="0", help="GAT_EDGE_LDS values (0 = none)")
    args = ap.parse_args()
    from atmlgraphattentionnetworks_amd import GraphAttentionLayer, _lib, get_csr
    from atmlgraphattentionnetworks_amd.layer import gat_forward
    from atmlgraphattentionnetworks_amd.synthetic import WORKLOADS, make_inputs
    from bench import edge_kernel_bytes

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
    hint = csr.num_edges // n
    bias = layer.bias.detach()
    order = csr.order

    def tables(s):
        wh = torch.empty(n * hf, device=dev)
        ss = torch.empty(n * H, device=dev)
        sd = torch.empty(n * H, device=dev)

        def proj():
            stream = torch.cuda.current_stream().cuda_stream  # the capture stream in a graph
            if s == 1:
                rc = lib.gat_project(x.data_ptr(), n, fin, pp.w.data_ptr(), pp.b.data_ptr(),
                                     pp.a_src.data_ptr(), pp.c_src.data_ptr(),
                                     pp.a_dst.data_ptr(), pp.c_dst.data_ptr(), H, F,
                                     wh.data_ptr(), hf, ss.data_ptr(), H, sd.data_ptr(), stream)
            else:
                rc = lib.gat_project_sliced(x.data_ptr(), n, fin, pp.w.data_ptr(),
                                            pp.b.data_ptr(), pp.a_src.data_ptr(),
                                            pp.c_src.data_ptr(), pp.a_dst.data_ptr(),
                                            pp.c_dst.data_ptr(), H, F, s, wh.data_ptr(), n,
                                            ss.data_ptr(), H, sd.data_ptr(), stream)
            _lib.check(rc, "project")
        return wh, sd, proj

    def edge_fn(s, wh, sd, out):
        def run():
            stream = torch.cuda.current_stream().cuda_stream
            if s == 1:
                rc = lib.gat_edge_aggregate(
                    csr.rowptr.data_ptr(), csr.col.data_ptr(), order.data_ptr(), 0, n,
                    wh.data_ptr(), hf, 0, H, pp.a_src.data_ptr(), pp.c_src.data_ptr(),
                    sd.data_ptr(), H, F, 1, 0.2, bias.data_ptr(), out.data_ptr(), 0, hint, stream)
            else:
                rc = lib.gat_edge_aggregate_sliced(
                    csr.rowptr.data_ptr(), csr.col.data_ptr(), order.data_ptr(), 0, n,
                    wh.data_ptr(), n, s, pp.a_src.data_ptr(), pp.c_src.data_ptr(),
                    sd.data_ptr(), H, F, 0.2, bias.data_ptr(), out.data_ptr(), hint, stream)
            _lib.check(rc, "edge")
        return run

    slices = [int(v) for v in args.slices.split(",")]
    vs = [int(v) for v in args.vs.split(",")]
    us = [int(v) for v in args.us.split(",")] if args.us else [0]
    occs = [int(v) for v in args.pipes.split(",")]
    ldss = [int(v) for v in args.lds.split(",")]
    variants = [(s, v, u, o, d) for s in slices for v in vs for u in us for o in occs for d in ldss]
    res = {k: [] for k in variants}
    pres = {s: [] for s in slices}
    fres = {s: [] for s in slices}
    outs = {}
    prepared = {}
    with torch.no_grad():
        for s in slices:
            wh, sd, proj = tables(s)
            proj()
            prepared[s] = (wh, sd, proj)
        for _ in range(args.rounds):
            for (s, v, u, o, d) in variants:
                os.environ["GAT_EDGE_LDS"] = str(d)
                os.environ["GAT_EDGE_V"] = str(v)
                os.environ["GAT_EDGE_PIPE"] = str(o)
                if u:
                    os.environ["GAT_EDGE_U"] = str(u)
                else:
                    os.environ.pop("GAT_EDGE_U", None)
                tuning.reload()
                wh, sd, _ = prepared[s]
                out = torch.empty(n, hf, device=dev)
                res[(s, v, u, o, d)].append(time_fn(edge_fn(s, wh, sd, out), args.iters))
                outs[(s, v, u, o, d)] = out
            os.environ.pop("GAT_EDGE_V", None)
            os.environ.pop("GAT_EDGE_U", None)
            os.environ.pop("GAT_EDGE_PIPE", None)
            os.environ.pop("GAT_EDGE_LDS", None)
            tuning.reload()
            for s in slices:
                pres[s].append(time_fn(prepared[s][2], args.iters))
                os.environ["GAT_WH_SLICES"] = str(s)
                tuning.reload()
                fres[s].append(time_fn(lambda: gat_forward(x, csr, pp, bias, H, F, True, 0.2),
                                       args.iters))
            os.environ.pop("GAT_WH_SLICES", None)
            tuning.reload()
    alg = edge_kernel_bytes(n, csr.num_edges, H, F, True)
    ref = outs[variants[0]]
    summary = {}
    for k, ts in res.items():
        med = statistics.median(ts)
        summary[f"edge_s{k[0]}_v{k[1]}_u{k[2]}_pipe{k[3]}_lds{k[4]}"] = {
            "median_ms": round(med, 5), "min_ms": round(min(ts), 5),
            "GBps_alg": round(alg / med / 1e6, 1),
            "max_abs_diff": float((outs[k] - ref).abs().max())}
    for s in slices:
        summary[f"proj_s{s}"] = {"median_ms": round(statistics.median(pres[s]), 5)}
        summary[f"layer_s{s}"] = {"median_ms": round(statistics.median(fres[s]), 5),
                                  "edges_per_s": csr.num_edges / statistics.median(fres[s]) * 1e3}
    print(json.dumps({"workload": args.workload, "N": n, "E'": csr.num_edges,
                      "results": summary}, indent=1))


if __name__ == "__main__":
    main()
