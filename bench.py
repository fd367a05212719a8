#!/usr/bin/env python3
"""Benchmark: edges/sec through the 8-head GAT layer forward, PPI shape.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload ppi|reddit|arxiv|cifar...]

A "step" is one GraphAttentionLayer forward (eval, fp32) over the synthetic
PPI-shape graph (BASELINE.json configs[1]: N=44,906, E=1,226,368 + N loops,
Fin=50, H=8, F=8, concat) with inputs resident in HBM: the HIP projection +
the fused edge kernel.  The CSR (built once per edge_index and cached, as in
the module) is outside the timed region; it is timed separately.

Prints ONE JSON line (rank 0).  See DESIGN.md "Measurement".
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md: 8.0 TB/s)
MFMA_F32_PEAK_TFLOPS = 157.3  # dense fp32 matrix peak (v_mfma_f32_16x16x4_f32)
METRIC = "edges/sec through 8-head GAT layer forward, PPI shape, at 1/2/4/8 MI355X"


def edge_kernel_bytes(n_rows: int, n_edges: int, heads: int, f: int, concat: bool) -> int:
    """Algorithmic HBM bytes of one edge-kernel launch:
    per edge 4 (col) + 4*H*F (Wh_j) + 4*H (s_src_j); per target row
    4 (rowptr) + 4*H (s_dst) + 4*C_out (output write)."""
    c_out = heads * f if concat else f
    return n_edges * (4 + 4 * heads * f + 4 * heads) + n_rows * (4 + 4 * heads + 4 * c_out)


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def load_traffic(workload: str):
    """Per-launch HBM bytes of the edge kernel from the committed PMC summary
    (tools/pmc_traffic.py -> profiles/pmc_<workload>.json), if present."""
    path = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    try:
        with open(path) as fh:
            d = json.load(fh)
        return d.get("edge_kernel_hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def cpu_baseline(layer_state, x, ei, heads, concat, n_edges_total, budget_s: float = 10.0):
    """The oracle (pure-PyTorch restatement of GAT.py:37-67, same op order)
    on the host cores over the same synthetic workload: at least 5 timed
    forwards after one warm-up (SURVEY.md §8d's rule), continuing to ~budget_s
    of CPU work (at most 40), median reported."""
    from oracle import gat_layer_forward_from_state

    threads = torch.get_num_threads()
    xc, eic = x.cpu(), ei.cpu()
    st = {k: v.cpu() for k, v in layer_state.items()}
    gat_layer_forward_from_state(st, xc, eic, heads, concat)  # warm-up
    times = []
    t_start = time.perf_counter()
    while len(times) < 40 and (len(times) < 5 or (time.perf_counter() - t_start) < budget_s):
        t0 = time.perf_counter()
        gat_layer_forward_from_state(st, xc, eic, heads, concat)
        times.append(time.perf_counter() - t0)
    med = statistics.median(times)
    return {"value": n_edges_total / med, "unit": "edges/s", "cores": threads, "kind": "port",
            "sample": (f"full workload, {len(times)} timed fwd after 1 warm-up, median "
                       f"{med * 1e3:.1f} ms; oracle/gat_oracle.py (torch CPU, "
                       f"{threads} threads, {cpu_model()})")}


def time_edge_kernel(layer, x, csr, iters: int):
    """Mean launch time (ms) of the edge kernel the layer's eval forward uses,
    on a node table in that forward's layout (layer.wh_slices), with HIP
    events on the stream it is launched on.  Returns (ms, slices)."""
    from atmlgraphattentionnetworks_amd.layer import (alloc_table, edge_aggregate, project,
                                                      wh_slices)
    n = x.size(0)
    heads, f = layer.num_heads, layer.output_channels
    pp = layer.packed()
    slices = wh_slices(heads, f, layer.concat, layer.negative_slope,
                       csr.num_edges // max(n, 1))
    table, s_dst = project(x, pp, heads, f,
                           table=alloc_table(n, heads, f, x.device, slices=slices))
    out = torch.empty(n, heads * f if layer.concat else f, device=x.device)

    def run():
        edge_aggregate(csr, table, s_dst, heads, f, layer.concat, layer.bias, out=out, pp=pp)

    for _ in range(5):
        run()
    stream = torch.cuda.current_stream()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for _ in range(iters):
        run()
    ev1.record(stream)
    ev1.synchronize()
    return ev0.elapsed_time(ev1) / iters, slices


def edge_kernel_name(slices: int) -> str:
    return ("gat_edge_aggregate_sliced (k_edge_grp, %d column planes)" % slices if slices > 1
            else "gat_edge_aggregate (k_edge_grp)")


def train_step(layer, x, ei, n_edges: int, steps: int) -> dict:
    """One training step of the layer: forward in training
    mode with the layer's attention dropout (0.6, GAT.py:61) and the HIP
    backward to x and every parameter, with a fixed upstream gradient; timed
    with events over ``steps`` steps.  Not part of ``value`` (the metric is the
    eval forward)."""
    layer.train()
    xg = x.detach().clone().requires_grad_(True)
    gout = torch.randn(x.size(0), layer.num_heads * layer.output_channels if layer.concat
                       else layer.output_channels, device=x.device)

    def one():
        layer.zero_grad(set_to_none=True)
        xg.grad = None
        layer(xg, ei).backward(gout)

    for _ in range(5):
        one()
    stream = torch.cuda.current_stream()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    ev0.record(stream)
    for _ in range(steps):
        one()
    ev1.record(stream)
    ev1.synchronize()
    step_ms = ev0.elapsed_time(ev1) / steps
    with torch.no_grad():
        for _ in range(3):
            layer(x, ei)
        ev0.record(stream)
        for _ in range(steps):
            layer(x, ei)
        ev1.record(stream)
        ev1.synchronize()
    fwd_ms = ev0.elapsed_time(ev1) / steps
    # the same step captured in a HIP graph (device-seeded dropout: a fresh mask
    # per replay), as a trainer that graphs its step runs it
    graph_ms = None
    try:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                one()
        torch.cuda.current_stream().wait_stream(s)
        layer.zero_grad(set_to_none=True)
        xg.grad = None
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            layer(xg, ei).backward(gout)
        for _ in range(3):
            g.replay()
        ev0.record(stream)
        for _ in range(steps):
            g.replay()
        ev1.record(stream)
        ev1.synchronize()
        graph_ms = ev0.elapsed_time(ev1) / steps
    except Exception:  # noqa: BLE001  (the eager number above stands alone)
        graph_ms = None
    layer.eval()
    return {"what": "layer forward (training mode, attention dropout 0.6) + HIP backward to x "
                    "and all parameters",
            "train_step_ms": step_ms, "forward_train_ms": fwd_ms,
            "backward_ms": step_ms - fwd_ms, "train_edges_per_s": n_edges / (step_ms * 1e-3),
            "train_step_graph_ms": graph_ms,
            "train_edges_per_s_graph": None if not graph_ms else n_edges / (graph_ms * 1e-3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="ppi")
    ap.add_argument("--graph", action="store_true",
                    help="replay each step as a captured HIP graph (default: eager launches, "
                         "which measured faster: the host enqueue of a step is shorter than its "
                         "GPU time, and graph replays add a ~9 us gap each)")
    ap.add_argument("--no-graph", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--edge-iters", type=int, default=50)
    ap.add_argument("--dist", action="store_true",
                    help="take the torch.distributed path even at WORLD_SIZE=1 (testing)")
    ap.add_argument("--no-strong-probe", action="store_true",
                    help="multi-GPU: skip the strong-scaling all-gather/replicate measurement")
    ap.add_argument("--no-train", action="store_true",
                    help="skip the training-step (forward with dropout + backward) measurement")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if world > 1 or args.gpus > 1 or args.dist:
        from atmlgraphattentionnetworks_amd.distributed import bench_distributed
        return bench_distributed(args, METRIC)

    from atmlgraphattentionnetworks_amd import GraphAttentionLayer, get_csr
    from atmlgraphattentionnetworks_amd.layer import project
    from atmlgraphattentionnetworks_amd.synthetic import WORKLOADS, make_inputs

    dev = torch.device("cuda", 0)
    w = WORKLOADS[args.workload]
    x, ei = make_inputs(w, dev)
    n = x.size(0)
    torch.manual_seed(0)
    layer = GraphAttentionLayer(w.in_channels, w.out_channels, num_heads=w.heads,
                                concat=w.concat).to(dev).eval()

    # CSR build (one-time, cached by the module): timed separately
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    csr = get_csr(ei, n)
    torch.cuda.synchronize()
    csr_ms = (time.perf_counter() - t0) * 1e3
    n_edges = csr.num_edges

    def step():
        return layer(x, ei)

    with torch.no_grad():
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        graph = None
        if args.graph and not args.no_graph:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                step()
            torch.cuda.current_stream().wait_stream(s)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                static_out = step()
            run = graph.replay
        else:
            run = step
        for _ in range(args.warmup):
            run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            run()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        ms_per_step = elapsed * 1e3 / args.steps

        # edge kernel alone, in the layer's table layout, HIP events on its stream
        edge_ms, slices = time_edge_kernel(layer, x, csr, args.edge_iters)
        pp = layer.packed()
        table, s_dst = project(x, pp, w.heads, w.out_channels)
        stream = torch.cuda.current_stream()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        # projection alone: short kernel, so time launches captured in a graph
        gp = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gp):
            for _ in range(args.edge_iters):
                project(x, pp, w.heads, w.out_channels, table=table, s_dst=s_dst)
        gp.replay()
        ev0.record(stream)
        gp.replay()
        ev1.record(stream)
        ev1.synchronize()
        proj_ms = ev0.elapsed_time(ev1) / args.edge_iters

    training = None if args.no_train else train_step(layer, x, ei, n_edges, args.steps)

    alg_bytes = edge_kernel_bytes(n, n_edges, w.heads, w.out_channels, w.concat)
    proj_tflops = 2.0 * n * w.in_channels * w.heads * w.out_channels / (proj_ms * 1e-3) / 1e12
    achieved = alg_bytes / (edge_ms * 1e-3) / 1e9
    traffic = load_traffic(args.workload)
    result = {
        "metric": METRIC,
        "value": n_edges / (ms_per_step * 1e-3),
        "unit": "edges/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded uniform graph of the PPI shape; reference-order random init)",
        "config": {"workload": f"{w.name}: N={n} E={w.num_edges if w.kind == 'uniform' else ei.size(1)}"
                               f" (+N self-loops = {n_edges}) Fin={w.in_channels} H={w.heads}"
                               f" F={w.out_channels} concat={w.concat}",
                   "parallelism": "single GPU", "launch": "hipGraph" if graph else "eager"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": edge_kernel_name(slices),
                     "kernel_ms": edge_ms,
                     "algorithmic_bytes_per_launch": alg_bytes},
        "breakdown_ms": {"project": proj_ms, "edge": edge_ms, "csr_build_once": csr_ms},
        "projection": {"bound": "mfma", "achieved": proj_tflops, "peak": MFMA_F32_PEAK_TFLOPS,
                       "unit": "TFLOP/s", "frac": proj_tflops / MFMA_F32_PEAK_TFLOPS,
                       "kernel": "k_project (fp32 MFMA 16x16x4)"},
    }
    if training is not None:
        result["training"] = training
    if not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(layer.state_dict(), x, ei, w.heads, w.concat,
                                              n_edges)
    print(json.dumps(result), flush=True)


if __name__ == "__main__":
    main()
