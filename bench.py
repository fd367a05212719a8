#!/usr/bin/env python3
"""Benchmark: edges/sec through the 8-head GAT layer forward.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload ppi|...]

N = 1 (the default): a "step" is one GraphAttentionLayer forward (eval, fp32)
over the synthetic PPI-shape graph (BASELINE.json configs[1]: N=44,906,
E=1,226,368 + N loops, Fin=50, H=8, F=8, concat) with inputs resident in HBM:
the HIP projection + the fused edge kernel.  The CSR (built once per
edge_index and cached, as in the module) is outside the timed region and is
timed separately.  The line also carries, under "workloads", the same
measurement for the other single-GPU configs: Reddit scale (configs[4], the
north-star roofline target), its power-law degree-skew variant, ogbn-arxiv
scale (configs[3]) and the CIFAR10 superpixel batch (configs[2]).

N > 1 (torchrun, one process per GPU): the same PPI-shape workload as ONE
shared graph, node-partitioned over the GPUs, the exchange inside the step
(the RCCL all-gather of the node table, at its fastest chunk count; every rank
projecting all rows, "replicate", is reported beside it), with Reddit and arxiv scale under
"workloads" (atmlgraphattentionnetworks_amd/distributed.py).  The N = 1 line
carries the per-rank compute of that partitioned step at P = 2/4/8, emulated
on its one GPU ("multi_gpu_emulated").

Prints ONE JSON line (rank 0).  See DESIGN.md "Measurement".
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import platform
import shutil
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md: 8.0 TB/s)
L2_PEAK_GBS = 34500.0  # aggregate L2 bandwidth, 8 XCDs (MI355X_MICROARCH.md: ~34.5 TB/s)
# measured chip-wide rate of row gathers served by the XCD's L2 (MI355X_MICROARCH.md,
# "Indexed rows: gather into LDS": 16.8-18.8 TB/s); the edge kernel's practical ceiling
L2_GATHER_CEILING_GBS = 18800.0
MFMA_F32_PEAK_TFLOPS = 157.3  # dense fp32 matrix peak (v_mfma_f32_16x16x4_f32)
MFMA_BF16_PEAK_TFLOPS = 2500.0  # dense bf16 matrix peak (v_mfma_f32_16x16x32_bf16)
SPLIT_PRODUCTS = 6  # bf16 MFMA products per fp32 product in the split-bf16 projections
_PROCESS_WARMUP_MS = None  # the first graph build of the process (one-time costs)


def projection_kernel(fin: int, f: int = 8) -> dict:
    """The projection kernel the library picks for this Fin and head width F
    (gat_project.hip project_impl, default knobs) and the matrix dtype it issues."""
    if fin <= 64:
        return {"kernel": "k_project_wk", "mfma": "fp32 (v_mfma_f32_16x16x4_f32)",
                "split": False}
    if fin <= 128:
        name = "k_project_wres_d" if f in (4, 8, 16) else "k_project_wres"
    else:
        name = "k_project_x3"
    return {"kernel": name, "mfma": "bf16, operands split exactly into 3 bf16 terms, "
            "6 v_mfma_f32_16x16x32_bf16 per fp32 product", "split": True}


def projection_roofline(flops: float, nbytes: float, ms: float, fin: int, f: int = 8) -> dict:
    """fp32-equivalent TFLOP/s, the fraction of the matrix peak of the dtype the
    kernel issues, and the HBM fraction; ``bound`` = the larger of the two time
    bounds."""
    k = projection_kernel(fin, f)
    sec = ms * 1e-3
    if k["split"]:
        mfma_flops, peak = SPLIT_PRODUCTS * flops, MFMA_BF16_PEAK_TFLOPS
    else:
        mfma_flops, peak = flops, MFMA_F32_PEAK_TFLOPS
    t_mfma = mfma_flops / (peak * 1e12)
    t_hbm = nbytes / (HBM_PEAK_GBS * 1e9)
    return {"kernel": k["kernel"], "mfma_dtype": k["mfma"],
            "TFLOPs": flops / sec / 1e12,
            "mfma_issued_TFLOPs": mfma_flops / sec / 1e12, "mfma_peak_TFLOPs": peak,
            "mfma_frac": mfma_flops / sec / 1e12 / peak,
            "hbm_bytes": nbytes, "hbm_frac": nbytes / sec / 1e9 / HBM_PEAK_GBS,
            "bound": "mfma" if t_mfma >= t_hbm else "hbm",
            "bound_frac": max(t_mfma, t_hbm) / sec}
NUM_CUS = 256
METRIC = "edges/sec through 8-head GAT layer forward, PPI shape, at 1/2/4/8 MI355X"
NORTH_STAR_REDDIT_EDGES_PER_S = 16.4e9  # >= 60% of the §8d HBM ceiling


def _log(msg: str) -> None:
    """Progress on stderr (stdout carries only the JSON line)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


# ---------------------------------------------------------------------------
# byte / flop models
# ---------------------------------------------------------------------------
def edge_kernel_bytes(n_rows: int, n_edges: int, heads: int, f: int, concat: bool) -> int:
    """SURVEY.md §8d's per-edge model, no reuse of a gathered row: per edge
    4 (col) + 4*H*F (Wh_j) + 4*H (s_src_j); per target row 4 (rowptr) + 4*H
    (s_dst) + 4*C_out (output).  Every Wh gather counted as if it came from
    HBM, so it is the 'effective gather' traffic, not an HBM byte count."""
    c_out = heads * f if concat else f
    return n_edges * (4 + 4 * heads * f + 4 * heads) + n_rows * (4 + 4 * heads + 4 * c_out)


def edge_kernel_compulsory_bytes(n_rows: int, n_table: int, n_edges: int, heads: int, f: int,
                                 concat: bool) -> int:
    """Bytes any implementation must move to or from HBM per launch: the CSR
    (col 4/edge, rowptr 4/row, the row schedule 4/row), the Wh table once
    (4*H*F per source node; s_src is recomputed from it), s_dst (4*H per row)
    and the output (4*C_out per row).  achieved = this / kernel time cannot
    exceed the HBM peak unless the kernel beat HBM."""
    c_out = heads * f if concat else f
    return (4 * n_edges + 8 * n_rows + 4 * heads * f * n_table
            + n_rows * (4 * heads + 4 * c_out))


def l2_request_bytes(n_edges: int, heads: int, f: int) -> int:
    """Bytes the edge kernel requests from L2 per launch (L1 hits aside): every
    edge gathers its source's whole Wh row (4*H*F, the score is recomputed
    from it) and its column index (4)."""
    return n_edges * (4 + 4 * heads * f)


def projection_bytes(n: int, fin: int, hf: int, heads: int) -> int:
    """HBM bytes of the projection: read x once, W once; write Wh and s_dst."""
    return 4 * (n * fin + fin * hf + n * hf + n * heads)


# ---------------------------------------------------------------------------
# host CPU facts (the CPU baseline's context)
# ---------------------------------------------------------------------------
def host_cpu_info() -> dict:
    info = {"os_cpu_count": os.cpu_count()}
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        info["affinity_cpus"] = None
    quota = None
    try:  # cgroup v2 CPU quota (the share a gpurun box gives one GPU)
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    info["cgroup_cpu_quota"] = quota
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        kv = {}
        for line in out.splitlines():
            if ":" in line:
                k, v = line.split(":", 1)
                kv[k.strip()] = v.strip()
        info["model"] = kv.get("Model name")
        info["sockets"] = int(kv["Socket(s)"]) if "Socket(s)" in kv else None
        info["cores_per_socket"] = int(kv["Core(s) per socket"]) if "Core(s) per socket" in kv \
            else None
        info["threads_per_core"] = int(kv["Thread(s) per core"]) if "Thread(s) per core" in kv \
            else None
        if info["sockets"] and info["cores_per_socket"]:
            info["physical_cores"] = info["sockets"] * info["cores_per_socket"]
    except (OSError, subprocess.SubprocessError, ValueError):
        pass
    if not info.get("model"):
        info["model"] = platform.processor() or "unknown"
    return info


def cpu_threads(info: dict) -> int:
    """Threads for the CPU baseline: os.cpu_count() (BASELINE.md's plan),
    limited to the CPUs this process may actually run on (affinity and the
    cgroup quota: a GPU box's share is far below its machine's count)."""
    n = info.get("os_cpu_count") or 1
    if info.get("affinity_cpus"):
        n = min(n, info["affinity_cpus"])
    if info.get("cgroup_cpu_quota"):
        n = min(n, max(1, int(info["cgroup_cpu_quota"])))
    return max(1, n)


def cpu_baseline(state, x, ei, heads, concat, n_edges, threads, budget_s=4.0,
                 sample=None) -> dict:
    """The oracle (pure-PyTorch restatement of GAT.py:37-67 in the reference's
    op order) on the host cores: one warm-up, then the median of >= 5 timed
    forwards, continuing up to ~budget_s."""
    from oracle import gat_layer_forward_from_state

    torch.set_num_threads(threads)
    xc, eic = x.cpu(), ei.cpu()
    st = {k: v.cpu() for k, v in state.items()}
    gat_layer_forward_from_state(st, xc, eic, heads, concat)  # warm-up
    times = []
    t_start = time.perf_counter()
    while len(times) < 5 or (len(times) < 40 and time.perf_counter() - t_start < budget_s):
        t0 = time.perf_counter()
        gat_layer_forward_from_state(st, xc, eic, heads, concat)
        times.append(time.perf_counter() - t0)
    med = statistics.median(times)
    return {"value": n_edges / med, "unit": "edges/s", "cores": threads, "kind": "port",
            "ms_per_forward": med * 1e3,
            "sample": (sample or "full workload") + (
                f"; {len(times)} timed forwards after 1 warm-up, median {med * 1e3:.1f} ms; "
                f"oracle/gat_oracle.py (torch CPU, {threads} threads)")}


# ---------------------------------------------------------------------------
# GPU measurement of one single-GPU workload
# ---------------------------------------------------------------------------
def _events_ms(fn, iters: int, stream, rounds: int = 1) -> float:
    """Mean time of fn over iters, HIP events recorded on `stream` (the stream
    the library launches on: torch's current stream); with rounds > 1 the
    median of that many such means (one slow round — a clock ramp, another
    process on the host — does not set the roofline's kernel time)."""
    means = []
    for _ in range(rounds):
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(stream)
        for _ in range(iters):
            fn()
        ev1.record(stream)
        ev1.synchronize()
        means.append(ev0.elapsed_time(ev1) / iters)
    return statistics.median(means)


def measure_workload(name: str, dev, steps: int, warmup: int, edge_iters: int,
                     graph: bool = False) -> dict:
    """One workload on one GPU: the layer forward's edges/s (eager steps, host
    clock around K synchronized steps), plus each phase alone with HIP events
    (projection; edge kernel(s)) on the exact plan the layer runs."""
    from atmlgraphattentionnetworks_amd import GraphAttentionLayer, _lib
    from atmlgraphattentionnetworks_amd.graph import get_csr
    from atmlgraphattentionnetworks_amd.layer import ForwardPlan
    from atmlgraphattentionnetworks_amd.synthetic import WORKLOADS, make_inputs

    w = WORKLOADS[name]
    _log(f"{name}: inputs")
    x, ei = make_inputs(w, dev)
    n = x.size(0)
    torch.manual_seed(0)
    layer = GraphAttentionLayer(w.in_channels, w.out_channels, num_heads=w.heads,
                                concat=w.concat).to(dev).eval()
    torch.cuda.synchronize()
    # the process's first graph build also pays one-time costs: the load of the
    # library's GPU code objects (the first launch from each of libgat_amd.so's
    # modules) and torch's first-use allocations.  A 64-node graph takes them
    # (reported as csr_process_warmup_ms), so csr_build_once is this graph's
    # first build in a warmed process
    from atmlgraphattentionnetworks_amd.graph import build_csr
    global _PROCESS_WARMUP_MS
    if _PROCESS_WARMUP_MS is None:
        t0 = time.perf_counter()
        build_csr(torch.randint(0, 64, (2, 256), device=dev), 64)
        torch.cuda.synchronize()
        _PROCESS_WARMUP_MS = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    csr = get_csr(ei, n)
    torch.cuda.synchronize()
    csr_ms = (time.perf_counter() - t0) * 1e3
    # the same build again (every buffer allocated before: the build's own time)
    t0 = time.perf_counter()
    build_csr(ei, n)
    torch.cuda.synchronize()
    csr_warm_ms = (time.perf_counter() - t0) * 1e3
    e_prime = csr.num_edges
    lib = _lib.load()
    stream = torch.cuda.current_stream()
    with torch.no_grad():
        def step():
            return layer(x, ei)
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        run, launch = step, "eager"
        if graph:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                step()
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                step()
            run, launch = g.replay, "hipGraph"
        for _ in range(warmup):
            run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            run()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / steps
        # the same step replayed from a captured graph (the one-GPU value that
        # graph-replayed per-rank compute is compared with: like for like)
        ms_graph = ms if graph else _graph_step_ms(step, warmup, steps)

        # the two phases alone, on the plan the layer's forward builds
        pp = layer.packed()
        bias = layer.bias.detach()
        plan = ForwardPlan(x, csr, w.heads, w.out_channels, w.concat, layer.negative_slope)
        out = torch.empty(n, w.heads * w.out_channels if w.concat else w.out_channels,
                          device=dev)
        plan.project(lib, x, pp)
        for _ in range(3):
            plan.edge(lib, csr, pp, bias, out)
        edge_ms = _events_ms(lambda: plan.edge(lib, csr, pp, bias, out), edge_iters, stream,
                             rounds=5)
        # projection alone: a short kernel, so launches captured in a graph
        gp = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gp):
            for _ in range(edge_iters):
                plan.project(lib, x, pp)
        gp.replay()
        proj_ms = _events_ms(gp.replay, 1, stream, rounds=5) / edge_iters
        # the two phases IN the step sequence: the layer's ping-pong workspaces
        # alternating, events between the launches (the isolated timings above
        # run each phase back to back on its own, so their sum need not equal
        # the step)
        seq = ForwardPlan(x, csr, w.heads, w.out_channels, w.concat, layer.negative_slope,
                          pingpong=True)
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(edge_iters)]
        for i in range(edge_iters + 3):
            seq.cur ^= 1
            seq.p_wh, seq.p_ss, seq.p_sd = seq.bufs[seq.cur]
            e = evs[i - 3] if i >= 3 else None
            if e:
                e[0].record(stream)
            seq.project(lib, x, pp)
            if e:
                e[1].record(stream)
            seq.edge(lib, csr, pp, bias, out)
            if e:
                e[2].record(stream)
        torch.cuda.synchronize()
        in_step = {"project": statistics.median(a.elapsed_time(b) for a, b, _ in evs),
                   "edge": statistics.median(b.elapsed_time(c) for _, b, c in evs),
                   "what": "median per step of events between the two launches in the layer's "
                           "own sequence (ping-pong workspaces)"}
        del seq
        fused = fused_small_fin(w.in_channels, plan)
        if fused:
            # Fin <= 4: the layer's forward is ONE kernel (gat_layer_forward fuses
            # the projection into the edge kernel); time exactly that launch
            for _ in range(3):
                plan.run(lib, x, pp, bias, out, csr)
            edge_ms = _events_ms(lambda: plan.run(lib, x, pp, bias, out, csr), edge_iters,
                                 stream, rounds=5)
    hf = w.heads * w.out_channels
    comp = edge_kernel_compulsory_bytes(n, n, e_prime, w.heads, w.out_channels, w.concat)
    alg = edge_kernel_bytes(n, e_prime, w.heads, w.out_channels, w.concat)
    l2b = l2_request_bytes(e_prime, w.heads, w.out_channels)
    es = edge_ms * 1e-3
    flops = 2.0 * n * w.in_channels * hf
    res = {
        "workload": name, "N": n, "E_prime": e_prime, "Fin": w.in_channels, "H": w.heads,
        "F": w.out_channels, "concat": w.concat,
        "value": e_prime / (ms * 1e-3), "unit": "edges/s", "ms_per_step": ms, "launch": launch,
        "ms_per_step_graph": ms_graph,
        "csr_build_once_ms": csr_ms, "csr_build_warm_ms": csr_warm_ms,
        "csr_process_warmup_ms": _PROCESS_WARMUP_MS,
        "phases_in_step_ms": None if fused else in_step,
        "edge_kernel": {
            "kernel": ("k_edge_grp<..., XF> with the projection fused (gat_layer_forward, "
                       "Fin <= 4; x rows gathered, not Wh rows)") if fused else plan.kernel_name(),
            "ms": edge_ms,
            "edges_per_s": e_prime / es,
            "compulsory_bytes": comp, "compulsory_GBps": comp / es / 1e9,
            "hbm_frac": comp / es / 1e9 / HBM_PEAK_GBS,
            "l2_request_bytes": l2b, "l2_GBps": l2b / es / 1e9,
            "l2_frac": l2b / es / 1e9 / L2_PEAK_GBS,
            "effective_gather_GBps": alg / es / 1e9,
            "algorithmic_8d_bytes": alg,
            "hub_rows_split": 0 if csr.hubs is None else csr.hubs.n_hub,
        },
        "projection": ({"ms": 0.0, "kernel": "fused into the edge kernel (Fin <= 4)",
                        "two_kernel_projection_ms": proj_ms} if fused else
                       dict(ms=proj_ms, **projection_roofline(
                           flops, projection_bytes(n, w.in_channels, hf, w.heads), proj_ms,
                           w.in_channels, w.out_channels))),
        "_inputs": (x, ei, layer),
    }
    _log(f"{name}: {res['value'] / 1e9:.2f} G edges/s, edge {edge_ms * 1e3:.1f} us, "
         f"projection {proj_ms * 1e3:.1f} us")
    return res


def _graph_step_ms(step, warmup: int, steps: int, per_replay: int = 2):
    """ms per ``step`` replayed from a captured graph (None if capture fails).
    ``per_replay`` consecutive steps are captured into one graph: with the
    layer's two ping-pong workspaces a one-step graph would replay the same
    workspace every time (the projection writing the table the previous
    replay's edge kernel read), and the sharded graphs
    (distributed.capture_steps) hold two steps per replay as well."""
    try:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(per_replay):
                step()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(per_replay):
                step()
    except Exception:  # noqa: BLE001  (the eager number stands alone)
        return None
    reps = max(1, steps // per_replay)
    for _ in range(max(1, warmup // per_replay)):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / (reps * per_replay)


def fused_small_fin(fin: int, plan) -> bool:
    """Whether the layer's eval forward runs the fused small-Fin kernel: the
    cached plan enqueues gat_layer_forward (over the scheduled CSR, no hub
    split), and the library says that call fuses this shape
    (gat_layer_forward_fuses, include/gat_amd.h)."""
    from atmlgraphattentionnetworks_amd import _lib
    if plan.sched is None or plan.split:
        return False
    return _lib.load().gat_layer_forward_fuses(plan.n, fin, plan.heads, plan.f, int(plan.concat),
                                               plan.slope) == 1


def pmc_child(names) -> None:
    """Workload runner for the in-run rocprofv3 --pmc passes (child process):
    launches each workload's projection + edge kernel(s) a few times."""
    from atmlgraphattentionnetworks_amd import GraphAttentionLayer, _lib
    from atmlgraphattentionnetworks_amd.graph import get_csr
    from atmlgraphattentionnetworks_amd.layer import ForwardPlan
    from atmlgraphattentionnetworks_amd.synthetic import WORKLOADS, make_inputs
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    for name in names:
        w = WORKLOADS[name]
        x, ei = make_inputs(w, dev)
        torch.manual_seed(0)
        layer = GraphAttentionLayer(w.in_channels, w.out_channels, num_heads=w.heads,
                                    concat=w.concat).to(dev).eval()
        csr = get_csr(ei, x.size(0))
        del ei
        with torch.no_grad():
            pp = layer.packed()
            bias = layer.bias.detach()
            plan = ForwardPlan(x, csr, w.heads, w.out_channels, w.concat, layer.negative_slope)
            out = torch.empty(x.size(0), w.heads * w.out_channels, device=dev)
            fused = fused_small_fin(w.in_channels, plan)
            for _ in range(4):
                if fused:  # one kernel: the layer's own launch
                    plan.run(lib, x, pp, bias, out, csr)
                else:
                    plan.project(lib, x, pp)
                    plan.edge(lib, csr, pp, bias, out)
            torch.cuda.synchronize()
        # a marker between workloads (the parent splits the dispatch list here)
        torch.zeros(1, device=dev).add_(1)
        torch.cuda.synchronize()
        del x, csr, layer, plan, out
        torch.cuda.empty_cache()
        print(f"pmc child: {name} done", flush=True)


PMC_PASSES = [
    # exact L2 -> fabric read bytes (per-size request counters; MI355X_MICROARCH.md
    # §HBM: calibrated 1.00 on a streaming copy, profiles/pmc_ppi.json)
    ["TCC_EA0_RDREQ_128B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_32B_sum"],
    # write bytes (exact for 16-B stores), L2 hit rate, MFMA busy (projection)
    ["WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum", "SQ_VALU_MFMA_BUSY_CYCLES",
     "GRBM_GUI_ACTIVE"],
]


def _parse_pmc_pass(d: str, names, res: dict) -> None:
    """Per-dispatch counters of one pass -> res[workload][kernel class][counter]
    lists.  The child separates workloads with a marker (a fill + add of one
    element) after each workload's launches."""
    rows = []
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows.extend(csv.DictReader(open(path)))
    per = {}  # dispatch -> (name, {counter: value})
    for r_ in rows:
        key = int(r_["Dispatch_Id"])
        nm, c = per.setdefault(key, (r_["Kernel_Name"], {}))
        c[r_["Counter_Name"]] = c.get(r_["Counter_Name"], 0.0) + float(r_["Counter_Value"])
    # split the dispatch list into workloads at the marker kernels
    wl = 0
    seen_edge = False  # this pass has seen the current workload's edge kernel
    for key in sorted(per):
        nm, c = per[key]
        if "k_edge" in nm or "k_project" in nm:
            if wl >= len(names):
                break
            kind = ("merge" if "k_edge_merge" in nm else
                    "edge" if "k_edge" in nm else "project")
            seen_edge = seen_edge or kind == "edge"
            slot = res.setdefault(names[wl], {}).setdefault(kind, {})
            for ctr, v in c.items():
                slot.setdefault(ctr, []).append(v)
        elif seen_edge and ("fill" in nm.lower() or "elementwise" in nm.lower()):
            # torch.zeros(1).add_(1): the marker ends a workload once its
            # kernels were seen
            wl += 1
            seen_edge = False


def pmc_traffic(names, out_dir: str, timeout_s: int = 150) -> dict:
    """Run the PMC passes over a child process and return, per workload and
    kernel class, the median per-dispatch counters.  Failures return
    {"error": ...} and never cost the bench line."""
    rocprof = shutil.which("rocprofv3")
    if rocprof is None:
        return {"error": "rocprofv3 not found"}
    res = {}
    os.makedirs(out_dir, exist_ok=True)
    env = dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp"))
    for i, ctrs in enumerate(PMC_PASSES):
        d = os.path.join(out_dir, f"pass{i}")
        shutil.rmtree(d, ignore_errors=True)
        cmd = ["timeout", "-s", "KILL", str(timeout_s), rocprof, "--pmc", *ctrs,
               "--output-format", "csv", "-d", d, "-o", "run", "--",
               sys.executable, os.path.abspath(__file__), "--pmc-child", ",".join(names)]
        _log(f"pmc pass {i}: {' '.join(ctrs)}")
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, env=env,
                               timeout=timeout_s + 30)
        except subprocess.SubprocessError as exc:
            return {"error": f"pass {i}: {type(exc).__name__}"}
        if r.returncode != 0:
            return {"error": f"pass {i} rc={r.returncode}: {(r.stderr or '')[-300:]}"}
        _parse_pmc_pass(d, names, res)
    out = {}
    for name, kinds in res.items():
        o = {}
        for kind, ctrs in kinds.items():
            med = {k: statistics.median(v) for k, v in ctrs.items()}
            o[kind] = med
        e = o.get("edge", {})
        rd = None
        if "TCC_EA0_RDREQ_128B_sum" in e:
            rd = (128 * e["TCC_EA0_RDREQ_128B_sum"] + 64 * e.get("TCC_EA0_RDREQ_64B_sum", 0)
                  + 32 * e.get("TCC_EA0_RDREQ_32B_sum", 0))
        wr = e.get("WRITE_SIZE", None)
        o["edge_fabric_read_bytes"] = rd
        o["edge_fabric_write_bytes"] = None if wr is None else wr * 1024.0
        o["edge_fabric_bytes"] = None if rd is None or wr is None else rd + wr * 1024.0
        hit, miss = e.get("TCC_HIT_sum"), e.get("TCC_MISS_sum")
        o["edge_l2_hit_rate"] = hit / (hit + miss) if hit is not None and miss else None
        p = o.get("project", {})
        if p.get("SQ_VALU_MFMA_BUSY_CYCLES") and p.get("GRBM_GUI_ACTIVE"):
            # MFMA busy cycles summed over SIMDs / (4 SIMDs x CUs x kernel cycles);
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md)
            o["project_mfma_busy_frac"] = p["SQ_VALU_MFMA_BUSY_CYCLES"] / (
                4 * NUM_CUS * p["GRBM_GUI_ACTIVE"] / 8.0)
        out[name] = o
    return out


def _roofline(meas: dict, traffic: dict) -> dict:
    ek = meas["edge_kernel"]
    es = ek["ms"] * 1e-3
    fab = traffic.get("edge_fabric_bytes") if traffic else None
    alg8d = ek["algorithmic_8d_bytes"]
    r = {"bound": "hbm", "achieved": ek["compulsory_GBps"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": ek["hbm_frac"], "traffic": fab,
         # SURVEY.md §8(d)'s no-reuse model beside it: every edge gathers its
         # source's Wh row as if from HBM; > 1 means the rows are re-read from
         # L2 / the Infinity Cache, so it is not an HBM fraction
         "achieved_8d": alg8d / es / 1e9, "frac_8d": alg8d / es / 1e9 / HBM_PEAK_GBS,
         "algorithmic_8d_bytes_per_launch": alg8d,
         "kernel": ek["kernel"], "kernel_ms": ek["ms"],
         "algorithmic_bytes_per_launch": ek["compulsory_bytes"],
         "algorithmic_model": "compulsory: col 4/edge + rowptr and row schedule 8/row + Wh "
                              "table once 4*H*F/node + s_dst 4*H/row + output 4*C_out/row",
         "fabric": None if fab is None else {
             "bytes_per_launch": fab, "GBps": fab / es / 1e9,
             "frac_of_hbm_peak": fab / es / 1e9 / HBM_PEAK_GBS,
             "x_compulsory": fab / ek["compulsory_bytes"],
             "l2_hit_rate": traffic.get("edge_l2_hit_rate"),
             "source": "in-run rocprofv3 --pmc TCC_EA0_RDREQ_{128B,64B,32B}_sum + WRITE_SIZE "
                       "(L2->fabric bytes; Infinity-Cache hits included, so an upper bound "
                       "on HBM bytes)"},
         "l2": {"request_bytes_per_launch": ek["l2_request_bytes"], "GBps": ek["l2_GBps"],
                "peak": L2_PEAK_GBS, "frac": ek["l2_frac"],
                "gather_ceiling_GBps": L2_GATHER_CEILING_GBS,
                "frac_of_gather_ceiling": ek["l2_GBps"] / L2_GATHER_CEILING_GBS,
                "what": "the kernel's L2 request rate (both 128-B plane rows, or the 256-B "
                        "row, per edge) against the L2 spec and against the measured rate of "
                        "L2-served row gathers, the practical ceiling of a gather kernel whose "
                        "table stays on-die"},
         "effective_gather_GBps": ek["effective_gather_GBps"]}
    return r


def _workload_summary(meas: dict, traffic: dict) -> dict:
    d = {k: v for k, v in meas.items() if not k.startswith("_")}
    d["roofline"] = _roofline(meas, traffic)
    if traffic and traffic.get("project_mfma_busy_frac") is not None:
        d["projection"]["mfma_busy_frac_pmc"] = traffic["project_mfma_busy_frac"]
    return d


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
    # gradients cleared as the reference's loops do (optimizer.zero_grad(),
    # run_inductive.py:76); Module.zero_grad walks the module tree instead
    opt = torch.optim.Adam([xg, *layer.parameters()], lr=1e-3)

    def one():
        opt.zero_grad(set_to_none=True)
        layer(xg, ei).backward(gout)

    for _ in range(5):
        one()
    stream = torch.cuda.current_stream()
    torch.cuda.synchronize()
    step_ms = _events_ms(one, steps, stream)
    with torch.no_grad():
        for _ in range(3):
            layer(x, ei)
        fwd_ms = _events_ms(lambda: layer(x, ei), steps, stream)
    graph_ms = None
    try:  # the same step captured in a HIP graph (device-seeded dropout)
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
        graph_ms = _events_ms(g.replay, steps, stream)
    except Exception:  # noqa: BLE001  (the eager number above stands alone)
        graph_ms = None
    layer.eval()
    return {"what": "layer forward (training mode, attention dropout 0.6) + HIP backward to x "
                    "and all parameters",
            "train_step_ms": step_ms, "forward_train_ms": fwd_ms,
            "backward_ms": step_ms - fwd_ms, "train_edges_per_s": n_edges / (step_ms * 1e-3),
            "train_step_graph_ms": graph_ms,
            "train_edges_per_s_graph": None if not graph_ms else n_edges / (graph_ms * 1e-3)}


def reddit_cpu_sample(meas: dict, threads: int, rows: int = 1024) -> dict:
    """CPU baseline at Reddit scale (uniform or power-law) on a bounded
    sample: the oracle over the complete in-edge sets of `rows` random target
    rows (the full forward materialises ~90 GB of edge tensors on the host).
    The oracle still projects all N nodes and adds all N self-loops."""
    x, ei, layer = meas["_inputs"]
    g = torch.Generator(device="cpu")
    g.manual_seed(7)
    pick = torch.randperm(x.size(0), generator=g)[:rows].to(ei.device)
    sub = ei[:, torch.isin(ei[1], pick)]
    n_edges = sub.size(1) + x.size(0)
    return cpu_baseline(layer.state_dict(), x, sub, layer.num_heads, layer.concat, n_edges,
                        threads, budget_s=3.0,
                        sample=f"{rows} random target rows with their {sub.size(1)} in-edges, "
                               f"+ N self-loops = {n_edges} edges, projection over all N nodes")


def emulated_ranks(meas: dict, ranks, exchanges=("allgather",)) -> dict:
    """SURVEY.md §8e's compute terms, measured: the per-rank projection and
    edge passes of the node-partitioned step at P ranks, each rank's work run
    alone on this GPU (distributed.emulate_rank_times), plus the bytes each
    rank would receive in the all-gather.  ``compute_only_speedup_bound`` =
    the one-GPU step / the slowest rank's compute: what P GPUs could reach if
    the collective were free (it is not; the N > 1 lines measure it).  Like
    for like: the graph-replayed one-GPU step over the graph-replayed per-rank
    compute, and (``_eager``) the eager step over the eager compute."""
    from atmlgraphattentionnetworks_amd.distributed import emulate_rank_times
    from atmlgraphattentionnetworks_amd.graph import get_csr
    x, ei, layer = meas["_inputs"]
    csr = get_csr(ei, x.size(0))
    out = {}
    with torch.no_grad():
        for exch in exchanges:
            for p in ranks:
                _log(f"{meas['workload']}: emulated P={p} ({exch})")
                # "allgather_k1": one unsplit edge pass (the compute floor, no overlap)
                kind, chunks = ("allgather", 1) if exch == "allgather_k1" else (exch, None)
                r = emulate_rank_times(layer, csr, x, p, exchange=kind, chunks=chunks)
                g1 = meas.get("ms_per_step_graph")
                r["one_gpu_step_ms_graph"] = g1
                r["compute_only_speedup_bound"] = None if not g1 else g1 / r["max_compute_ms"]
                r["compute_only_speedup_bound_eager"] = \
                    meas["ms_per_step"] / r["max_compute_ms_eager"]
                r["per_rank"] = [{k: (round(v, 5) if isinstance(v, float) else v)
                                  for k, v in d.items()} for d in r["per_rank"]]
                out[f"{exch}_P{p}"] = r
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 100 timed steps: the first step's host enqueue and the closing synchronize
    # (~25-30 us together) are paid once per timed region; over 20 steps they
    # added ~1.5 us to every 36-us PPI step, over 100 they add ~0.3 us
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="ppi")
    ap.add_argument("--graph", action="store_true",
                    help="replay each step as a captured HIP graph (default: eager launches, "
                         "which measured faster: the host enqueue of a step is shorter than its "
                         "GPU time, and graph replays add a ~9 us gap each)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--edge-iters", type=int, default=20)
    ap.add_argument("--workloads", default="reddit,reddit_powerlaw,arxiv,cifar,cifar_h8",
                    help="extra single-GPU workloads reported under 'workloads' ('' for none)")
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the in-run rocprofv3 --pmc passes (traffic, L2 hit, MFMA busy)")
    ap.add_argument("--no-train", action="store_true",
                    help="skip the training-step (forward with dropout + backward) measurement")
    ap.add_argument("--dist", action="store_true",
                    help="take the torch.distributed path even at WORLD_SIZE=1 (testing)")
    ap.add_argument("--dist-workloads", default="ppi,reddit,arxiv",
                    help="multi-GPU: shared-graph workloads, the first is the headline")
    ap.add_argument("--emulate-ranks", default="2,4,8",
                    help="N=1: per-rank compute of the partitioned step at these rank counts, "
                         "emulated on the one GPU ('' for none)")
    ap.add_argument("--no-weak", action="store_true",
                    help="multi-GPU: skip the data-parallel PPI-block secondary run")
    ap.add_argument("--detail-out", default=os.path.join(ROOT, "gpurun_out", "bench_detail.json"),
                    help="where the full-detail JSON goes (stdout carries the compact line)")
    ap.add_argument("--pmc-child", default=None, help=argparse.SUPPRESS)
    args = ap.parse_args()

    if args.pmc_child is not None:
        return pmc_child([s for s in args.pmc_child.split(",") if s])

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if world > 1 or args.gpus > 1 or args.dist:
        from atmlgraphattentionnetworks_amd.distributed import bench_distributed
        return bench_distributed(args, METRIC)

    from atmlgraphattentionnetworks_amd.synthetic import WORKLOADS

    dev = torch.device("cuda", 0)
    head = measure_workload(args.workload, dev, args.steps, args.warmup, args.edge_iters,
                            args.graph)
    w = WORKLOADS[args.workload]
    emu_ranks = [int(v) for v in args.emulate_ranks.split(",") if v]
    emulated = {}
    if emu_ranks:
        emulated[args.workload] = emulated_ranks(head, emu_ranks, ("allgather", "replicate"))
    x, ei, layer = head["_inputs"]
    training = None if args.no_train else train_step(layer, x, ei, head["E_prime"], args.steps)
    if training is not None:
        training["x_eval_forward"] = training["train_step_ms"] / head["ms_per_step"]
    extra = [s for s in args.workloads.split(",") if s and s != args.workload]
    measured = {}
    info = host_cpu_info()
    threads = cpu_threads(info)
    cpu = {}
    if not args.no_cpu_baseline:
        _log(f"cpu baseline {args.workload} ({threads} threads)")
        cpu[args.workload] = cpu_baseline(layer.state_dict(), x, ei, w.heads, w.concat,
                                          head["E_prime"], threads)
    for nm in extra:
        m = measure_workload(nm, dev, args.steps, args.warmup, args.edge_iters, args.graph)
        if not args.no_cpu_baseline:
            _log(f"cpu baseline {nm}")
            xw, eiw, lw = m["_inputs"]
            if nm in ("reddit", "reddit_powerlaw"):
                cpu[nm] = reddit_cpu_sample(m, threads)
            else:
                cpu[nm] = cpu_baseline(lw.state_dict(), xw, eiw, lw.num_heads, lw.concat,
                                       m["E_prime"], threads)
        if emu_ranks and nm in ("arxiv", "reddit"):
            emulated[nm] = emulated_ranks(m, emu_ranks, ("allgather", "replicate")
                                          if nm == "arxiv" else ("allgather",))
            if nm == "reddit" and 8 in emu_ranks:
                # the same step with one unsplit edge pass (no all-gather overlap)
                emulated[nm].update(emulated_ranks(m, [8], ("allgather_k1",)))
        if nm == "reddit" and not args.no_train:
            # the training step against the eval forward
            xw, eiw, lw = m["_inputs"]
            tr = train_step(lw, xw, eiw, m["E_prime"], min(args.steps, 10))
            tr["x_eval_forward"] = tr["train_step_ms"] / m["ms_per_step"]
            m["training"] = tr
        m.pop("_inputs")
        measured[nm] = m
        torch.cuda.empty_cache()
    traffic = {}
    if not args.no_pmc:
        names = [args.workload] + extra
        traffic = pmc_traffic(names, os.path.join(ROOT, "gpurun_out", "bench_pmc"))
    head_sum = _workload_summary(head, traffic.get(args.workload))
    workloads = {nm: _workload_summary(m, traffic.get(nm)) for nm, m in measured.items()}
    if "reddit" in workloads:
        rv = workloads["reddit"]["value"]
        workloads["reddit"]["north_star"] = {
            "target_edges_per_s": NORTH_STAR_REDDIT_EDGES_PER_S, "value": rv,
            "met": rv >= NORTH_STAR_REDDIT_EDGES_PER_S,
            "what": "SURVEY.md §8d: Reddit scale at 1 GPU >= 60% of the §8d HBM ceiling "
                    "(27.3 G edges/s), i.e. >= 16.4 G edges/s through the layer forward"}
        if "reddit_powerlaw" in workloads:
            workloads["reddit_powerlaw"]["vs_uniform_reddit"] = \
                workloads["reddit_powerlaw"]["value"] / rv
    result = {
        "metric": METRIC,
        "value": head["value"],
        "unit": "edges/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": head["ms_per_step"],
        "higher_is_better": True,
        # the N > 1 lines partition this same graph (total work fixed as N grows)
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded uniform graph of the PPI shape; reference-order random init)",
        "config": {"workload": f"{w.name}: N={head['N']} E={w.num_edges} (+N self-loops = "
                               f"{head['E_prime']}) Fin={w.in_channels} H={w.heads} "
                               f"F={w.out_channels} concat={w.concat}",
                   "parallelism": "single GPU", "launch": head["launch"]},
        "roofline": head_sum["roofline"],
        "breakdown_ms": {"project": head["projection"]["ms"], "edge": head["edge_kernel"]["ms"],
                         "csr_build_once": head["csr_build_once_ms"],
                         "csr_build_warm": head["csr_build_warm_ms"],
                         "csr_process_warmup": head["csr_process_warmup_ms"],
                         "in_step": {k: v for k, v in (head.get("phases_in_step_ms") or {}).items()
                                     if k != "what"}},
        "projection": {"bound": "mfma", "kernel": head["projection"]["kernel"],
                       "mfma_dtype": head["projection"].get("mfma_dtype"),
                       "achieved": head["projection"].get("mfma_issued_TFLOPs"),
                       "peak": head["projection"].get("mfma_peak_TFLOPs"), "unit": "TFLOP/s",
                       "frac": head["projection"].get("mfma_frac"),
                       "mfma_busy_frac_pmc": head_sum["projection"].get("mfma_busy_frac_pmc"),
                       "hbm_frac": head["projection"].get("hbm_frac")},
        "workloads": workloads,
    }
    if emulated:
        result["multi_gpu_emulated"] = {
            "what": "per-rank compute of the node-partitioned step (SURVEY.md §8e) at P ranks, "
                    "each rank's projection and edge passes run alone on this one GPU; the "
                    "collective is not included (bytes received per rank given instead)",
            **emulated}
    if training is not None:
        result["training"] = training
    if cpu:
        base = cpu.get(args.workload)
        if base is not None:
            result["cpu_baseline"] = dict(base, host=info)
        result["cpu_baselines"] = {k: v for k, v in cpu.items() if k != args.workload}
    if traffic.get("error"):
        result["pmc_error"] = traffic["error"]
    from atmlgraphattentionnetworks_amd.benchline import compact_single, write_detail
    detail_path = write_detail(result, args.detail_out)
    print(json.dumps(compact_single(result, detail_path)), flush=True)


if __name__ == "__main__":
    main()
