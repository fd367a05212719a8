"""Node-range partitioned GAT layer forward across the GPUs of one node.

The reference runs on one device (``run_inductive.py:55``); there is no
distributed code to mirror.  This is the scaling axis SURVEY.md §8e defines:

* target rows are split into P contiguous ranges, edge-balanced by a prefix
  sum over ``rowptr`` (each rank gets ~E'/P in-edges, not N/P rows);
* each rank projects its own rows (``gat_project``) into its slot of a padded
  node table [P * M, ld] (M = the largest range), then ONE RCCL all-gather
  (``all_gather_into_tensor``, in place) fills every other slot over xGMI —
  Wh and s_src travel together in the packed table row;
* each rank runs the edge kernel over its own rows; col ids were remapped
  once, at setup, from global node ids to table rows (p * M + local);
* outputs stay sharded; ``gather_output`` concatenates them for checks.

``exchange="replicate"`` is the alternative SURVEY.md §8e lists: every rank
holds all of x and recomputes the full projection, so there is no
collective in the step at all.

The compute ops are pluggable (``ops``) so the partition / remap / all-gather
logic can be exercised on CPU with gloo (tests/test_distributed_gloo.py);
the default ops are the HIP kernels.
"""
from __future__ import annotations

import json
import os
import sys
import time
from dataclasses import dataclass
from typing import List, Optional

import torch
import torch.distributed as dist



def partition_rows(rowptr: torch.Tensor, parts: int) -> List[int]:
    """Edge-balanced contiguous row ranges: boundaries b_0=0 <= ... <= b_P=N
    with rowptr[b_k] ~= k * E' / P."""
    n = rowptr.numel() - 1
    total = int(rowptr[-1])
    targets = torch.tensor([round(k * total / parts) for k in range(1, parts)],
                           dtype=rowptr.dtype, device=rowptr.device)
    cuts = torch.searchsorted(rowptr, targets).clamp_(0, n).tolist() if parts > 1 else []
    bounds = [0] + [int(c) for c in cuts] + [n]
    for k in range(1, len(bounds)):  # monotone
        bounds[k] = max(bounds[k], bounds[k - 1])
    return bounds


@dataclass
class LocalCSR:
    rowptr: torch.Tensor  # int32 [n_local + 1], starts at 0
    col: torch.Tensor  # int32 table-row ids
    num_nodes: int  # n_local rows
    num_edges: int
    order: Optional[torch.Tensor] = None  # int32 [n_local], rows by descending in-degree


def degree_order(rowptr: torch.Tensor) -> torch.Tensor:
    """Rows by descending in-degree, stable (the same schedule gat_csr_build emits)."""
    deg = (rowptr[1:] - rowptr[:-1]).to(torch.int64)
    return torch.argsort(deg, descending=True, stable=True).to(torch.int32)


def remap_to_table(col: torch.Tensor, bounds: List[int], rows_per_part: int) -> torch.Tensor:
    """Global node id -> row of the padded, all-gathered table (p * M + local)."""
    b = torch.tensor(bounds, dtype=torch.int64, device=col.device)
    c = col.to(torch.int64)
    part = torch.searchsorted(b[1:], c, right=True)
    return (part * rows_per_part + (c - b[part])).to(torch.int32)


class HipOps:
    """The HIP kernels (default)."""

    @staticmethod
    def alloc_table(n, heads, f, device, packed=True, wh_only=False, slices=1):
        from .layer import alloc_table
        if slices > 1:
            return alloc_table(n, heads, f, device, slices=slices)
        return alloc_table(n, heads, f, device, packed=packed, wh_only=wh_only)

    @staticmethod
    def project(x, pp, heads, f, table, s_dst):
        from .layer import project
        return project(x, pp, heads, f, table=table, s_dst=s_dst)

    @staticmethod
    def edge_aggregate(csr, table, s_dst, heads, f, concat, bias, negative_slope, out, pp=None):
        from .layer import edge_aggregate
        return edge_aggregate(csr, table, s_dst, heads, f, concat, bias, negative_slope, out=out,
                              pp=pp)


def _default_score(layer) -> bool:
    """LeakyReLU score activation with slope in [0, 1] (the fused-score kernels)."""
    act = getattr(layer, "score_activation", None)
    if act is None:
        return True  # layers without the hook (test stand-ins) use the reference default
    code, param = act()
    return code == 0 and 0.0 <= param <= 1.0


class ShardedGAT:
    """One rank's share of a node-range partitioned GAT layer forward."""

    def __init__(self, layer, csr, world: int, rank: int, exchange: str = "allgather",
                 group=None, ops=None, packed=None):
        if exchange not in ("allgather", "replicate"):
            raise ValueError(exchange)
        self.layer, self.world, self.rank, self.group = layer, world, rank, group
        self.exchange = exchange
        self.ops = ops or HipOps
        self.heads, self.f = layer.num_heads, layer.output_channels
        self.concat = layer.concat
        self.pp = packed if packed is not None else layer.packed()
        self.bias = layer.bias.detach()
        dev = csr.rowptr.device
        self.bounds = partition_rows(csr.rowptr, world)
        self.r0, self.r1 = self.bounds[rank], self.bounds[rank + 1]
        self.n_local = self.r1 - self.r0
        self.rows_per_part = max(max(self.bounds[k + 1] - self.bounds[k] for k in range(world)), 1)
        rp = csr.rowptr
        e0, e1 = int(rp[self.r0]), int(rp[self.r1])
        col = csr.col[e0:e1]
        if exchange == "allgather":
            col = remap_to_table(col, self.bounds, self.rows_per_part)
            n_table = world * self.rows_per_part
        else:
            col = col.clone()
            n_table = csr.num_nodes
        lrp = (rp[self.r0:self.r1 + 1] - e0).to(torch.int32).contiguous()
        self.local = LocalCSR(lrp, col.contiguous(), self.n_local, e1 - e0, degree_order(lrp))
        # allgather: the table rows every rank needs travel in ONE collective
        # (zero-filled: padding rows are defined).  Where the edge kernel
        # recomputes s_src from the gathered Wh row (LeakyReLU, f/4 a power of
        # two) only Wh travels: 256-B, 128-B-aligned rows at H*F = 64 (the packed
        # [Wh | s_src] row is 288 B and every gather straddles an extra line).
        # Otherwise one packed buffer [Wh | s_src].  replicate: the default
        # separate layout (no collective to feed).
        # Wh-only tables can also be sliced into column planes (layer.wh_slices,
        # the single-GPU eval forward's layout): one all-gather per plane.
        hl = self.f // 4
        self.wh_only = (exchange == "allgather" and self.f % 4 == 0 and hl > 0 and
                        (hl & (hl - 1)) == 0 and _default_score(layer))
        self.slices = 1
        if self.wh_only:
            from .layer import wh_slices
            self.slices = wh_slices(self.heads, self.f, self.concat, 0.2,
                                    csr.num_edges // max(csr.num_nodes, 1))
        if self.wh_only and self.slices > 1:
            self.table = self.ops.alloc_table(n_table, self.heads, self.f, dev,
                                              slices=self.slices)
        elif self.wh_only:
            self.table = self.ops.alloc_table(n_table, self.heads, self.f, dev, wh_only=True)
        else:
            self.table = self.ops.alloc_table(n_table, self.heads, self.f, dev,
                                              packed=(exchange == "allgather"))
        self.s_dst_full = torch.empty(csr.num_nodes if exchange == "replicate" else self.n_local,
                                      self.heads, dtype=torch.float32, device=dev)
        width = self.heads * self.f if self.concat else self.f
        self.out = torch.empty(self.n_local, width, dtype=torch.float32, device=dev)

    # -- the three phases of a step (split so compute can be graph-captured) --
    def phase_project(self, x):
        if self.exchange == "allgather":
            m = self.rows_per_part
            slot = self.table.rows(self.rank * m, self.rank * m + self.n_local)
            self.ops.project(x, self.pp, self.heads, self.f, slot, self.s_dst_full)
        else:
            self.ops.project(x, self.pp, self.heads, self.f, self.table, self.s_dst_full)

    def phase_exchange(self):
        if self.exchange == "allgather" and self.world > 1:
            m = self.rows_per_part
            # one in-place all-gather per column plane (a single one for the
            # row-major table)
            planes = [self.table.buf[g] for g in range(self.slices)] if self.slices > 1 \
                else [self.table.buf]
            for buf in planes:
                dist.all_gather_into_tensor(buf, buf[self.rank * m:(self.rank + 1) * m],
                                            group=self.group)

    def phase_edges(self):
        s_dst = self.s_dst_full if self.exchange == "allgather" else \
            self.s_dst_full[self.r0:self.r1]
        return self.ops.edge_aggregate(self.local, self.table, s_dst, self.heads, self.f,
                                       self.concat, self.bias, 0.2, self.out, pp=self.pp)

    def forward(self, x):
        """x: this rank's rows [n_local, Fin] (allgather) or all rows (replicate)."""
        self.phase_project(x)
        self.phase_exchange()
        return self.phase_edges()

    def local_x(self, x_full):
        # a fresh copy: a row view of x can start off a 16-B boundary, which the
        # whole-K projection (the one that writes the sliced table) needs
        return x_full[self.r0:self.r1].clone() if self.exchange == "allgather" else x_full


def gather_output(local_out: torch.Tensor, bounds: List[int], group=None) -> torch.Tensor:
    """Concatenate the sharded outputs (for checks only; not part of a step)."""
    world = len(bounds) - 1
    m = max(bounds[k + 1] - bounds[k] for k in range(world))
    pad = torch.zeros(m, local_out.size(1), dtype=local_out.dtype, device=local_out.device)
    pad[:local_out.size(0)] = local_out
    allp = torch.empty(world * m, local_out.size(1), dtype=local_out.dtype,
                       device=local_out.device)
    dist.all_gather_into_tensor(allp, pad, group=group)
    return torch.cat([allp[k * m:k * m + bounds[k + 1] - bounds[k]] for k in range(world)])


# ---------------------------------------------------------------------------
# bench.py --gpus N (torchrun, one process per GPU, RCCL)
# ---------------------------------------------------------------------------
def _time_steps(step, warmup: int, steps: int, dev) -> float:
    """W untimed steps, then K steps bracketed by barrier + synchronize on both
    sides; returns the MAX over ranks of the K-step wall time (seconds).  Each
    rank's clock runs from just after the opening barrier to its own final
    synchronize, so a straggler shows up in the max while the closing
    barrier's latency is not billed as step time."""
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    dist.barrier()
    # the default group is gloo (bench_distributed): a host tensor
    t = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _strong_probe(w, layer, dev, world, rank, exchange, steps, warmup, use_graph, group=None):
    """ONE shared graph of the workload's shape, node-range partitioned across
    the ranks: per step, project own rows -> RCCL all-gather of
    the packed [Wh | s_src] table (exchange="allgather") or full projection on
    every rank (exchange="replicate") -> local edge kernel."""
    from .graph import get_csr
    from .synthetic import make_inputs

    x, ei = make_inputs(w, dev)  # same seeds on every rank -> the same graph
    csr = get_csr(ei, x.size(0))
    del ei
    sh = ShardedGAT(layer, csr, world, rank, exchange=exchange, group=group)
    xl = sh.local_x(x)
    launch = "eager"
    g_proj = g_edge = None
    for _ in range(3):
        sh.forward(xl)
    torch.cuda.synchronize()
    if use_graph:
        try:  # capture the compute phases; the collective runs between them
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                sh.phase_project(xl)
                sh.phase_edges()
            torch.cuda.current_stream().wait_stream(s)
            g_proj, g_edge = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(g_proj):
                sh.phase_project(xl)
            with torch.cuda.graph(g_edge):
                sh.phase_edges()
            launch = "hipGraph(project) + collective + hipGraph(edges)"
        except Exception as exc:  # capture unsupported -> eager
            g_proj = g_edge = None
            launch = f"eager (graph capture failed: {type(exc).__name__})"

    def step():
        if g_proj is not None:
            g_proj.replay()
            sh.phase_exchange()
            g_edge.replay()
        else:
            sh.forward(xl)

    t = _time_steps(step, warmup, steps, dev)
    ex_ms = None
    if exchange == "allgather" and world > 1:
        t_ex = _time_steps(sh.phase_exchange, 3, steps, dev)
        ex_ms = t_ex * 1e3 / steps
    ms = t * 1e3 / steps
    return {"exchange": exchange, "value": csr.num_edges / (ms * 1e-3), "unit": "edges/s",
            "ms_per_step": ms, "collective_ms": ex_ms, "rows_per_rank": sh.rows_per_part,
            "table_bytes": int(sh.table.wh.numel() * 4) if exchange == "allgather" else None,
            "launch": launch}


def bench_distributed(args, metric: str):
    """One process per GPU.  The reported line is WEAK scaling: every rank owns
    one PPI-shape block of a block-diagonal graph (the real PPI dataset is a set
    of disjoint graphs), so the node-range partition falls on block boundaries,
    the halo is empty and the step needs no collective; value = world x E'
    per block / max-over-ranks step time.  The same run also measures the
    STRONG-scaling north-star path on one shared graph (RCCL all-gather of the
    packed table, and the replicate alternative) and reports it under
    "strong_scaling"."""
    from .layer import GraphAttentionLayer
    from .synthetic import WORKLOADS, make_inputs
    from .graph import get_csr

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    if os.environ.get("GAT_BENCH_SHARE_GPU0"):  # testing on a one-GPU box: every rank on cuda:0
        local_rank = 0
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    # rank 0 prints exactly one JSON line on stdout; RCCL prints its banner and
    # warnings to stdout from C, so fd 1 points at stderr until the result is ready
    sys.stdout.flush()
    saved_stdout = os.dup(1)
    os.dup2(2, 1)
    # The weak-scaling step has no data-path collective, so the default group is
    # gloo (barriers and the max-over-ranks reduction on the host): no RCCL
    # proxy threads compete with the launch thread while it is timed.  The RCCL
    # group is created afterwards, for the strong-scaling probe's all-gather.
    # single node, rendezvous on 127.0.0.1: keep gloo on loopback rather than on
    # whatever interface the (possibly unresolvable) hostname maps to
    os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
    dist.init_process_group("gloo")

    w = WORKLOADS[args.workload]
    torch.manual_seed(0)
    layer = GraphAttentionLayer(w.in_channels, w.out_channels, num_heads=w.heads,
                                concat=w.concat).to(dev).eval()

    def layer_for(pw):
        if pw is w:
            return layer
        torch.manual_seed(0)
        return GraphAttentionLayer(pw.in_channels, pw.out_channels, num_heads=pw.heads,
                                   concat=pw.concat).to(dev).eval()
    # this rank's block: seeds offset by rank (rank 0's block is the 1-GPU graph)
    x, ei = make_inputs(w, dev, x_seed=1 + 1000 * rank, edge_seed=2 + 1000 * rank)
    csr = get_csr(ei, x.size(0))
    with torch.no_grad():
        for _ in range(3):
            layer(x, ei)
        torch.cuda.synchronize()
        step, launch = (lambda: layer(x, ei)), "eager"
        if args.graph:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                layer(x, ei)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                layer(x, ei)
            step, launch = g.replay, "hipGraph"
        t = _time_steps(step, args.warmup, args.steps, dev)
        ms = t * 1e3 / args.steps
        e_blk = torch.tensor([csr.num_edges], dtype=torch.float64)
        dist.all_reduce(e_blk)
        total_edges = float(e_blk.item())

        # edge kernel alone on this rank's block (roofline), in the layer's table
        # layout, HIP events on its stream
        from bench import time_edge_kernel
        edge_ms, slices = time_edge_kernel(layer, x, csr, args.edge_iters)
        n_block = x.size(0)
        del x, ei

        strong = []
        if not getattr(args, "no_strong_probe", False):
            # evidence only (the reported value is the weak-scaling line): a failure
            # here is recorded in the JSON instead of costing the line
            try:
                rccl = dist.new_group(backend="nccl")
            except Exception as exc:  # noqa: BLE001
                rccl = None
                strong.append({"error": f"RCCL group: {type(exc).__name__}: {exc}"[:300]})
            if rccl is not None:
                probes = [(w, "allgather"), (w, "replicate")]
                if (world > 1 or os.environ.get("GAT_BENCH_PROBE_REDDIT")) and w.name == "ppi":
                    # the shape the all-gather is designed for: edge work
                    # shrinks as 1/N while the exchanged table is 67 MB; its 1-GPU
                    # reference is `bench.py --workload reddit`
                    probes.append((WORKLOADS["reddit"], "allgather"))
                for pw, ex in probes:
                    try:
                        r = _strong_probe(pw, layer_for(pw), dev, world, rank, ex,
                                          max(args.steps // 2, 5), max(args.warmup // 2, 2),
                                          not args.no_graph, group=rccl)
                        r["workload"] = pw.name
                        strong.append(r)
                    except Exception as exc:  # noqa: BLE001
                        strong.append({"workload": pw.name, "exchange": ex,
                                       "error": f"{type(exc).__name__}: {exc}"[:300]})
                    torch.cuda.empty_cache()

    from bench import HBM_PEAK_GBS, edge_kernel_bytes, edge_kernel_name, load_traffic  # noqa: E402
    alg = edge_kernel_bytes(n_block, csr.num_edges, w.heads, w.out_channels, w.concat)
    ach = alg / (edge_ms * 1e-3) / 1e9
    res = None
    if rank == 0:
        res = {
            "metric": metric, "value": total_edges / (ms * 1e-3), "unit": "edges/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (seeded uniform PPI-shape blocks, one per GPU; reference-order "
                    "random init)",
            "config": {"workload": f"{w.name} x {world}: block-diagonal graph, {world} PPI-shape "
                                   f"blocks of N={n_block} E'={csr.num_edges} Fin={w.in_channels} "
                                   f"H={w.heads} F={w.out_channels} concat={w.concat}",
                       "parallelism": f"node-range partition x{world} on block boundaries "
                                      "(empty halo: no collective in the step)",
                       "launch": launch},
            "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": ach / HBM_PEAK_GBS, "traffic": load_traffic(args.workload),
                         "kernel": edge_kernel_name(slices) + " (rank 0 block)",
                         "kernel_ms": edge_ms,
                         "algorithmic_bytes_per_launch": alg},
            "strong_scaling": {"graph": "one graph of the named workload's shape shared by "
                                        f"{world} ranks, node-range partitioned",
                               "runs": strong},
        }
    dist.barrier()
    dist.destroy_process_group()
    sys.stdout.flush()
    os.dup2(saved_stdout, 1)
    os.close(saved_stdout)
    if res is not None:
        print(json.dumps(res), flush=True)
