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
    def alloc_table(n, heads, f, device, packed=True):
        from .layer import alloc_table
        return alloc_table(n, heads, f, device, packed=packed)

    @staticmethod
    def project(x, pp, heads, f, table, s_dst):
        from .layer import project
        return project(x, pp, heads, f, table=table, s_dst=s_dst)

    @staticmethod
    def edge_aggregate(csr, table, s_dst, heads, f, concat, bias, negative_slope, out, pp=None):
        from .layer import edge_aggregate
        return edge_aggregate(csr, table, s_dst, heads, f, concat, bias, negative_slope, out=out,
                              pp=pp)


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
        # allgather: one packed buffer [Wh | s_src] per node row, so a single
        # collective moves both (zero-filled: padding rows are defined);
        # replicate: the default separate layout (no collective to feed)
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
            buf = self.table.buf
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
        return x_full[self.r0:self.r1].contiguous() if self.exchange == "allgather" else x_full


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
def bench_distributed(args, metric: str):
    from .layer import GraphAttentionLayer
    from .graph import get_csr
    from .synthetic import WORKLOADS, make_inputs

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    dist.init_process_group("nccl", device_id=dev)
    exchange = getattr(args, "exchange", "allgather")

    w = WORKLOADS[args.workload]
    x, ei = make_inputs(w, dev)  # same seeds on every rank -> the same graph
    n = x.size(0)
    torch.manual_seed(0)
    layer = GraphAttentionLayer(w.in_channels, w.out_channels, num_heads=w.heads,
                                concat=w.concat).to(dev).eval()
    csr = get_csr(ei, n)
    sh = ShardedGAT(layer, csr, world, rank, exchange=exchange)
    xl = sh.local_x(x)
    del ei

    with torch.no_grad():
        for _ in range(3):
            sh.forward(xl)
        torch.cuda.synchronize()
        # graph-capture the compute phases; the collective runs between them
        launch = "eager"
        g_proj = g_edge = None
        if not args.no_graph:
            try:
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
                launch = "hipGraph(project) + RCCL + hipGraph(edges)"
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

        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        dist.barrier()
        elapsed = time.perf_counter() - t0
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

        # edge kernel alone on this rank's rows (roofline)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        stream = torch.cuda.current_stream()
        ev0.record(stream)
        for _ in range(args.edge_iters):
            sh.phase_edges()
        ev1.record(stream)
        ev1.synchronize()
        edge_ms = ev0.elapsed_time(ev1) / args.edge_iters

    from bench import HBM_PEAK_GBS, edge_kernel_bytes, load_traffic  # noqa: E402
    ms = elapsed * 1e3 / args.steps
    alg = edge_kernel_bytes(sh.n_local, sh.local.num_edges, w.heads, w.out_channels, w.concat)
    ach = alg / (edge_ms * 1e-3) / 1e9
    if rank == 0:
        res = {
            "metric": metric, "value": csr.num_edges / (ms * 1e-3), "unit": "edges/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (seeded uniform graph of the PPI shape; reference-order random init)",
            "config": {"workload": f"{w.name}: N={n} E'={csr.num_edges} Fin={w.in_channels} "
                                   f"H={w.heads} F={w.out_channels} concat={w.concat}",
                       "parallelism": f"node-range partition x{world}, exchange={exchange}",
                       "launch": launch},
            "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": ach / HBM_PEAK_GBS, "traffic": load_traffic(args.workload),
                         "kernel": "gat_edge_aggregate (rank 0 rows)", "kernel_ms": edge_ms,
                         "algorithmic_bytes_per_launch": alg},
        }
        print(json.dumps(res), flush=True)
    dist.barrier()
    dist.destroy_process_group()
