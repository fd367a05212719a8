"""Node-range partitioned GAT layer forward across the GPUs of one node.

The reference runs on one device (``run_inductive.py:55``); there is no
distributed code to mirror.  This is the scaling axis SURVEY.md §8e defines:

* target rows are split into P contiguous ranges, edge-balanced by a prefix
  sum over ``rowptr`` (each rank gets ~E'/P in-edges, not N/P rows);
* each rank projects its own rows (``gat_project``) into its slots of ONE
  node table that every rank holds, and an RCCL all-gather over xGMI fills
  the other ranks' slots;
* each rank runs the edge kernel over its own target rows; source ids were
  remapped once, at setup, from global node ids to table rows;
* outputs stay sharded; ``gather_output`` concatenates them for checks.

Overlap.  The table is laid out in K CHUNKS, [K][P][S planes][B rows][W]:
chunk c holds rows [c*B, (c+1)*B) of every rank.  A step issues, per chunk,
the projection of the rank's rows of that chunk and then an asynchronous
in-place ``all_gather_into_tensor`` of the chunk (RCCL runs it on its own
stream); the edge work then runs as K passes, pass c over the in-edges whose
sources lie in chunk c (each row's sources are sorted by table row, so they
form one contiguous segment), carrying the online-softmax state (m, l, acc)
from pass to pass (``gat_edge_aggregate_seg``).  Pass c waits only for chunk
c, so the all-gather of chunks c+1.. proceeds under pass c.  K = 1 is the
plain project -> all-gather -> edge kernel step.

``exchange="replicate"`` is the alternative SURVEY.md §8e lists: every rank
holds all of x and recomputes the full projection, so there is no
collective in the step at all.

The compute ops are pluggable (``ops``) so the partition / remap / chunk /
segment logic runs on CPU under gloo (tests/test_distributed_gloo.py); the
default ops are the HIP kernels, and the one-GPU emulation (``emulate``)
runs them for P virtual ranks (tests/test_gpu_distributed.py).
"""
from __future__ import annotations

import json
import os
import statistics
import sys
import time
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from . import _lib


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


def degree_order(rowptr: torch.Tensor) -> torch.Tensor:
    """Rows by descending in-degree, stable (the schedule gat_csr_build emits)."""
    deg = (rowptr[1:] - rowptr[:-1]).to(torch.int64)
    return torch.argsort(deg, descending=True, stable=True).to(torch.int32)


@dataclass(frozen=True)
class TableLayout:
    """The node table every rank holds: [chunks][world][slices][block_rows][width]
    fp32.  ``kind``: "planes" (Wh as column planes, the eval forward's layout),
    "wh" (row-major Wh only: the edge kernel recomputes s_src from the row) or
    "packed" ([Wh | s_src] rows, for score activations the fused kernels do not
    take).  A node's table row is its plane-0 row index:
    (c * world + p) * slices * block_rows + i for the i-th row of rank p's
    chunk c; plane g of it lies g * block_rows rows further (the kernels'
    plane stride n_table = block_rows)."""
    kind: str
    world: int
    chunks: int
    block_rows: int
    slices: int
    width: int
    s_off: int = 0

    @property
    def block_floats(self) -> int:
        return self.slices * self.block_rows * self.width

    @property
    def numel(self) -> int:
        return self.chunks * self.world * self.block_floats

    @property
    def table_rows(self) -> int:
        return self.chunks * self.world * self.slices * self.block_rows

    def block_offset(self, c: int, p: int) -> int:
        return (c * self.world + p) * self.block_floats

    def chunk_range(self, c: int):
        per = self.world * self.block_floats
        return c * per, (c + 1) * per

    def row_of(self, part: torch.Tensor, local: torch.Tensor) -> torch.Tensor:
        c = torch.div(local, self.block_rows, rounding_mode="floor")
        i = local - c * self.block_rows
        return (c * self.world + part) * (self.slices * self.block_rows) + i

    def chunk_of_row(self, trow: torch.Tensor) -> torch.Tensor:
        return torch.div(trow, self.world * self.slices * self.block_rows, rounding_mode="floor")


@dataclass
class LocalCSR:
    rowptr: torch.Tensor  # int32 [n_local + 1], starts at 0
    col: torch.Tensor  # int32 table rows, ascending within each row
    num_nodes: int  # n_local rows
    num_edges: int
    order: Optional[torch.Tensor] = None  # int32 [n_local], rows by descending in-degree
    seg: Optional[torch.Tensor] = None  # int32 [chunks + 1, n_local]: pass c = [seg[c], seg[c+1])



def _score(layer):
    """(activation code, parameter) of the layer's score activation."""
    act = getattr(layer, "score_activation", None)
    if act is None:
        return _lib.GAT_ACT_LEAKY_RELU, 0.2  # test stand-ins: the reference default
    return act()


def fused_score_ok(heads: int, f: int, act: int, param: float) -> bool:
    """The fused-score kernels (Wh-only / planes tables, segmented passes):
    LeakyReLU with slope in [0, 1], f % 4 == 0 and f/4 a power of two."""
    hl = f // 4
    return (act == _lib.GAT_ACT_LEAKY_RELU and 0.0 <= param <= 1.0 and f % 4 == 0 and hl > 0
            and (hl & (hl - 1)) == 0)


EDGES_PER_CHUNK = 4_000_000  # per-rank edges per all-gather chunk / edge pass


def default_chunks(world: int, total_edges: int, fused: bool) -> int:
    """All-gather chunks (= edge passes) per step: one pass per ~4M edges per
    rank, at most 2 (each extra pass re-runs every row's prologue and carries
    its state through memory: Reddit at P = 8, edge passes 279 / 287 us at 2 / 3
    chunks, P = 4 555 us at 4; profiles/r04/emu_reddit_p8.json); 1 on a single
    rank or without the fused kernels.

    Every rank must pick the SAME count (it fixes the table layout and the
    collectives' sizes), so the argument is the graph's total edge count E',
    which all ranks see, never a rank's own share."""
    if world <= 1 or not fused:
        return 1
    return max(1, min(2, (total_edges // world) // EDGES_PER_CHUNK))


class HipOps:
    """The HIP kernels (default)."""

    @staticmethod
    def workspace(x_device, fin: int, heads: int, f: int):
        """The projection's optional workspace (gat_project_ex), or None."""
        from .layer import project_workspace
        return project_workspace(x_device, fin, heads, f)

    @staticmethod
    def project_rows(x, pp, heads, f, layout: TableLayout, table, offset, s_dst, s_scratch,
                     ws=None):
        """Project rows x into the table block at float offset ``offset``
        (gat_project_ex; ``ws`` its optional workspace)."""
        lib = _lib.load()
        n, fin = x.shape
        if n == 0:
            return
        stream = torch._C._cuda_getCurrentRawStream(x.device.index)
        wh = table.data_ptr() + 4 * offset
        args = (x.data_ptr(), n, fin, pp.w.data_ptr(), pp.b.data_ptr(), pp.a_src.data_ptr(),
                pp.c_src.data_ptr(), pp.a_dst.data_ptr(), pp.c_dst.data_ptr(), heads, f)
        wsa = (0, 0) if ws is None else (ws.data_ptr(), ws.numel())
        if layout.kind == "planes":
            rc = lib.gat_project_ex(*args, layout.slices, wh, layout.block_rows, 0, heads,
                                    s_dst.data_ptr(), 0, 0, *wsa, stream)
        elif layout.kind == "wh":
            rc = lib.gat_project_ex(*args, 1, wh, layout.width, s_scratch.data_ptr(), heads,
                                    s_dst.data_ptr(), 0, 0, *wsa, stream)
        else:
            rc = lib.gat_project_ex(*args, 1, wh, layout.width, wh + 4 * layout.s_off,
                                    layout.width, s_dst.data_ptr(), 0, 0, *wsa, stream)
        _lib.check(rc, "gat_project_ex (shard block)")

    @staticmethod
    def project_chunked(x, pp, heads, f, layout: TableLayout, table, rank: int, s_dst, ws=None):
        """All of a rank's rows in ONE launch (gat_project_ex with row chunks):
        row chunk c goes to the rank's block of table chunk c (planes only)."""
        lib = _lib.load()
        n, fin = x.shape
        if n == 0:
            return
        stream = torch._C._cuda_getCurrentRawStream(x.device.index)
        wsa = (0, 0) if ws is None else (ws.data_ptr(), ws.numel())
        rc = lib.gat_project_ex(
            x.data_ptr(), n, fin, pp.w.data_ptr(), pp.b.data_ptr(), pp.a_src.data_ptr(),
            pp.c_src.data_ptr(), pp.a_dst.data_ptr(), pp.c_dst.data_ptr(), heads, f,
            layout.slices, table.data_ptr() + 4 * layout.block_offset(0, rank),
            layout.block_rows, 0, heads, s_dst.data_ptr(), layout.block_rows,
            layout.world * layout.block_floats, *wsa, stream)
        _lib.check(rc, "gat_project_ex (shard, row chunks)")

    @staticmethod
    def edge_pass(local: LocalCSR, c: int, layout: TableLayout, table, s_dst, pp, bias, heads,
                  f, concat, act, param, out, st_acc, st_ml, flags):
        lib = _lib.load()
        n = local.num_nodes
        if n == 0:
            return out
        stream = torch._C._cuda_getCurrentRawStream(table.device.index)
        hint = local.num_edges // max(n, 1)
        order = 0 if local.order is None else local.order.data_ptr()
        if layout.kind == "packed":
            if flags:
                raise ValueError("the packed table runs one pass")
            rc = lib.gat_edge_aggregate_ex(
                local.rowptr.data_ptr(), local.col.data_ptr(), order, 0, n, table.data_ptr(),
                layout.width, table.data_ptr() + 4 * layout.s_off, layout.width, 0, 0,
                s_dst.data_ptr(), heads, f, int(concat), act, float(param), 0.0, 0, 0,
                bias.data_ptr(), out.data_ptr(), 0, 0, hint, stream)
            _lib.check(rc, "gat_edge_aggregate_ex (shard)")
            return out
        sb = local.seg[c].data_ptr()
        se = local.seg[c + 1].data_ptr()
        rc = lib.gat_edge_aggregate_seg(
            sb, se, 0, local.col.data_ptr(), order, 0, n, table.data_ptr(), layout.width,
            layout.block_rows, layout.slices, pp.a_src.data_ptr(), pp.c_src.data_ptr(),
            s_dst.data_ptr(), heads, f, int(concat), float(param),
            0 if st_acc is None else st_acc.data_ptr(), 0 if st_ml is None else st_ml.data_ptr(),
            flags, 0, bias.data_ptr(), out.data_ptr(), hint, stream)
        _lib.check(rc, "gat_edge_aggregate_seg (shard pass)")
        return out


class CollectiveExchange:
    """In-place all-gather of one table chunk over a process group (RCCL for
    CUDA tensors; gloo for the CPU tests), asynchronous: ``start`` returns the
    work handle and ``wait`` makes the current stream wait for it."""

    def __init__(self, group=None):
        self.group = group

    def start(self, chunk: torch.Tensor, part: torch.Tensor):
        return dist.all_gather_into_tensor(chunk, part, group=self.group, async_op=True)

    @staticmethod
    def wait(handle) -> None:
        if handle is not None:
            handle.wait()


class HostStagedExchange:
    """The same all-gather staged through host memory over a CPU (gloo)
    group: for rehearsing the multi-process path with several ranks on ONE
    GPU, where RCCL refuses duplicate devices.  Synchronous."""

    def __init__(self, group=None):
        self.group = group

    def start(self, chunk: torch.Tensor, part: torch.Tensor):
        host = torch.empty(chunk.numel(), dtype=chunk.dtype)
        dist.all_gather_into_tensor(host, part.cpu(), group=self.group)
        chunk.copy_(host)
        return None

    @staticmethod
    def wait(handle) -> None:
        return None


class NoExchange:
    """A single rank, or the one-process emulation (``emulate``) that copies
    the blocks itself."""

    @staticmethod
    def start(chunk, part):
        return None

    @staticmethod
    def wait(handle) -> None:
        return None


class ShardedGAT:
    """One rank's share of a node-range partitioned GAT layer forward."""

    def __init__(self, layer, csr, world: int, rank: int, exchange: str = "allgather",
                 group=None, ops=None, packed=None, chunks: Optional[int] = None,
                 exchanger=None, force_exchange: bool = False, pingpong: bool = True):
        """force_exchange: issue the chunk collectives even at world 1 (an
        in-place all-gather of a rank's own block), so the RCCL path can be
        exercised on a one-GPU box (tests, ``bench.py --dist``).
        pingpong: ``forward()`` alternates two node tables (the phase_* methods
        work on the current one)."""
        if exchange not in ("allgather", "replicate"):
            raise ValueError(exchange)
        self.layer, self.world, self.rank = layer, world, rank
        self.exchange = exchange
        self.force_exchange = bool(force_exchange)
        self.ops = ops or HipOps
        self.heads, self.f = layer.num_heads, layer.output_channels
        self.concat = layer.concat
        self.pp = packed if packed is not None else layer.packed()
        self.bias = layer.bias.detach()
        self.act, self.param = _score(layer)
        heads, f, hf = self.heads, self.f, self.heads * self.f
        dev = csr.rowptr.device
        self.bounds = partition_rows(csr.rowptr, world)
        self.r0, self.r1 = self.bounds[rank], self.bounds[rank + 1]
        self.n_local = self.r1 - self.r0
        self.rows_per_part = max(max(self.bounds[k + 1] - self.bounds[k] for k in range(world)), 1)
        rp = csr.rowptr
        e0, e1 = int(rp[self.r0]), int(rp[self.r1])
        self.fused = fused_score_ok(heads, f, self.act, self.param)
        # table layout: planes where the single-GPU eval forward would use them
        # (layer.wh_slices), else Wh-only rows, else packed [Wh | s_src]
        from .layer import wh_slices
        slices = 1
        if self.fused:
            slices = wh_slices(heads, f, self.concat, self.param,
                               csr.num_edges // max(csr.num_nodes, 1))
        kind = "planes" if slices > 1 else ("wh" if self.fused else "packed")
        if kind == "planes":
            width = hf // slices
            s_off = 0
        elif kind == "wh":
            width = (hf + 3) // 4 * 4
            s_off = 0
        else:
            width, s_off = _lib.table_layout(heads, f)
        if exchange == "allgather":
            k = chunks if chunks is not None else default_chunks(world, csr.num_edges, self.fused)
            if not self.fused:
                k = 1
            k = max(1, min(k, self.rows_per_part))
            # block rows: a multiple of 64 keeps every chunk's x rows 16-B
            # aligned and the projection's row tiles whole
            b = (self.rows_per_part + k - 1) // k
            b = (b + 63) // 64 * 64
            self.layout = TableLayout(kind, world, k, b, slices, width, s_off)
        else:
            b = (csr.num_nodes + 63) // 64 * 64
            self.layout = TableLayout(kind, 1, 1, b, slices, width, s_off)
        lay = self.layout
        self.chunks = lay.chunks
        self.slices = slices
        self.wh_only = kind != "packed"
        self.local = self._local_csr(csr, e0, e1, dev)
        # two tables, used by alternate forward() calls: the projection and the
        # all-gather then write lines the previous step's edge passes did not
        # read (layer.ForwardPlan pingpong: writing lines another kernel just
        # gathered from costs 12 vs 4.3 us per 11.5 MB on this GPU)
        self.tables = [torch.zeros(lay.numel, dtype=torch.float32, device=dev)
                       for _ in range(2 if pingpong else 1)]
        self._tix = 0
        self.table = self.tables[0]
        n_sd = csr.num_nodes if exchange == "replicate" else self.n_local
        self.s_dst = torch.empty(max(n_sd, 1), heads, dtype=torch.float32, device=dev)
        blk = lay.block_rows if exchange == "allgather" else csr.num_nodes
        self.s_scratch = (torch.empty(max(blk, 1), heads, dtype=torch.float32, device=dev)
                          if kind == "wh" else None)
        width_out = hf if self.concat else f
        self.out = torch.empty(self.n_local, width_out, dtype=torch.float32, device=dev)
        if self.chunks > 1:
            self.st_acc = torch.empty(max(self.n_local, 1), (hf + 3) // 4 * 4,
                                      dtype=torch.float32, device=dev)
            self.st_ml = torch.empty(max(self.n_local, 1), 2 * heads, dtype=torch.float32,
                                     device=dev)
        else:
            self.st_acc = self.st_ml = None
        # the projection's optional workspace (HIP ops only; CPU stand-ins take none)
        self.pws = (self.ops.workspace(dev, layer.input_channels, heads, f)
                    if hasattr(self.ops, "workspace") else None)
        if exchanger is None:
            exchanger = CollectiveExchange(group) if (
                exchange == "allgather" and (world > 1 or self.force_exchange)) else NoExchange()
        self.exchanger = exchanger

    def _local_csr(self, csr, e0: int, e1: int, dev) -> LocalCSR:
        """This rank's rows with source ids remapped to table rows, sorted
        within each row by table row, and the per-pass segment bounds."""
        lay = self.layout
        rp = csr.rowptr
        lrp = (rp[self.r0:self.r1 + 1] - e0).to(torch.int64)
        col = csr.col[e0:e1].to(torch.int64)
        if self.exchange == "allgather":
            b = torch.tensor(self.bounds, dtype=torch.int64, device=dev)
            owner = torch.searchsorted(b[1:], col, right=True)
            trow = lay.row_of(owner, col - b[owner])
        else:
            trow = lay.row_of(torch.zeros_like(col), col)
        deg = lrp[1:] - lrp[:-1]
        row_id = torch.repeat_interleave(torch.arange(self.n_local, device=dev), deg)
        # sources ascending by table row inside each row: each pass's sources
        # are one contiguous segment, and concurrently scheduled rows sweep the
        # table in step (the L2 locality of the single-GPU CSR)
        key = row_id * lay.table_rows + trow
        key, _ = torch.sort(key)
        trow = key - row_id * lay.table_rows
        seg = torch.empty(lay.chunks + 1, self.n_local, dtype=torch.int32, device=dev)
        seg[0] = lrp[:-1].to(torch.int32)
        if lay.chunks > 1:
            ch = lay.chunk_of_row(trow)
            cnt = torch.zeros(self.n_local * lay.chunks, dtype=torch.int64, device=dev)
            cnt.index_add_(0, row_id * lay.chunks + ch, torch.ones_like(ch))
            cum = lrp[:-1].unsqueeze(1) + cnt.view(self.n_local, lay.chunks).cumsum(1)
            seg[1:] = cum.t().to(torch.int32)
        else:
            seg[1] = lrp[1:].to(torch.int32)
        lrp32 = lrp.to(torch.int32).contiguous()
        return LocalCSR(lrp32, trow.to(torch.int32).contiguous(), self.n_local, e1 - e0,
                        degree_order(lrp32), seg.contiguous())

    # -- the pieces of a step ------------------------------------------------
    def local_x(self, x_full):
        """This rank's input rows (allgather) or all of x (replicate).  A fresh
        copy: a row view of x starts off a 16-B boundary whenever r0 * Fin is
        not a multiple of 4, and the projection kernels load x in float4s."""
        return x_full[self.r0:self.r1].clone() if self.exchange == "allgather" else x_full

    def project_chunk(self, xl, c: int) -> None:
        lay = self.layout
        if self.exchange == "replicate":
            self.ops.project_rows(xl, self.pp, self.heads, self.f, lay, self.table, 0,
                                  self.s_dst, self.s_scratch, **self._ws_kw())
            return
        lo = c * lay.block_rows
        hi = min(lo + lay.block_rows, self.n_local)
        if hi <= lo:
            return
        self.ops.project_rows(xl[lo:hi], self.pp, self.heads, self.f, lay, self.table,
                              lay.block_offset(c, self.rank), self.s_dst[lo:hi], self.s_scratch,
                              **self._ws_kw())

    def _ws_kw(self):
        return {} if self.pws is None else {"ws": self.pws}

    def project_all(self, xl) -> None:
        """Every chunk's projection: one launch over all of the rank's rows
        where the ops and the table layout allow it (planes, several chunks:
        a per-chunk launch pays a whole block's latency for 1/K of the rows),
        else one launch per chunk."""
        lay = self.layout
        if (self.exchange == "allgather" and lay.kind == "planes" and self.chunks > 1
                and hasattr(self.ops, "project_chunked") and lay.block_rows % 64 == 0):
            self.ops.project_chunked(xl, self.pp, self.heads, self.f, lay, self.table,
                                     self.rank, self.s_dst, **self._ws_kw())
            return
        for c in range(self.chunks):
            self.project_chunk(xl, c)

    def exchange_start(self, c: int):
        if self.exchange != "allgather" or (self.world == 1 and not self.force_exchange):
            return None
        lo, hi = self.layout.chunk_range(c)
        off = self.layout.block_offset(c, self.rank)
        return self.exchanger.start(self.table[lo:hi],
                                    self.table[off:off + self.layout.block_floats])

    def edge_pass(self, c: int):
        k = self.chunks
        flags = (_lib.GAT_SEG_LOAD if c > 0 else 0) | (_lib.GAT_SEG_STORE if c < k - 1 else 0)
        s_dst = self.s_dst[self.r0:self.r1] if self.exchange == "replicate" else self.s_dst
        return self.ops.edge_pass(self.local, c, self.layout, self.table, s_dst, self.pp,
                                  self.bias, self.heads, self.f, self.concat, self.act,
                                  self.param, self.out, self.st_acc, self.st_ml, flags)

    def forward(self, xl):
        """One step: x = this rank's rows (allgather) or all rows (replicate)."""
        if len(self.tables) > 1:
            self._tix ^= 1
            self.table = self.tables[self._tix]
        if self.exchange == "replicate":
            self.project_chunk(xl, 0)
            return self.edge_pass(0)
        self.project_all(xl)
        handles = [self.exchange_start(c) for c in range(self.chunks)]
        for c in range(self.chunks):
            self.exchanger.wait(handles[c])
            self.edge_pass(c)
        return self.out

    # split phases, for timing the collective and the compute alone
    def phase_project(self, xl):
        self.project_all(xl)

    def phase_exchange(self):
        hs = [self.exchange_start(c) for c in range(self.chunks)]
        for h in hs:
            self.exchanger.wait(h)

    def phase_edges(self):
        for c in range(self.chunks):
            self.edge_pass(c)
        return self.out


def emulate(layer, csr, x, world: int, exchange: str = "allgather",
            chunks: Optional[int] = None) -> torch.Tensor:
    """P ranks in ONE process on one device: every rank's projection, the
    all-gather emulated by block copies, every rank's edge passes; returns the
    concatenated output [N, width].  Runs the real kernels on the real
    per-rank tables, segments and state buffers."""
    ranks, xs = _emulated_ranks(layer, csr, x, world, exchange, chunks)
    outs = [sh.phase_edges() for sh in ranks]
    return torch.cat(outs)


def _emulated_ranks(layer, csr, x, world: int, exchange: str, chunks: Optional[int]):
    """Every rank's ShardedGAT in one process, projected, tables filled by
    block copies (the all-gather's result)."""
    ranks = [ShardedGAT(layer, csr, world, r, exchange=exchange, chunks=chunks,
                        exchanger=NoExchange(), pingpong=False) for r in range(world)]
    lay = ranks[0].layout
    for sh in ranks[1:]:
        # the layout fixes the collectives' sizes: every rank must agree
        if sh.layout != lay:
            raise RuntimeError(f"rank {sh.rank} table layout {sh.layout} != rank 0's {lay}")
    xs = [sh.local_x(x) for sh in ranks]
    for sh, xl in zip(ranks, xs):
        sh.phase_project(xl)
    if exchange == "allgather" and world > 1:
        for c in range(lay.chunks):
            for src in ranks:
                off = lay.block_offset(c, src.rank)
                blk = src.table[off:off + lay.block_floats]
                for dst in ranks:
                    if dst is not src:
                        dst.table[off:off + lay.block_floats].copy_(blk)
    return ranks, xs


def emulate_rank_times(layer, csr, x, world: int, exchange: str = "allgather",
                       chunks: Optional[int] = None, iters: int = 20) -> Dict:
    """The COMPUTE side of one partitioned step, measured on one GPU: for each
    of ``world`` emulated ranks, its projection (``phase_project``) and its
    edge passes (``phase_edges``) alone, HIP events on the current stream, on
    the rank's real table, local CSR and segments.  A rank of a real
    multi-GPU run does exactly this work on its own GPU, plus the collective;
    the max over ranks bounds the step from below (SURVEY.md §8e cost model)."""
    ranks, xs = _emulated_ranks(layer, csr, x, world, exchange, chunks)
    per = []
    for sh, xl in zip(ranks, xs):
        # median of 3 measurements of `iters` launches each: one rank's single
        # disturbed measurement would otherwise set the max over ranks.  GPU
        # time: the launches replayed from a captured graph (a rank's share of
        # a small graph is a few microseconds of GPU work, less than the
        # Python + ctypes enqueue of an eager launch, which the eager numbers
        # beside it include)
        proj = statistics.median(_graph_ms(lambda: sh.phase_project(xl), iters) for _ in range(3))
        edge = statistics.median(_graph_ms(sh.phase_edges, iters) for _ in range(3))
        proj_e = statistics.median(_event_ms(lambda: sh.phase_project(xl), iters)
                                   for _ in range(3))
        edge_e = statistics.median(_event_ms(sh.phase_edges, iters) for _ in range(3))
        per.append({"rank": sh.rank, "rows": sh.n_local, "local_edges": sh.local.num_edges,
                    "project_ms": proj, "edge_passes_ms": edge,
                    "project_ms_eager": proj_e, "edge_passes_ms_eager": edge_e})
    lay = ranks[0].layout
    blk_bytes = 4 * lay.block_floats
    recv = blk_bytes * lay.chunks * (world - 1) if exchange == "allgather" else 0
    res = {"ranks": world, "exchange": exchange, "chunks": lay.chunks,
           "table_layout": lay.kind, "table_bytes_per_rank": 4 * lay.numel,
           "collective_bytes_received_per_rank": recv,
           "max_project_ms": max(p["project_ms"] for p in per),
           "max_edge_passes_ms": max(p["edge_passes_ms"] for p in per),
           "max_compute_ms": max(p["project_ms"] + p["edge_passes_ms"] for p in per),
           "max_compute_ms_eager": max(p["project_ms_eager"] + p["edge_passes_ms_eager"]
                                       for p in per),
           "timing": "GPU time per step from a captured graph of `iters` steps (the _eager "
                     "fields: eager launches, host enqueue included)",
           "per_rank": per}
    del ranks, xs
    torch.cuda.empty_cache()
    return res


def gather_output(local_out: torch.Tensor, bounds: List[int], group=None) -> torch.Tensor:
    """Concatenate the sharded outputs on every rank (checks only; not part of
    a step).  Staged through host memory, so any group backend works."""
    world = len(bounds) - 1
    m = max(bounds[k + 1] - bounds[k] for k in range(world))
    pad = torch.zeros(m, local_out.size(1), dtype=local_out.dtype)
    pad[:local_out.size(0)] = local_out.cpu()
    allp = torch.empty(world * m, local_out.size(1), dtype=local_out.dtype)
    dist.all_gather_into_tensor(allp, pad, group=group)
    return torch.cat([allp[k * m:k * m + bounds[k + 1] - bounds[k]] for k in range(world)])


# ---------------------------------------------------------------------------
# bench.py --gpus N (torchrun, one process per GPU, RCCL)
# ---------------------------------------------------------------------------
def _time_steps(step, warmup: int, steps: int) -> float:
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
    t = torch.tensor([elapsed], dtype=torch.float64)  # default group: gloo, on the host
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _event_ms(fn, iters: int) -> float:
    """Mean GPU time of fn over iters, HIP events on the current stream."""
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record(s)
    for _ in range(iters):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


def _graph_ms(fn, iters: int) -> float:
    """Mean GPU time of fn over iters calls captured into one graph and
    replayed (no host enqueue between the launches); events on the stream."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()  # warm: plans, workspaces and lazy buffers exist before capture
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    ms = _event_ms(g.replay, 1) / iters
    del g
    return ms


def _make_layer(w, dev):
    from .layer import GraphAttentionLayer
    torch.manual_seed(0)
    return GraphAttentionLayer(w.in_channels, w.out_channels, num_heads=w.heads,
                               concat=w.concat).to(dev).eval()


def _max_over_ranks(v: float) -> float:
    t = torch.tensor([v], dtype=torch.float64)  # default group: gloo, on the host
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _strategy_key(exchange: str, chunks: int) -> str:
    return "replicate" if exchange == "replicate" else f"allgather_k{chunks}"


def _sharded_workload(w, dev, world: int, rank: int, exchanger, args, strategies,
                      force_exchange: bool = False, keep_for_graph: bool = False) -> Dict:
    """ONE shared graph of workload w, node-range partitioned over the ranks
    (SURVEY.md §8e).  Each strategy in ``strategies`` — (exchange, chunks):
    ("allgather", K) = project own rows -> K-chunk all-gather of the node table
    over the exchanger (RCCL) -> K edge passes overlapped with it;
    ("replicate", 1) = every rank projects all rows, no collective — is timed
    for a few steps.  The workload's ``value`` is the fastest all-gather
    strategy (the north-star design), timed for the full K steps;
    "replicate" is timed too and reported beside it (``replicate``), never in
    its place.  Each with its collective and compute phases alone.
    Also on rank 0: the same layer forward on the whole graph on one GPU (the
    1-GPU reference for this workload) and a check that every reported
    strategy's gathered output equals it."""
    from .graph import build_csr
    from .synthetic import make_inputs

    x, ei = make_inputs(w, dev)  # same seeds on every rank -> the same graph
    csr = build_csr(ei, x.size(0))
    layer = _make_layer(w, dev)
    res = {"workload": w.name, "N": x.size(0), "E_prime": csr.num_edges,
           "Fin": w.in_channels, "H": w.heads, "F": w.out_channels, "concat": w.concat}
    ref = None
    with torch.no_grad():
        if rank == 0:  # the single-GPU forward of the same workload (others wait)
            def one():  # the layer module with its cached plan, as bench.py's N = 1 line
                return layer(x, ei)
            for _ in range(max(3, args.warmup)):
                ref = one()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                one()
            torch.cuda.synchronize()
            ms1 = (time.perf_counter() - t0) * 1e3 / args.steps
            ref = one().cpu()
            res["one_gpu"] = {"value": csr.num_edges / (ms1 * 1e-3), "ms_per_step": ms1,
                              "launch": "eager",
                              "what": "the same layer forward on the whole graph on rank 0's "
                                      "GPU alone (bench.py's single-GPU path: the layer "
                                      "module, eager)"}
            if keep_for_graph:
                # the same forward replayed from a captured graph: the one-GPU
                # value a graph-replayed N-rank step is compared with
                res["one_gpu"]["graph"] = _one_gpu_graph(one, csr.num_edges, args)
        dist.barrier()
        from .graph import csr_cache
        csr_cache.clear()  # the module's own CSR of ei (rank 0): not needed any more
        del ei
        # try each strategy for a few steps (every rank runs the same list: the
        # layout, hence the skip decision, depends only on global values)
        tried = {}
        built = {}
        for exch, k in strategies:
            sh = ShardedGAT(layer, csr, world, rank, exchange=exch, chunks=k,
                            exchanger=exchanger if exch == "allgather" else NoExchange(),
                            force_exchange=force_exchange)
            if exch == "allgather" and sh.chunks != k:
                continue
            key = _strategy_key(exch, k)
            xl = sh.local_x(x)
            t = _time_steps(lambda: sh.forward(xl), 2, 5)
            tried[key] = t * 1e3 / 5
            built[key] = (sh, xl)
        # the headline is the north-star design (node-range partition + RCCL
        # all-gather), its fastest chunk count; "replicate" (no collective) is
        # measured and reported beside it, never in its place
        ag = [k_ for k_ in tried if k_.startswith("allgather")]
        best = min(ag, key=tried.get) if ag else min(tried, key=tried.get)
        rep = "replicate" if "replicate" in tried and best != "replicate" else None
        for key in list(built):  # free the other trials' tables
            if key not in (best, rep):
                del built[key]
        torch.cuda.empty_cache()

        def measure(key):
            sh, xl = built[key]
            t = _time_steps(lambda: sh.forward(xl), args.warmup, args.steps)
            ms = t * 1e3 / args.steps
            d = {"strategy": key, "exchange": sh.exchange, "chunks": sh.chunks,
                 "value": csr.num_edges / (ms * 1e-3), "ms_per_step": ms}
            # the pieces alone (max over ranks): collective, projection, edge passes
            if sh.exchange == "allgather" and (world > 1 or force_exchange):
                d["collective_ms"] = _time_steps(sh.phase_exchange, 2, args.steps) * 1e3 / \
                    args.steps
            d["project_ms_max_over_ranks"] = _max_over_ranks(
                _event_ms(lambda: sh.phase_project(xl), args.steps))
            d["edge_passes_ms_max_over_ranks"] = _max_over_ranks(
                _event_ms(sh.phase_edges, args.steps))
            lay = sh.layout
            d.update({"rows_per_rank": sh.rows_per_part, "table_bytes": int(sh.table.numel() * 4),
                      "table_layout": lay.kind, "planes": sh.slices,
                      "rank0_local_edges": sh.local.num_edges if rank == 0 else None,
                      "collective_bytes_received_per_rank":
                          4 * lay.block_floats * lay.chunks * (world - 1)
                          if sh.exchange == "allgather" else 0})
            # check: gathered sharded output == the single-GPU forward
            sh.forward(xl)
            full = gather_output(sh.out, sh.bounds)
            if rank == 0:
                diff = float((full - ref).abs().max())
                scale = float(ref.abs().max())
                d["check"] = {"max_abs_diff_vs_one_gpu": diff, "max_abs_ref": scale}
                if not diff <= 1e-5 + 1e-5 * scale:
                    raise RuntimeError(f"sharded {w.name} ({key}) output differs from the "
                                       f"single-GPU forward: max |diff| {diff:.3e} "
                                       f"(max |ref| {scale:.3e})")
            return d

        head = measure(best)
        repd = measure(rep) if rep is not None else None
        if keep_for_graph and head["exchange"] == "allgather":
            # kept for graph_trial() after every eager measurement
            res["_graph_ctx"] = (built[best][0], built[best][1], ref, csr.num_edges, best)
    res.update({k_: v for k_, v in head.items()})
    res["unit"] = "edges/s"
    res["strategy_trials_ms"] = tried
    res["replicate"] = repd
    if rank == 0:
        res["speedup_vs_one_gpu"] = res["value"] / res["one_gpu"]["value"]
        if repd is not None:
            repd["speedup_vs_one_gpu"] = repd["value"] / res["one_gpu"]["value"]
    del built, x, csr
    torch.cuda.empty_cache()
    return res


def _one_gpu_graph(one, e_prime: int, args, per_replay: int = 2) -> Dict:
    """``one`` (the layer forward on the whole graph) replayed from a captured
    graph, timed as the eager steps are (synchronize around K steps).  Like
    the sharded graphs (``capture_steps``), ``per_replay`` consecutive
    forwards are captured into one graph, so both sides of the graph
    speed-up pay the same replay cost per step and alternate their ping-pong
    workspaces the same way."""
    try:
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(3):
                one()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            for _ in range(per_replay):
                one()
    except Exception as exc:  # noqa: BLE001 -- reported; the eager value stands
        return {"ok": False, "error": f"{type(exc).__name__}: {exc}"[:300]}
    reps = max(1, args.steps // per_replay)
    for _ in range(max(3, args.warmup // per_replay)):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / (reps * per_replay)
    del g
    return {"ok": True, "value": e_prime / (ms * 1e-3), "ms_per_step": ms,
            "launch": f"hipGraph ({per_replay} steps per replay)"}


def capture_steps(sh: "ShardedGAT", xl, steps: int = 2) -> "torch.cuda.CUDAGraph":
    """``steps`` consecutive sharded forwards (the two ping-pong node tables,
    the chunk all-gathers included) captured into ONE graph: a replay is
    ``steps`` complete steps with no host enqueue between their launches.
    The collectives are RCCL kernels recorded in the graph (the process
    group's stream joins the capture through its event wait); every rank
    must replay its graph in the same order, as with eager collectives."""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):  # warm on a side stream before capturing
        for _ in range(steps):
            sh.forward(xl)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        for _ in range(steps):
            sh.forward(xl)
    return g


def graph_trial(ctx, world: int, rank: int, args, w_name: str,
                compute_only: bool = False) -> Dict:
    """The headline all-gather strategy replayed from a captured graph (two
    steps per replay; ``capture_steps``), timed as the eager steps are
    (barrier + synchronize around K steps, max over ranks) and checked
    against the one-GPU forward.  At a small graph's share a rank's eager
    step is host-bound (the c10d + RCCL enqueue of the all-gather alone is
    ~20-30 us at one rank), which the graph removes.  Runs after every eager
    measurement: a capture that fails on any rank (the ranks agree over the
    host group before any replay) is reported, and no graph is replayed.

    compute_only (the one-GPU rehearsal, whose host-staged exchange copies
    through host memory and cannot be captured): both ping-pong tables are
    filled by eager steps with the exchange, and the graph holds each rank's
    projection and edge passes only (the remote rows stay those of the eager
    exchange: the inputs do not change).  The capture, the ranks' agreement
    and the replay run as in the real step; the value is not a step's."""
    sh, xl, ref, e_prime, key = ctx
    per = 2
    ok, err = 1, None
    saved = sh.exchanger
    try:
        if compute_only:
            for _ in range(per):  # both tables, with the exchange
                sh.forward(xl)
            torch.cuda.synchronize()
            sh.exchanger = NoExchange()
        g = capture_steps(sh, xl, per)
    except Exception as exc:  # noqa: BLE001 -- reported, never replayed
        ok, err, g = 0, f"{type(exc).__name__}: {exc}"[:300], None
    flag = torch.tensor([ok], dtype=torch.int64)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)  # default group: gloo, on the host
    if int(flag.item()) == 0:
        sh.exchanger = saved
        return {"ok": False, "error": err or "capture failed on another rank"}
    reps = max(1, args.steps // per)
    t = _time_steps(g.replay, max(1, args.warmup // per), reps)
    ms = t * 1e3 / (reps * per)
    launch = f"hipGraph ({per} steps per replay)"
    if compute_only:
        launch += ", compute only (exchange eager before capture: rehearsal)"
    d = {"ok": True, "strategy": key, "launch": launch, "compute_only": compute_only,
         "value": e_prime / (ms * 1e-3), "ms_per_step": ms}
    g.replay()
    torch.cuda.synchronize()
    sh.exchanger = saved
    full = gather_output(sh.out, sh.bounds)
    if rank == 0:
        diff = float((full - ref).abs().max())
        scale = float(ref.abs().max())
        d["check"] = {"max_abs_diff_vs_one_gpu": diff, "max_abs_ref": scale}
        if not diff <= 1e-5 + 1e-5 * scale:
            raise RuntimeError(f"graphed sharded {w_name} ({key}) output differs from the "
                               f"single-GPU forward: max |diff| {diff:.3e}")
    del g
    return d


def _ppi_blocks_weak(w, dev, world: int, rank: int, args) -> Dict:
    """Secondary: data-parallel PPI-shape blocks (the real PPI dataset is a set
    of disjoint graphs): rank k owns one block seeded +1000k, the halo is empty
    and the step has no collective.  Weak scaling."""
    from .graph import get_csr
    from .synthetic import make_inputs
    layer = _make_layer(w, dev)
    x, ei = make_inputs(w, dev, x_seed=1 + 1000 * rank, edge_seed=2 + 1000 * rank)
    csr = get_csr(ei, x.size(0))
    with torch.no_grad():
        t = _time_steps(lambda: layer(x, ei), args.warmup, args.steps)
    e_blk = torch.tensor([csr.num_edges], dtype=torch.float64)
    dist.all_reduce(e_blk)
    ms = t * 1e3 / args.steps
    return {"value": float(e_blk.item()) / (ms * 1e-3), "unit": "edges/s", "ms_per_step": ms,
            "scaling": "weak",
            "what": f"{world} disjoint PPI-shape blocks, one per GPU (N={x.size(0)}, "
                    f"E'={csr.num_edges} each); no collective in the step"}


def bench_distributed(args, metric: str):
    """One process per GPU (torchrun).  The reported line is BASELINE.json's
    metric on its own workload: the PPI-shape graph (configs[1]) as ONE
    shared graph, node-range partitioned over the ranks, the
    exchange inside the timed step.  Strong scaling: total work is fixed as N
    grows, so ``value`` at N GPUs compares directly with the N = 1 line's PPI
    ``value``.  Reddit scale (configs[4]) and ogbn-arxiv scale (configs[3])
    run the same way under ``workloads``, each with its own one-GPU time and
    ``speedup_vs_one_gpu``; the data-parallel PPI-block run is a secondary
    field.

    At WORLD_SIZE = 1 (``--dist``) the all-gather strategies still issue their
    collectives, in place, over a one-rank RCCL group, so the RCCL path runs on
    a one-GPU box."""
    from .synthetic import WORKLOADS

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    share = bool(os.environ.get("GAT_BENCH_SHARE_GPU0"))  # rehearsal: every rank on cuda:0
    if share:
        local_rank = 0
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    # rank 0 prints exactly one JSON line on stdout; RCCL prints its banner and
    # warnings to stdout from C, so fd 1 points at stderr until the result is ready
    sys.stdout.flush()
    saved_stdout = os.dup(1)
    os.dup2(2, 1)
    # default group gloo: barriers and the max-over-ranks reduction on the host;
    # the table all-gather runs on an RCCL group (nccl backend = RCCL on ROCm)
    os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
    if "MASTER_ADDR" not in os.environ:  # plain `python bench.py --dist` (one rank)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0",
                          WORLD_SIZE="1")
    dist.init_process_group("gloo")
    force = False
    if not share:
        exchanger = CollectiveExchange(dist.new_group(backend="nccl"))
        xname = "RCCL all_gather_into_tensor (in place, async, one per chunk)"
        force = world == 1
        if force:
            xname += ", one-rank group (in-place self all-gather)"
    else:
        exchanger = HostStagedExchange(None)
        xname = "gloo all-gather staged through host memory (one-GPU rehearsal)"
    names = [s for s in getattr(args, "dist_workloads", "ppi,reddit,arxiv").split(",") if s]
    chunk_choices = [1, 2, 4] if world > 1 else [1, 2]
    strategies = [("allgather", k) for k in chunk_choices] + [("replicate", 1)]
    # graph-replayed steps for the small shapes, where a rank's eager step is
    # host-bound; the one-GPU rehearsal (host-staged exchange, not capturable)
    # captures each rank's compute only, to exercise the capture agreement and
    # the replay, and never reports it as the step
    graph_names = set() if getattr(args, "no_dist_graph", False) else \
        {nm for nm in names if nm in ("ppi", "arxiv", "cifar")}
    work = {}
    for nm in names:
        work[nm] = _sharded_workload(WORKLOADS[nm], dev, world, rank, exchanger, args,
                                     strategies, force_exchange=force,
                                     keep_for_graph=nm in graph_names)
    # the eager results reach the detail file before any capture is attempted
    if rank == 0:
        from .benchline import write_detail
        write_detail({"stage": "eager measurements, before any graph capture",
                      "workloads": {k: {kk: vv for kk, vv in v.items() if kk != "_graph_ctx"}
                                    for k, v in work.items()}},
                     getattr(args, "detail_out", None))
    for i, nm in enumerate(names):
        ctx = work[nm].pop("_graph_ctx", None)
        if ctx is None:
            continue
        gt = graph_trial(ctx, world, rank, args, nm, compute_only=share)
        del ctx
        work[nm]["graph"] = gt
        if not gt.get("ok"):
            # no further capture after a failure: free the other trials' tables
            for rest in names[i + 1:]:
                work[rest].pop("_graph_ctx", None)
            torch.cuda.empty_cache()
            break
        if rank == 0:
            og = work[nm]["one_gpu"]
            work[nm]["speedup_vs_one_gpu_eager"] = work[nm]["value"] / og["value"]
            if og.get("graph", {}).get("ok"):
                gt["speedup_vs_one_gpu_graph"] = gt["value"] / og["graph"]["value"]
        if not share and gt["value"] > work[nm]["value"]:
            # the same strategy and work per step, launched from the graph; the
            # speed-up against the one-GPU forward launched the same way
            work[nm]["eager"] = {"value": work[nm]["value"],
                                 "ms_per_step": work[nm]["ms_per_step"]}
            work[nm]["value"], work[nm]["ms_per_step"] = gt["value"], gt["ms_per_step"]
            work[nm]["launch"] = gt["launch"]
            if rank == 0:
                og = work[nm]["one_gpu"]
                if og.get("graph", {}).get("ok"):
                    work[nm]["speedup_vs_one_gpu"] = gt["speedup_vs_one_gpu_graph"]
                    work[nm]["speedup_launch_mode"] = "hipGraph vs hipGraph"
                else:  # no graphed one-GPU value: keep the like-for-like eager ratio
                    work[nm]["speedup_vs_one_gpu"] = work[nm]["speedup_vs_one_gpu_eager"]
                    work[nm]["speedup_launch_mode"] = "eager vs eager (one-GPU capture failed)"
        torch.cuda.empty_cache()
    for nm in names:
        work[nm].pop("_graph_ctx", None)
        if rank == 0:
            work[nm].setdefault("speedup_launch_mode", "eager vs eager")
    weak = None
    if not getattr(args, "no_weak", False):
        weak = _ppi_blocks_weak(WORKLOADS["ppi"], dev, world, rank, args)
    res = None
    if rank == 0:
        head = work[names[0]]
        w = WORKLOADS[names[0]]
        if head["exchange"] == "allgather":
            par = (f"node-range partition x{world} (edge-balanced), node table all-gathered "
                   f"in {head['chunks']} chunk(s) overlapped with the edge passes")
        else:
            par = (f"node-range partition x{world} (edge-balanced) of the edge work; every rank "
                   "projects all rows (SURVEY.md §8e 'replicate': no collective in the step)")
        res = {
            "metric": metric, "value": head["value"], "unit": "edges/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": head["ms_per_step"],
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (seeded uniform graph of the named shape; reference-order random "
                    "init)",
            "config": {"workload": f"{w.name}: N={head['N']} E={w.num_edges} (+N self-loops = "
                                   f"{head['E_prime']}) Fin={w.in_channels} H={w.heads} "
                                   f"F={w.out_channels} concat={w.concat}, one graph shared by "
                                   f"{world} GPUs",
                       "parallelism": par, "strategy": head["strategy"],
                       "strategy_choice": "fastest all-gather chunk count of the strategy "
                                          "trials; 'replicate' reported beside it (every "
                                          "reported strategy checked against the one-GPU "
                                          "forward)",
                       "exchange": xname, "launch": head.get("launch", "eager")},
            "one_gpu_same_workload": head.get("one_gpu"),
            "speedup_vs_one_gpu": head.get("speedup_vs_one_gpu"),
            "speedup_launch_mode": head.get("speedup_launch_mode"),
            "replicate": head.pop("replicate", None),
            "workloads": {k: v for k, v in work.items() if k != names[0]},
            "headline_detail": head,
            "ppi_blocks_data_parallel": weak,
        }
    dist.barrier()
    dist.destroy_process_group()
    sys.stdout.flush()
    os.dup2(saved_stdout, 1)
    os.close(saved_stdout)
    if res is not None:
        from .benchline import compact_dist, write_detail
        path = write_detail(res, getattr(args, "detail_out", None))
        print(json.dumps(compact_dist(res, path)), flush=True)


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]
