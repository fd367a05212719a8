"""Graph preprocessing: COO ``edge_index`` -> CSR by target with self-loops.

Replaces ``torch_geometric.utils.add_self_loops`` (``GAT.py:38``) and the
grouping of edges by target that PyG's ``propagate`` / ``softmax`` /
``aggregate`` perform on every call (``GAT.py:53,60``).  The CSR is built on
the GPU by ``gat_csr_build`` (one stable radix sort of (target, source) keys
over the input edges plus the N self-loops: rows grouped by target, sources
ascending within a row) and cached per ``edge_index`` tensor, because every caller runs
the layer several times on one graph (``GATNet.py:79,85``: two layers per
forward; the ``run_*.py`` loops: every epoch).
"""
from __future__ import annotations

import collections
import weakref
from typing import NamedTuple, Optional

import torch

from . import _lib, tuning


class HubPlan(NamedTuple):
    """Degree-skew schedule (split hub rows, (m, l, acc) merge).

    Rows with more than 2 * seg_len in-edges ("hubs") are cut into segments
    of seg_len edges that run as separate lane groups of the edge kernel,
    scheduled ahead of the whole rows; gat_edge_merge then combines each
    hub's segment states.  Without this, one 100k-edge row walks serially on
    one lane group and outlasts the rest of the kernel many times over."""
    n_hub: int
    n_vrows: int  # segments of all hubs = the first n_vrows schedule positions
    seg_len: int
    hub_rows: torch.Tensor  # int32 [n_hub]
    hub_vptr: torch.Tensor  # int32 [n_hub + 1]: hub k's segments
    sched_row: torch.Tensor  # int32 [n_vrows + N - n_hub]: target row per position
    sched_b: torch.Tensor  # int32: CSR range of each position
    sched_e: torch.Tensor
    # int32 [n_vrows]: schedule position (= state row) of segment j in hub order,
    # or None when the segments run hub by hub (position j)
    seg_slot: Optional[torch.Tensor] = None


class CSRGraph(NamedTuple):
    rowptr: torch.Tensor  # int32 [N+1]
    col: torch.Tensor  # int32 [E+N], source node ids, ascending within each row
    num_nodes: int
    num_edges: int  # E + N (edges after add_self_loops)
    order: Optional[torch.Tensor] = None  # int32 [N], rows by descending in-degree
    hubs: Optional[HubPlan] = None  # split schedule for rows far above the average
    local: bool = False  # sources lie near their targets in node order (locality_hint)
    max_degree: int = 0  # the longest row's in-edges (0: unknown)

    def kernel_hint(self) -> int:
        """The edge kernels' scheduling hint: E'/N, with GAT_HINT_LOCAL OR'd in
        for a local graph and GAT_HINT_SHORT when every row has fewer than
        1024 in-edges (include/gat_amd.h)."""
        h = self.num_edges // max(self.num_nodes, 1)
        if h <= 0:
            return h
        if self.local:
            h |= _lib.GAT_HINT_LOCAL
        if 0 < self.max_degree < 1024:
            h |= _lib.GAT_HINT_SHORT
        return h


def _check_edge_index(edge_index: torch.Tensor, device: torch.device) -> torch.Tensor:
    if not isinstance(edge_index, torch.Tensor):
        raise TypeError(f"edge_index must be a torch.Tensor, got {type(edge_index).__name__}")
    if edge_index.dim() != 2 or edge_index.size(0) != 2:
        raise ValueError(f"edge_index must have shape [2, E], got {tuple(edge_index.shape)}")
    if edge_index.dtype not in (torch.int64, torch.int32):
        raise ValueError(f"edge_index must be an integer (long) tensor, got {edge_index.dtype}")
    if edge_index.device != device:
        raise ValueError(f"edge_index is on {edge_index.device} but x is on {device}")
    return edge_index.to(torch.int64).contiguous()


def build_csr(edge_index: torch.Tensor, num_nodes: int,
              device: Optional[torch.device] = None) -> CSRGraph:
    """Build the CSR-by-target (with the self-loops added) on ``edge_index``'s
    GPU.  ``device``: the device of the node features; an ``edge_index`` on
    another device raises, as the reference's ``index_select`` would."""
    if edge_index.device.type != "cuda":
        raise RuntimeError("build_csr needs a ROCm device tensor; there is no CPU path")
    ei = _check_edge_index(edge_index, edge_index.device if device is None else device)
    lib = _lib.load()
    E = ei.size(1)
    dev = ei.device
    if E + num_nodes > 0x7FFFFFFF:
        raise ValueError("E + N must fit int32 CSR indices")
    rowptr = torch.empty(num_nodes + 1, dtype=torch.int32, device=dev)
    col = torch.empty(E + num_nodes, dtype=torch.int32, device=dev)
    order = torch.empty(num_nodes, dtype=torch.int32, device=dev)
    ws = torch.empty(_lib.csr_workspace_size(E, num_nodes), dtype=torch.uint8, device=dev)
    flag = torch.empty(1, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    _lib.check(lib.gat_csr_build(ei.data_ptr(), E, num_nodes, rowptr.data_ptr(), col.data_ptr(),
                                 order.data_ptr(), ws.data_ptr(), ws.numel(), flag.data_ptr(),
                                 stream), "gat_csr_build")
    # the range flag and the longest row (order[0]: rows by descending degree)
    # in one device -> host read
    if num_nodes > 0:
        top = order[:1].to(torch.int64).clamp_(0, num_nodes - 1)  # in bounds even if bad
        maxdeg = (rowptr[top + 1] - rowptr[top]).to(torch.int32)
        bad, max_degree = torch.cat([flag, maxdeg]).tolist()
    else:
        bad, max_degree = int(flag.item()), 0
    if bad != 0:
        # PyG's index_select raises on the same input (GAT.py:53 -> __lift__)
        raise ValueError(f"edge_index contains node ids outside [0, {num_nodes})")
    return CSRGraph(rowptr, col, num_nodes, E + num_nodes, order,
                    hub_plan(rowptr, order, E + num_nodes, col=col, max_degree=int(max_degree)),
                    locality_hint(rowptr, col, num_nodes), int(max_degree))


def locality_hint(rowptr: torch.Tensor, col: torch.Tensor, num_nodes: int,
                  window: int = 1024, samples: int = 65536) -> bool:
    """Whether most edges join nodes within ``window`` of each other in node
    order (block-diagonal batches of small graphs such as the CIFAR10
    superpixel batches, kNN graphs): then the rows a wave processes together
    share source rows, and narrow rows prefer two float4s per lane
    (GAT_HINT_LOCAL).  Judged on up to ``samples`` evenly spaced CSR entries;
    graphs of at most 4 * window nodes are never called local (every edge
    would be)."""
    nnz = col.numel()
    if nnz == 0 or num_nodes <= 4 * window:
        return False
    k = min(nnz, samples)
    pos = torch.linspace(0, nnz - 1, k, device=col.device).to(torch.int64)
    row = torch.searchsorted(rowptr[1:].to(torch.int64), pos, right=True)
    near = ((col[pos].to(torch.int64) - row).abs() <= window).to(torch.float32).mean()
    return bool(near >= 0.5)


def hub_segment_len(num_edges: int) -> int:
    """Edges per hub segment: a power of two in [256, 1024], ~E'/50000 (a
    segment should take a small fraction of the whole edge kernel: PPI and
    arxiv scale 256, Reddit scale 1024).  With the segments ordered by source
    (hub_plan), power-law Reddit's edge kernel ran 2.234 / 2.154 / 2.346 /
    2.531 ms at 2048 / 1024 / 512 / 4096 (profiles/r05/edge_ab_hubseg_powerlaw.json);
    uniform Reddit has no row past 2 x 1024.  GAT_HUB_SEG overrides."""
    env = tuning.get("GAT_HUB_SEG")
    if env is not None:
        return max(16, int(env))
    s = 256
    while s < 1024 and 2 * s <= num_edges // 50000:
        s *= 2
    return s


def hub_plan(rowptr: torch.Tensor, order: torch.Tensor, num_edges: int,
             seg_len: Optional[int] = None, col: Optional[torch.Tensor] = None,
             max_degree: Optional[int] = None) -> Optional[HubPlan]:
    """The split schedule for rows with more than 2 * seg_len in-edges, or
    None when there are none (every uniform BASELINE graph).  ``order`` is
    the degree-descending row order, so the hubs are its first rows;
    ``max_degree`` (the longest row, when known) skips the count.
    GAT_HUB_SPLIT=0 disables splitting."""
    if tuning.get("GAT_HUB_SPLIT") == "0" or rowptr.numel() <= 1:
        return None
    seg = seg_len or hub_segment_len(num_edges)
    thresh = 2 * seg
    if max_degree is not None and max_degree <= thresh:
        return None  # (the CSR build read its longest row already: no device sync)
    deg = (rowptr[1:] - rowptr[:-1]).to(torch.int64)
    n_hub = int((deg > thresh).sum())
    if n_hub == 0:
        return None
    o = order.to(torch.int64)
    hub_rows = o[:n_hub]
    hdeg = deg[hub_rows]
    nseg = (hdeg + seg - 1) // seg
    vptr = torch.zeros(n_hub + 1, dtype=torch.int64, device=rowptr.device)
    vptr[1:] = nseg.cumsum(0)
    n_v = int(vptr[-1])
    vhub = torch.repeat_interleave(torch.arange(n_hub, device=rowptr.device), nseg)
    k = torch.arange(n_v, device=rowptr.device) - vptr[vhub]
    rp = rowptr.to(torch.int64)
    # segments of seg edges and a short tail (equal-length segments per hub
    # measured slower on power-law Reddit: 2.072 -> 2.409 ms,
    # profiles/r05/edge_ab_hubshape_powerlaw.json)
    slen = torch.full_like(hdeg, seg)
    vb = rp[hub_rows][vhub] + k * slen[vhub]
    ve = torch.minimum(vb + slen[vhub], rp[hub_rows + 1][vhub])
    rest = o[n_hub:]
    i32 = torch.int32
    vrow = hub_rows[vhub]
    slot = None
    if col is not None:
        # segments by the first source id they gather (stable): the segments
        # running together then sweep the same part of the node table, as
        # equal-length whole rows do (ascending sources within every row).
        # Power-law Reddit edge kernel 2.289 -> 2.242 ms against the hub-by-hub
        # order (without col: segments hub by hub); whole rows by ascending
        # degree measured 3.26 ms and were dropped (profiles/r05/
        # edge_ab_hub_order_powerlaw.json)
        perm = torch.sort(col[vb].to(torch.int64), stable=True).indices
        vrow, vb, ve = vrow[perm], vb[perm], ve[perm]
        slot = torch.empty(n_v, dtype=torch.int64, device=rowptr.device)
        slot[perm] = torch.arange(n_v, device=rowptr.device)
        slot = slot.to(i32).contiguous()
    return HubPlan(n_hub, n_v, seg, hub_rows.to(i32).contiguous(), vptr.to(i32).contiguous(),
                   torch.cat([vrow, rest]).to(i32).contiguous(),
                   torch.cat([vb, rp[rest]]).to(i32).contiguous(),
                   torch.cat([ve, rp[rest + 1]]).to(i32).contiguous(), slot)


class SchedCSR(NamedTuple):
    """The CSR's ``col`` re-laid out in the eval edge kernel's row schedule
    (``order``, rows by descending in-degree): schedule position p's in-edges
    are ``col[b[p]:e[p]]``, adjacent to position p+1's.  A lane group then
    reads its row bounds in one load that does not wait for ``order[p]``, and
    the rows sharing a wave read one contiguous run of ``col``.  Built for
    short-row graphs only (``sched_csr``): there the row prologue's chain of
    dependent loads (order -> rowptr -> col -> Wh) is a large part of a
    wave's life."""
    b: torch.Tensor  # int32 [N]
    e: torch.Tensor  # int32 [N]
    col: torch.Tensor  # int32 [E']


SCHED_MAX_EPR = 64  # scheduled copy below this many in-edges per row (E'/N)
STAGGER_MIN_EPR = 16  # staggered sweeps from this many in-edges per row
ROTATE_STRIDE = 2  # long rows: schedule position p's sweep starts at node 2p mod N


def build_sched_csr(csr: "CSRGraph", stagger: bool = False) -> SchedCSR:
    """The scheduled copy (``gat_csr_schedule``).  ``stagger``: schedule position
    p's in-edges (sources ascending) are rotated to start at the first source
    >= p and wrap around, so the rows the kernel runs at one time sweep the
    node table from offsets that advance with their position in the schedule
    (roughly their start time) instead of all from node 0.  The same edges in
    another order: results equal up to fp32 summation order."""
    n, e = csr.num_nodes, csr.num_edges
    dev = csr.rowptr.device
    b = torch.empty(n, dtype=torch.int32, device=dev)
    en = torch.empty(n, dtype=torch.int32, device=dev)
    col = torch.empty(max(e, 1), dtype=torch.int32, device=dev)
    ws = torch.empty(_lib.csr_schedule_workspace_size(n), dtype=torch.uint8, device=dev)
    _lib.check(_lib.load().gat_csr_schedule(
        csr.rowptr.data_ptr(), csr.col.data_ptr(), csr.order.data_ptr(), n, 1 if stagger else 0,
        b.data_ptr(), en.data_ptr(), col.data_ptr(), ws.data_ptr(), ws.numel(),
        torch.cuda.current_stream(dev).cuda_stream), "gat_csr_schedule")
    return SchedCSR(b, en, col[:e])


def rotate_rows(csr: "CSRGraph", stride: int, max_degree: int = 0) -> torch.Tensor:
    """``csr.col`` with each row rotated to start at its first source >=
    (schedule position * stride) mod N and wrap around (``gat_csr_rotate``):
    the rows the kernel runs at one time then sweep the node table from
    offsets that advance with their start time.  CSR row order kept (so
    ``rowptr`` and the hub schedule still index it); the same edges in another
    order within each row.  Rows of more than ``max_degree`` (> 0) in-edges are
    copied unrotated."""
    dev = csr.rowptr.device
    out = torch.empty(max(csr.num_edges, 1), dtype=torch.int32, device=dev)
    _lib.check(_lib.load().gat_csr_rotate(
        csr.rowptr.data_ptr(), csr.col.data_ptr(), csr.order.data_ptr(), csr.num_nodes,
        int(stride), int(max_degree), out.data_ptr(),
        torch.cuda.current_stream(dev).cuda_stream),
        "gat_csr_rotate")
    return out[:csr.num_edges]


_sched_cache = {}
_rot_cache = {}


def rotated_col(csr: "CSRGraph") -> torch.Tensor:
    """The col array the eval forward walks for LONG rows (E'/N >=
    SCHED_MAX_EPR, where no scheduled copy is built): ``rotate_rows`` with
    stride ROTATE_STRIDE, built on first use and kept while ``csr.rowptr``
    lives (E' * 4 bytes).  Reddit layer step 2.011 -> 1.959 ms, power-law
    Reddit 2.261 -> 2.238 ms; strides 1 / 4 / 6 / 8 / 16: 1.982 / 1.961 /
    1.981 / 2.074 / 3.021 ms (profiles/r06/step_ab_rotate_long_rows.json).  Returns
    ``csr.col`` itself for short rows, no row order, or GAT_EDGE_SCHED=plain."""
    if (tuning.get("GAT_EDGE_SCHED") == "plain" or csr.order is None or csr.num_nodes == 0
            or csr.num_edges // csr.num_nodes < SCHED_MAX_EPR):
        return csr.col
    key = id(csr.rowptr)
    hit = _rot_cache.get(key)
    if hit is not None and hit[0]() is csr.rowptr:
        return hit[1]
    # hub rows (split into segments scheduled by the first source each
    # gathers) stay ascending: power-law Reddit 2.238 -> 2.229 ms
    # (profiles/r06/step_ab_hub_rows_unrotated_powerlaw.json)
    hubs = csr.hubs
    col = rotate_rows(csr, ROTATE_STRIDE, 2 * hubs.seg_len if hubs is not None else 0)
    _rot_cache[key] = (weakref.ref(csr.rowptr), col)
    weakref.finalize(csr.rowptr, _rot_cache.pop, key, None)
    return col




def sched_csr(csr: "CSRGraph") -> Optional[SchedCSR]:
    """The scheduled copy of ``csr`` for the eval forward (built on first use,
    kept while ``csr.rowptr`` lives), or None: long rows (E'/N >=
    SCHED_MAX_EPR: the prologue is a small share, and the copy would double a
    large col array), split hub rows (they have their own schedule), no row
    order, or GAT_EDGE_SCHED=0 (knob).  Costs E' * 4 + N * 8 bytes."""
    if (tuning.get("GAT_EDGE_SCHED") == "0" or csr.order is None or csr.hubs is not None
            or csr.num_nodes == 0 or csr.num_edges // csr.num_nodes >= SCHED_MAX_EPR):
        return None
    key = id(csr.rowptr)
    hit = _sched_cache.get(key)
    if hit is not None and hit[0]() is csr.rowptr:
        return hit[1]
    # staggered sweeps where rows average >= 16 in-edges (PPI: layer step
    # 33.92 -> 33.18 us, same box; arxiv's 8 per row 81.18 -> 81.65 us:
    # profiles/r06/step_ab_stagger.json); GAT_EDGE_SCHED=plain: never
    sc = build_sched_csr(csr, stagger=tuning.get("GAT_EDGE_SCHED") != "plain"
                         and csr.num_edges // csr.num_nodes >= STAGGER_MIN_EPR)
    _sched_cache[key] = (weakref.ref(csr.rowptr), sc)
    weakref.finalize(csr.rowptr, _sched_cache.pop, key, None)
    return sc


class _CSRCache:
    """Small LRU of CSRs keyed by the identity and version of ``edge_index``."""

    def __init__(self, capacity: int = 8):
        self.capacity = capacity
        self._entries = collections.OrderedDict()

    def get(self, edge_index: torch.Tensor, num_nodes: int,
            device: Optional[torch.device] = None) -> CSRGraph:
        if device is not None and isinstance(edge_index, torch.Tensor) and \
                edge_index.device != device:
            raise ValueError(f"edge_index is on {edge_index.device} but x is on {device}")
        # tuning.generation: the hub / row schedule knobs are read when the CSR
        # is built, so a tuning.reload() must not return a CSR built under the
        # previous values (the launch plans key on it too)
        key = (edge_index.data_ptr(), edge_index._version, tuple(edge_index.shape),
               edge_index.dtype, num_nodes, edge_index.device, tuning.generation)
        hit = self._entries.get(key)
        if hit is not None and hit[0]() is edge_index:
            self._entries.move_to_end(key)
            return hit[1]
        csr = build_csr(edge_index, num_nodes, device)
        self._entries[key] = (weakref.ref(edge_index), csr)
        # the entry goes when its edge_index does: the cache must not keep a
        # graph the caller dropped (a CSR can be GBs) alive until LRU eviction
        weakref.finalize(edge_index, self._drop_dead, key)
        while len(self._entries) > self.capacity:
            self._entries.popitem(last=False)
        return csr

    def _drop_dead(self, key) -> None:
        hit = self._entries.get(key)
        if hit is not None and hit[0]() is None:
            del self._entries[key]

    def clear(self) -> None:
        self._entries.clear()


csr_cache = _CSRCache()


def get_csr(edge_index: torch.Tensor, num_nodes: int,
            device: Optional[torch.device] = None) -> CSRGraph:
    return csr_cache.get(edge_index, num_nodes, device)


class CSCGraph(NamedTuple):
    """Transpose of a CSRGraph over its edge positions (``gat_csc_build``):
    the backward pass reduces each source row's gradient over its out-edges."""
    ptr: torch.Tensor  # int32 [N+1], first CSC slot per source node
    dst: torch.Tensor  # int32 [E'], target row per CSC slot
    eid: torch.Tensor  # int32 [E'], CSR position per CSC slot
    csr_to_csc: torch.Tensor  # int32 [E'], CSC slot of each CSR position


def build_csc(csr: CSRGraph) -> CSCGraph:
    lib = _lib.load()
    dev = csr.rowptr.device
    n, nnz = csr.num_nodes, csr.num_edges
    ptr = torch.empty(n + 1, dtype=torch.int32, device=dev)
    idx = torch.empty(3, max(nnz, 1), dtype=torch.int32, device=dev)
    ws = torch.empty(_lib.csc_workspace_size(nnz, n), dtype=torch.uint8, device=dev)
    _lib.check(lib.gat_csc_build(csr.rowptr.data_ptr(), csr.col.data_ptr(), n, nnz,
                                 ptr.data_ptr(), idx[0].data_ptr(), idx[1].data_ptr(),
                                 idx[2].data_ptr(), ws.data_ptr(), ws.numel(),
                                 torch.cuda.current_stream(dev).cuda_stream),
               "gat_csc_build")
    return CSCGraph(ptr, idx[0], idx[1], idx[2])


_csc_cache = {}


CSC_ROTATE_STRIDE = 8  # long rows: source j's out-edges start at target 8j mod N


def rotate_csc(csc: CSCGraph, n: int, e: int, stride: int) -> CSCGraph:
    """Staggered sweeps for the backward source pass (``gat_bwd_sources`` walks
    source rows in node order): source j's CSC slots rotated to start at its
    first target >= stride * j mod N and wrap around, ``dst`` and ``eid``
    together, ``csr_to_csc`` re-inverted (``gat_csc_rotate``).  The same
    out-edges per source in another order (gradients equal up to fp32
    summation order).  Reddit training step (dropout 0.6) 8.65 -> 8.46 ms at
    stride 8; strides 1 / 2 / 4 / 16 / 64: 8.59 / 8.60 / 8.49 / 8.61 / 9.04 ms
    (profiles/r06/train_ab_csc_rotate_reddit.json)."""
    dev = csc.ptr.device
    out = torch.empty(3, max(e, 1), dtype=torch.int32, device=dev)
    _lib.check(_lib.load().gat_csc_rotate(
        csc.ptr.data_ptr(), csc.dst.data_ptr(), csc.eid.data_ptr(), n, int(stride),
        out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(),
        torch.cuda.current_stream(dev).cuda_stream), "gat_csc_rotate")
    return CSCGraph(csc.ptr, out[0, :e], out[1, :e], out[2, :e])


def get_csc(csr: CSRGraph) -> CSCGraph:
    """The CSC of ``csr``, built on first use and kept while ``csr.rowptr`` lives;
    long rows (E'/N >= SCHED_MAX_EPR) get ``rotate_csc`` (GAT_EDGE_SCHED=plain:
    never)."""
    key = id(csr.rowptr)
    hit = _csc_cache.get(key)
    if hit is not None and hit[0]() is csr.rowptr:
        return hit[1]
    csc = build_csc(csr)
    if (tuning.get("GAT_EDGE_SCHED") != "plain" and csr.num_nodes > 0
            and csr.num_edges // csr.num_nodes >= SCHED_MAX_EPR):
        csc = rotate_csc(csc, csr.num_nodes, csr.num_edges, CSC_ROTATE_STRIDE)
    _csc_cache[key] = (weakref.ref(csr.rowptr), csc)
    weakref.finalize(csr.rowptr, _csc_cache.pop, key, None)
    return csc
