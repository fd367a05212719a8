"""Graph preprocessing: COO ``edge_index`` -> CSR by target with self-loops.

Replaces ``torch_geometric.utils.add_self_loops`` (``GAT.py:38``) and the
grouping of edges by target that PyG's ``propagate`` / ``softmax`` /
``aggregate`` perform on every call (``GAT.py:53,60``).  The CSR is built on
the GPU by ``gat_csr_build`` (stable radix sort by target, loop appended last
in each row) and cached per ``edge_index`` tensor, because every caller runs
the layer several times on one graph (``GATNet.py:79,85``: two layers per
forward; the ``run_*.py`` loops: every epoch).
"""
from __future__ import annotations

import collections
import weakref
from typing import NamedTuple, Optional

import torch

from . import _lib


class CSRGraph(NamedTuple):
    rowptr: torch.Tensor  # int32 [N+1]
    col: torch.Tensor  # int32 [E+N], source node ids, ascending within each row
    num_nodes: int
    num_edges: int  # E + N (edges after add_self_loops)
    order: Optional[torch.Tensor] = None  # int32 [N], rows by descending in-degree


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


def build_csr(edge_index: torch.Tensor, num_nodes: int) -> CSRGraph:
    """Build the CSR-by-target (with appended self-loops) on ``edge_index``'s GPU."""
    if edge_index.device.type != "cuda":
        raise RuntimeError("build_csr needs a ROCm device tensor; there is no CPU path")
    ei = _check_edge_index(edge_index, edge_index.device)
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
    if int(flag.item()) != 0:
        # PyG's index_select raises on the same input (GAT.py:53 -> __lift__)
        raise ValueError(f"edge_index contains node ids outside [0, {num_nodes})")
    return CSRGraph(rowptr, col, num_nodes, E + num_nodes, order)


class _CSRCache:
    """Small LRU of CSRs keyed by the identity and version of ``edge_index``."""

    def __init__(self, capacity: int = 8):
        self.capacity = capacity
        self._entries = collections.OrderedDict()

    def get(self, edge_index: torch.Tensor, num_nodes: int) -> CSRGraph:
        key = (edge_index.data_ptr(), edge_index._version, tuple(edge_index.shape),
               edge_index.dtype, num_nodes, edge_index.device)
        hit = self._entries.get(key)
        if hit is not None and hit[0]() is edge_index:
            self._entries.move_to_end(key)
            return hit[1]
        csr = build_csr(edge_index, num_nodes)
        self._entries[key] = (weakref.ref(edge_index), csr)
        while len(self._entries) > self.capacity:
            self._entries.popitem(last=False)
        return csr

    def clear(self) -> None:
        self._entries.clear()


csr_cache = _CSRCache()


def get_csr(edge_index: torch.Tensor, num_nodes: int) -> CSRGraph:
    return csr_cache.get(edge_index, num_nodes)


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


def get_csc(csr: CSRGraph) -> CSCGraph:
    """The CSC of ``csr``, built on first use and kept while ``csr.rowptr`` lives."""
    key = id(csr.rowptr)
    hit = _csc_cache.get(key)
    if hit is not None and hit[0]() is csr.rowptr:
        return hit[1]
    csc = build_csc(csr)
    _csc_cache[key] = (weakref.ref(csr.rowptr), csc)
    weakref.finalize(csr.rowptr, _csc_cache.pop, key, None)
    return csc
