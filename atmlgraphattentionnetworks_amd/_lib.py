"""ctypes binding of the C-ABI in ``include/gat_amd.h`` (libgat_amd.so, built
in-tree by ``atmlgraphattentionnetworks_amd.build``).

There is no fallback: if the library is missing or fails to load, every op
raises.  The symbols bound here are exactly the ones the header declares.
"""
from __future__ import annotations

import ctypes
import functools
import os
import threading

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_PKG, "libgat_amd.so")

GAT_OK = 0
GAT_EINVAL = -1
GAT_EUNSUPPORTED = -2
GAT_EWORKSPACE = -3
GAT_ABI_VERSION = 12
GAT_HINT_LOCAL = 1 << 30  # OR'd into edges_per_row_hint (include/gat_amd.h)
GAT_HINT_SHORT = 1 << 29  # every row < 1024 in-edges (include/gat_amd.h, ABI 11)
GAT_SEG_LOAD = 1
GAT_SEG_STORE = 2
GAT_MAX_HEADS = 64
GAT_MAX_HF = 256
GAT_ACT_LEAKY_RELU = 0
GAT_ACT_LOG_SIGMOID = 1
GAT_ACT_TANH = 2
GAT_ACT_HEAD_SOFTMAX = 3

_c_int, _c_ll, _c_float, _c_vp = ctypes.c_int, ctypes.c_longlong, ctypes.c_float, ctypes.c_void_p
_c_size_p = ctypes.POINTER(ctypes.c_size_t)
_c_int_p = ctypes.POINTER(ctypes.c_int)
_c_u64 = ctypes.c_ulonglong

# symbol -> (restype, argtypes); mirrors include/gat_amd.h line for line
SIGNATURES = {
    "gat_abi_version": (_c_int, []),
    "gat_tuning_reload": (_c_int, []),
    "gat_table_layout": (_c_int, [_c_int, _c_int, _c_int_p, _c_int_p]),
    "gat_project": (_c_int, [_c_vp, _c_int, _c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp,
                             _c_int, _c_int, _c_vp, _c_int, _c_vp, _c_int, _c_vp, _c_vp]),
    "gat_edge_aggregate": (_c_int, [_c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_vp, _c_int, _c_vp,
                                    _c_int, _c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_int,
                                    _c_float, _c_vp, _c_vp, _c_vp, _c_int, _c_vp]),
    "gat_project_sliced": (_c_int, [_c_vp, _c_int, _c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp,
                                    _c_vp, _c_int, _c_int, _c_int, _c_vp, _c_int, _c_vp, _c_int,
                                    _c_vp, _c_vp]),
    "gat_project_chunked": (_c_int, [_c_vp, _c_int, _c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp,
                                     _c_vp, _c_int, _c_int, _c_int, _c_vp, _c_int, _c_int, _c_ll,
                                     _c_vp, _c_vp]),
    "gat_project_workspace_size": (_c_int, [_c_int, _c_int, _c_int, _c_size_p]),
    "gat_project_ex": (_c_int, [_c_vp, _c_int, _c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp,
                                _c_int, _c_int, _c_int, _c_vp, _c_int, _c_vp, _c_int, _c_vp,
                                _c_int, _c_ll, _c_vp, ctypes.c_size_t, _c_vp]),
    "gat_edge_aggregate_sliced": (_c_int, [_c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_vp, _c_int,
                                           _c_int, _c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_float,
                                           _c_vp, _c_vp, _c_int, _c_vp]),
    "gat_edge_aggregate_seg": (_c_int, [_c_vp, _c_vp, _c_int, _c_vp, _c_vp, _c_int, _c_int,
                                        _c_vp, _c_int, _c_int, _c_int, _c_vp, _c_vp, _c_vp,
                                        _c_int, _c_int, _c_int, _c_float, _c_vp, _c_vp, _c_int,
                                        _c_int, _c_vp, _c_vp, _c_int, _c_vp]),
    "gat_edge_merge": (_c_int, [_c_vp, _c_vp, _c_int, _c_vp, _c_vp, _c_int, _c_int, _c_int,
                                _c_vp, _c_vp, _c_vp, _c_vp, _c_vp]),
    "gat_edge_merge_ex": (_c_int, [_c_vp, _c_vp, _c_vp, _c_int, _c_vp, _c_vp, _c_int, _c_int,
                                   _c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp]),
    "gat_csr_workspace_size": (_c_int, [_c_ll, _c_int, _c_size_p]),
    "gat_csr_build": (_c_int, [_c_vp, _c_ll, _c_int, _c_vp, _c_vp, _c_vp, _c_vp, ctypes.c_size_t,
                               _c_vp, _c_vp]),
    "gat_edge_aggregate_ex": (_c_int, [_c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_vp, _c_int,
                                       _c_vp, _c_int, _c_vp, _c_vp, _c_vp, _c_int, _c_int,
                                       _c_int, _c_int, _c_float, _c_float, _c_u64, _c_vp, _c_vp,
                                       _c_vp, _c_vp, _c_vp, _c_int, _c_vp]),
    "gat_edge_aggregate_train": (_c_int, [_c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_vp, _c_int,
                                          _c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_int, _c_float,
                                          _c_float, _c_u64, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp,
                                          _c_vp, _c_vp, _c_int, _c_vp]),
    "gat_dropout_seed_next": (_c_int, [_c_vp, _c_vp, _c_vp]),
    "gat_csr_rotate": (_c_int, [_c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_int, _c_vp, _c_vp]),
    "gat_csr_schedule_workspace_size": (_c_int, [_c_int, _c_size_p]),
    "gat_csr_schedule": (_c_int, [_c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_vp, _c_vp, _c_vp, _c_vp,
                                  ctypes.c_size_t, _c_vp]),
    "gat_csc_rotate": (_c_int, [_c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_vp, _c_vp, _c_vp, _c_vp]),
    "gat_csc_workspace_size": (_c_int, [_c_ll, _c_int, _c_size_p]),
    "gat_csc_build": (_c_int, [_c_vp, _c_vp, _c_int, _c_ll, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp,
                               ctypes.c_size_t, _c_vp]),
    "gat_bwd_table_layout": (_c_int, [_c_int, _c_int, _c_int, _c_int_p]),
    "gat_bwd_targets": (_c_int, [_c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_vp, _c_int, _c_vp,
                                 _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_int,
                                 _c_float, _c_float, _c_u64, _c_vp, _c_vp, _c_vp, _c_int, _c_int,
                                 _c_vp]),
    "gat_bwd_table": (_c_int, [_c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_int,
                               _c_int, _c_vp, _c_vp, _c_int, _c_vp]),
    "gat_bwd_sources_parts": (_c_int, [_c_int, _c_int, _c_int, _c_int_p]),
    "gat_bwd_sources": (_c_int, [_c_vp, _c_vp, _c_vp, _c_int, _c_vp, _c_int, _c_vp, _c_int,
                                 _c_vp, _c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_int, _c_float,
                                 _c_float, _c_u64, _c_vp, _c_vp, _c_int, _c_vp, _c_int, _c_int,
                                 _c_vp]),
    "gat_edge_backward_rows": (_c_int, [_c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_vp, _c_vp,
                                        _c_int, _c_vp, _c_int, _c_vp, _c_vp, _c_vp, _c_vp,
                                        _c_vp, _c_vp, _c_int, _c_int, _c_int, _c_int, _c_float,
                                        _c_float, _c_u64, _c_vp, _c_vp, _c_vp, _c_int, _c_vp]),
    "gat_weight_grad_workspace_size": (_c_int, [_c_int, _c_int, _c_int, _c_size_p]),
    "gat_weight_grad": (_c_int, [_c_vp, _c_int, _c_int, _c_vp, _c_int, _c_int, _c_vp, _c_vp,
                                 ctypes.c_size_t, _c_vp]),
    "gat_layer_forward": (_c_int, [_c_vp, _c_int, _c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp,
                                   _c_vp, _c_int, _c_int, _c_int, _c_vp, _c_vp, _c_vp, _c_vp,
                                   _c_vp, _c_vp, _c_vp, _c_int, _c_float, _c_vp, _c_vp, _c_int,
                                   _c_vp]),
    "gat_layer_forward_fuses": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _c_float]),
    "gat_input_grad": (_c_int, [_c_vp, _c_int, _c_int, _c_int, _c_vp, _c_int, _c_vp, _c_int,
                                _c_vp]),
    "gat_sum_partials_workspace_size": (_c_int, [_c_int, _c_ll, _c_size_p]),
    "gat_sum_partials": (_c_int, [_c_vp, _c_int, _c_ll, _c_vp, _c_vp, ctypes.c_size_t, _c_vp]),
    "gat_src_backward": (_c_int, [_c_vp, _c_vp, _c_int, _c_vp, _c_int, _c_vp, _c_vp, _c_vp,
                                  _c_vp, _c_vp, _c_int, _c_int, _c_int, _c_vp, _c_int,
                                  _c_vp, _c_vp, _c_int, _c_vp]),
}

_lock = threading.Lock()
_lib = None


class GatLibraryError(RuntimeError):
    """Raised on a non-zero status from the HIP library."""


def is_loaded() -> bool:
    return _lib is not None


def load() -> ctypes.CDLL:
    """Load libgat_amd.so (once).  Raises ImportError if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is not built; run `python -m atmlgraphattentionnetworks_amd.build` "
                "(hipcc --offload-arch=gfx950).  There is no CPU fallback.")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        ver = lib.gat_abi_version()
        if ver != GAT_ABI_VERSION:
            raise ImportError(f"libgat_amd.so ABI {ver} != expected {GAT_ABI_VERSION}; rebuild it")
        _lib = lib
        return lib


_MESSAGES = {
    GAT_EINVAL: "invalid argument",
    GAT_EUNSUPPORTED: f"unsupported shape (num_heads <= {GAT_MAX_HEADS}, "
                      f"num_heads*output_channels <= {GAT_MAX_HF})",
    GAT_EWORKSPACE: "workspace too small",
}


def check(status: int, what: str) -> None:
    if status != GAT_OK:
        msg = _MESSAGES.get(status, f"hipError_t {status}")
        raise GatLibraryError(f"{what} failed: {msg}")


@functools.lru_cache(maxsize=None)  # pure function of the shape
def table_layout(heads: int, f: int):
    ld, s_off = ctypes.c_int(), ctypes.c_int()
    check(load().gat_table_layout(heads, f, ctypes.byref(ld), ctypes.byref(s_off)),
          "gat_table_layout")
    return ld.value, s_off.value


def csr_workspace_size(num_edges: int, num_nodes: int) -> int:
    out = ctypes.c_size_t()
    check(load().gat_csr_workspace_size(num_edges, num_nodes, ctypes.byref(out)),
          "gat_csr_workspace_size")
    return out.value


def csr_schedule_workspace_size(num_nodes: int) -> int:
    out = ctypes.c_size_t()
    check(load().gat_csr_schedule_workspace_size(num_nodes, ctypes.byref(out)),
          "gat_csr_schedule_workspace_size")
    return out.value


def csc_workspace_size(nnz: int, num_nodes: int) -> int:
    out = ctypes.c_size_t()
    check(load().gat_csc_workspace_size(nnz, num_nodes, ctypes.byref(out)),
          "gat_csc_workspace_size")
    return out.value


@functools.lru_cache(maxsize=None)  # pure function of the shape
def weight_grad_workspace_size(num_nodes: int, fin: int, hf: int) -> int:
    out = ctypes.c_size_t()
    check(load().gat_weight_grad_workspace_size(num_nodes, fin, hf, ctypes.byref(out)),
          "gat_weight_grad_workspace_size")
    return out.value


@functools.lru_cache(maxsize=None)  # pure function of the shape
def bwd_table_layout(heads: int, f: int, concat: bool) -> int:
    ld = ctypes.c_int()
    check(load().gat_bwd_table_layout(heads, f, int(concat), ctypes.byref(ld)),
          "gat_bwd_table_layout")
    return ld.value


@functools.lru_cache(maxsize=None)  # pure function of the shape
def bwd_sources_parts(num_nodes: int, heads: int, f: int) -> int:
    out = ctypes.c_int()
    check(load().gat_bwd_sources_parts(num_nodes, heads, f, ctypes.byref(out)),
          "gat_bwd_sources_parts")
    return out.value


def project_workspace_bytes(fin: int, heads: int, f: int) -> int:
    """Bytes of the optional projection workspace (gat_project_workspace_size)."""
    n = ctypes.c_size_t(0)
    check(load().gat_project_workspace_size(fin, heads, f, ctypes.byref(n)),
          "gat_project_workspace_size")
    return int(n.value)
