"""The locality hint (graph.locality_hint -> GAT_HINT_LOCAL): host logic on CPU
tensors.  A block-diagonal batch of small kNN graphs (the CIFAR10 superpixel
batches, run_gnn_benchmark.py) is local; a uniform graph of the PPI shape is
not; tiny graphs are never called local."""
import numpy as np
import torch

from atmlgraphattentionnetworks_amd import _lib
from atmlgraphattentionnetworks_amd.graph import CSRGraph, locality_hint


def _csr(n, src, dst):
    """CSR by target with self-loops, sources ascending (gat_csr_build's layout)."""
    src = np.concatenate([src, np.arange(n)])
    dst = np.concatenate([dst, np.arange(n)])
    key = dst.astype(np.int64) * n + src
    o = np.argsort(key, kind="stable")
    col = src[o].astype(np.int32)
    rowptr = np.zeros(n + 1, dtype=np.int64)
    np.add.at(rowptr, dst + 1, 1)
    return torch.from_numpy(np.cumsum(rowptr).astype(np.int32)), torch.from_numpy(col)


def test_block_diagonal_batch_is_local():
    rng = np.random.default_rng(0)
    sizes = rng.integers(85, 151, size=200)
    off = np.concatenate([[0], np.cumsum(sizes)])
    src, dst = [], []
    for g, m in enumerate(sizes):
        d = np.repeat(np.arange(m), 8)
        s = rng.integers(0, m, size=8 * m)
        src.append(s + off[g])
        dst.append(d + off[g])
    n = int(off[-1])
    rowptr, col = _csr(n, np.concatenate(src), np.concatenate(dst))
    assert locality_hint(rowptr, col, n)


def test_uniform_graph_is_not_local():
    rng = np.random.default_rng(1)
    n, e = 44_906, 200_000
    dst = rng.integers(0, n, size=e)
    src = (dst + 1 + rng.integers(0, n - 1, size=e)) % n
    rowptr, col = _csr(n, src, dst)
    assert not locality_hint(rowptr, col, n)


def test_small_graph_never_local_and_hint_bit():
    rowptr, col = _csr(100, np.arange(99), np.arange(1, 100))
    assert not locality_hint(rowptr, col, 100)
    g = CSRGraph(rowptr, col, 100, int(col.numel()), None, None, True)
    assert g.kernel_hint() & _lib.GAT_HINT_LOCAL
    assert g.kernel_hint() & ~_lib.GAT_HINT_LOCAL == col.numel() // 100
    assert CSRGraph(rowptr, col, 100, int(col.numel())).kernel_hint() == col.numel() // 100

