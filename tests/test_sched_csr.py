"""The scheduled CSR copy (graph.SchedCSR) the short-row eval forward walks:
position p holds exactly row order[p]'s in-edges, in CSR order, and the
positions tile the copy contiguously.  Host logic only (CPU tensors)."""
import numpy as np
import torch

from atmlgraphattentionnetworks_amd.graph import CSRGraph, build_sched_csr


def _csr(n, e, seed):
    rng = np.random.default_rng(seed)
    s = np.concatenate([rng.integers(0, n, e), np.arange(n)])
    d = np.concatenate([rng.integers(0, n, e), np.arange(n)])
    idx = np.lexsort((s, d))
    rowptr = np.concatenate([[0], np.cumsum(np.bincount(d, minlength=n))]).astype(np.int32)
    deg = np.diff(rowptr)
    order = np.argsort(-deg, kind="stable").astype(np.int32)
    return CSRGraph(torch.from_numpy(rowptr), torch.from_numpy(s[idx].astype(np.int32)), n,
                    len(s), torch.from_numpy(order))


def test_sched_csr_positions_hold_their_rows():
    csr = _csr(500, 6000, 3)
    sc = build_sched_csr(csr)
    rp, col, order = csr.rowptr.numpy(), csr.col.numpy(), csr.order.numpy()
    b, e, scol = sc.b.numpy(), sc.e.numpy(), sc.col.numpy()
    assert b[0] == 0 and e[-1] == csr.num_edges and (b[1:] == e[:-1]).all()
    for p in range(csr.num_nodes):
        r = order[p]
        assert (scol[b[p]:e[p]] == col[rp[r]:rp[r + 1]]).all()
    assert sc.b.dtype == sc.e.dtype == sc.col.dtype == torch.int32


def test_staggered_sched_csr_rotates_each_row():
    """stagger=True: position p holds the same in-edges as its row, ascending
    from the first source >= p and wrapping around (a rotation of the sorted
    list), so a rows' sweep starts at node p."""
    csr = _csr(700, 14000, 5)
    plain, stag = build_sched_csr(csr), build_sched_csr(csr, stagger=True)
    assert torch.equal(plain.b, stag.b) and torch.equal(plain.e, stag.e)
    b, e = plain.b.numpy(), plain.e.numpy()
    pc, sc = plain.col.numpy(), stag.col.numpy()
    for p in range(csr.num_nodes):
        row, got = pc[b[p]:e[p]], sc[b[p]:e[p]]
        r = int((row < p).sum())
        assert (got == np.concatenate([row[r:], row[:r]])).all(), p
