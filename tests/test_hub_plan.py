"""Host logic of the hub split (graph.hub_plan, CPU): the schedule the edge
kernel walks and the segment-to-state map gat_edge_merge_ex reads.

Invariants, for both segment orders (the default, and hub by hub when
hub_plan is not given the CSR's col):
- positions [0, n_vrows) are the hub segments, each covering seg_len in-edges
  of its hub (the last one the remainder), and together exactly the hub's row;
- the positions after them are every other row once, whole;
- seg_slot (when present) maps segment j of the hub order to the position it
  runs at, so the merge combines a hub's segments in row order whatever the
  schedule (the bitwise-equality claim of tests/test_gpu_hubs.py);
- default: hub segments sorted by the first source id they gather;
  without col: hub by hub, in row order (no seg_slot);
- whole rows by descending in-degree.
"""
import numpy as np
import pytest
import torch


def _csr(n, e, hubs, seed):
    rng = np.random.default_rng(seed)
    dst = [rng.integers(0, n, e)]
    for row, deg in hubs:
        dst.append(np.full(deg, row))
    dst = np.concatenate(dst)
    src = rng.integers(0, n, dst.size)
    dst = np.concatenate([dst, np.arange(n)])  # self-loops
    src = np.concatenate([src, np.arange(n)])
    key = dst.astype(np.int64) * n + src
    o = np.argsort(key, kind="stable")
    dst, src = dst[o], src[o]
    rowptr = np.zeros(n + 1, dtype=np.int64)
    np.add.at(rowptr, dst + 1, 1)
    rowptr = np.cumsum(rowptr)
    deg = np.diff(rowptr)
    order = np.argsort(-deg, kind="stable")
    return (torch.from_numpy(rowptr.astype(np.int32)), torch.from_numpy(order.astype(np.int32)),
            torch.from_numpy(src.astype(np.int32)), deg)


@pytest.mark.parametrize("by_src", [True, False])
def test_hub_plan_invariants(by_src, monkeypatch):
    from atmlgraphattentionnetworks_amd import tuning
    from atmlgraphattentionnetworks_amd.graph import hub_plan
    for k in ("GAT_HUB_SPLIT", "GAT_HUB_SEG"):
        monkeypatch.delenv(k, raising=False)
    tuning.reload()
    n = 3000
    rowptr, order, col, deg = _csr(n, 40000, [(5, 7000), (17, 2600), (2999, 1300), (0, 900)],
                                   seed=4)
    plan = hub_plan(rowptr, order, int(rowptr[-1]), seg_len=256, col=col if by_src else None)
    assert plan is not None and plan.seg_len == 256
    rp = rowptr.numpy().astype(np.int64)
    hub_rows = plan.hub_rows.numpy()
    assert sorted(hub_rows.tolist()) == sorted(np.nonzero(deg > 512)[0].tolist())
    vptr = plan.hub_vptr.numpy()
    nv = plan.n_vrows
    assert vptr[-1] == nv
    srow, sb, se = plan.sched_row.numpy(), plan.sched_b.numpy(), plan.sched_e.numpy()
    assert srow.size == nv + n - plan.n_hub
    slot = np.arange(nv) if plan.seg_slot is None else plan.seg_slot.numpy()
    assert (plan.seg_slot is not None) == by_src
    assert sorted(slot.tolist()) == list(range(nv))  # a permutation of the segment positions
    for k, r in enumerate(hub_rows):
        pos = slot[vptr[k]:vptr[k + 1]]
        assert (srow[pos] == r).all()
        # segment j of the hub covers [rowptr[r] + 256 j, ...), in row order
        assert sb[pos[0]] == rp[r] and se[pos[-1]] == rp[r + 1]
        assert (sb[pos[1:]] == se[pos[:-1]]).all()
        assert ((se[pos] - sb[pos]) <= 256).all()
    if by_src:
        first = col.numpy()[sb[:nv]]
        assert (np.diff(first.astype(np.int64)) >= 0).all()
    rest = srow[nv:]
    assert sorted(rest.tolist()) == sorted(set(range(n)) - set(hub_rows.tolist()))
    assert (sb[nv:] == rp[rest]).all() and (se[nv:] == rp[rest + 1]).all()
    assert (np.diff(deg[rest]) <= 0).all()
    monkeypatch.undo()
    tuning.reload()


def test_hub_plan_without_col_keeps_hub_order():
    """The source order needs the CSR's col: without it the plan stays in hub order."""
    from atmlgraphattentionnetworks_amd.graph import hub_plan
    rowptr, order, col, _ = _csr(500, 3000, [(3, 2000)], seed=1)
    plan = hub_plan(rowptr, order, int(rowptr[-1]), seg_len=128)
    assert plan is not None and plan.seg_slot is None
