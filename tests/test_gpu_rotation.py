"""Staggered sweeps (graph.build_sched_csr(stagger=True), graph.rotated_col,
graph.rotate_csc): the eval forward and the training backward walk each row's
in-edges (the backward: each source's out-edges) from a position-dependent
start and wrap around.  Same edges, another summation order: outputs and
gradients agree with the unrotated walk (GAT_EDGE_SCHED=plain) to fp32
rounding and meet the oracle at the parity bar (GAT.py:53-67)."""
import numpy as np
import pytest
import torch

from oracle import gat_layer_forward_from_state, init_reference_params

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _graph(n, e, seed):
    rng = np.random.default_rng(seed)
    return torch.from_numpy(rng.integers(0, n, size=(2, e)).astype(np.int64))


@pytest.mark.parametrize("shape", [(2000, 60000, 8, 8), (600, 60000, 8, 8), (600, 60000, 4, 16)],
                         ids=["short_rows_sched", "long_rows_rotated", "long_rows_h4f16"])
def test_eval_forward_rotated_equals_plain(shape, monkeypatch):
    from atmlgraphattentionnetworks_amd import GraphAttentionLayer
    from atmlgraphattentionnetworks_amd.graph import SCHED_MAX_EPR, get_csr, rotated_col
    n, e, heads, f = shape
    fin = 24
    state = init_reference_params(fin, f, heads, True, seed=3)
    x = torch.randn(n, fin, generator=torch.Generator().manual_seed(4))
    ei = _graph(n, e, 5)
    outs = {}
    for mode in ("default", "plain"):
        if mode == "plain":
            monkeypatch.setenv("GAT_EDGE_SCHED", "plain")
        layer = GraphAttentionLayer(fin, f, num_heads=heads, concat=True)
        layer.load_state_dict(state)
        layer = layer.to(DEV).eval()
        eid = ei.to(DEV)
        if mode == "default" and e // n >= SCHED_MAX_EPR:
            csr = get_csr(eid, n)
            assert not torch.equal(rotated_col(csr), csr.col)  # the rotated walk is taken
        with torch.no_grad():
            outs[mode] = layer(x.to(DEV), eid).cpu()
    ref = gat_layer_forward_from_state(state, x, ei, heads, True)
    torch.testing.assert_close(outs["default"], ref, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(outs["default"], outs["plain"], atol=2e-6, rtol=1e-5)


def test_training_backward_rotated_csc_equals_plain(monkeypatch):
    """Long rows: the source pass over the rotated CSC gives the gradients the
    unrotated CSC gives (dropout 0: the same coefficients either way)."""
    from atmlgraphattentionnetworks_amd import GraphAttentionLayer
    n, e, fin, heads, f = 500, 50000, 20, 8, 8
    state = init_reference_params(fin, f, heads, True, seed=7)
    x = torch.randn(n, fin, generator=torch.Generator().manual_seed(8))
    gout = torch.randn(n, heads * f, generator=torch.Generator().manual_seed(9))
    ei = _graph(n, e, 10)
    res = {}
    for mode in ("default", "plain"):
        if mode == "plain":
            monkeypatch.setenv("GAT_EDGE_SCHED", "plain")
        layer = GraphAttentionLayer(fin, f, num_heads=heads, concat=True, dropout=0.0)
        layer.load_state_dict(state)
        layer = layer.to(DEV).train()
        xd = x.to(DEV).requires_grad_(True)
        out = layer(xd, ei.to(DEV))
        (out * gout.to(DEV)).sum().backward()
        res[mode] = [xd.grad.cpu()] + [p.grad.cpu() for p in layer.parameters()]
    for a, b in zip(res["default"], res["plain"]):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5 * float(b.abs().max()) + 1e-7)
