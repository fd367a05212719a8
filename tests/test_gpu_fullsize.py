"""Parity at BASELINE.json's full sizes.

PPI-shape is checked in full in test_gpu_parity.py.  Here: arxiv-scale and the
CIFAR10 superpixel batch in full against the oracle, and Reddit-scale
(N=232,965, E=114,615,892, Fin=602) by sampled rows: the oracle evaluates the
complete in-edge sets of 4,096 random targets plus the 16 longest rows
(gat_layer_forward_rows, in batches of 1,024 rows), which gives those rows'
exact reference outputs without materialising the 29 GB [E', H, F] message
tensor on the host.
"""
import pytest
import torch

from oracle import gat_layer_forward_from_state, gat_layer_forward_rows, init_reference_params

pytestmark = pytest.mark.gpu

ATOL = RTOL = 1e-5


def _layer(w, dev, state):
    from atmlgraphattentionnetworks_amd import GraphAttentionLayer
    layer = GraphAttentionLayer(w.in_channels, w.out_channels, num_heads=w.heads, concat=w.concat)
    layer.load_state_dict(state)
    return layer.to(dev).eval()


@pytest.mark.parametrize("name", ["arxiv", "cifar", "cifar_h8", "ppi_h4"])
def test_full_workload_vs_oracle(name):
    from atmlgraphattentionnetworks_amd.synthetic import WORKLOADS, make_inputs
    dev = torch.device("cuda", 0)
    w = WORKLOADS[name]
    x, ei = make_inputs(w, dev)
    state = init_reference_params(w.in_channels, w.out_channels, w.heads, w.concat, seed=0)
    with torch.no_grad():
        out = _layer(w, dev, state)(x, ei).cpu()
    ref = gat_layer_forward_from_state(state, x.cpu(), ei.cpu(), w.heads, w.concat)
    torch.testing.assert_close(out, ref, atol=ATOL, rtol=RTOL)


def test_reddit_scale_sampled_rows():
    from atmlgraphattentionnetworks_amd.synthetic import WORKLOADS, make_inputs
    dev = torch.device("cuda", 0)
    w = WORKLOADS["reddit"]
    x, ei = make_inputs(w, dev)
    state = init_reference_params(w.in_channels, w.out_channels, w.heads, w.concat, seed=0)
    with torch.no_grad():
        out = _layer(w, dev, state)(x, ei)
    from atmlgraphattentionnetworks_amd import get_csr
    csr = get_csr(ei, x.size(0))
    g = torch.Generator(device="cpu")
    g.manual_seed(123)
    rows = torch.cat([torch.randperm(x.size(0), generator=g)[:4096].to(dev),
                      csr.order[:16].long()]).unique()
    assert rows.numel() >= 4096
    ref = gat_layer_forward_rows(state, x.cpu(), ei.cpu(), rows.cpu(), w.heads, w.concat)
    torch.testing.assert_close(out[rows].cpu(), ref, atol=ATOL, rtol=RTOL)


def test_backward_paths_agree_at_arxiv_scale(monkeypatch):
    """Two independent backward implementations — recompute (gat_bwd_targets +
    gat_bwd_sources) and stored coefficients (gat_edge_backward_rows +
    gat_src_backward) — agree on every gradient at ogbn-arxiv scale (1.34M
    edges), with attention dropout on (size-independent property: the oracle's
    float64 autograd at this size would take minutes)."""
    import torch
    from atmlgraphattentionnetworks_amd import GraphAttentionLayer
    from atmlgraphattentionnetworks_amd.graph import get_csr
    from atmlgraphattentionnetworks_amd.synthetic import WORKLOADS, make_inputs
    from atmlgraphattentionnetworks_amd.training import gat_train_forward
    w = WORKLOADS["arxiv"]
    dev = torch.device("cuda", 0)
    x, ei = make_inputs(w, dev)
    torch.manual_seed(0)
    layer = GraphAttentionLayer(w.in_channels, w.out_channels, num_heads=w.heads,
                                concat=w.concat).to(dev)
    csr = get_csr(ei, x.size(0))
    gout = torch.randn(x.size(0), w.heads * w.out_channels, device=dev)
    grads = []
    for path in (None, "stored"):
        if path:
            monkeypatch.setenv("GAT_BWD_KERNEL", path)
        else:
            monkeypatch.delenv("GAT_BWD_KERNEL", raising=False)
        layer.zero_grad()
        xg = x.clone().requires_grad_(True)
        (gat_train_forward(layer, xg, csr, 0.6, 1234) * gout).sum().backward()
        grads.append([xg.grad] + [p.grad.clone() for p in layer.parameters()])
    names = ["x"] + [n for n, _ in layer.named_parameters()]
    for name, a, b in zip(names, *grads):
        scale = float(b.abs().max()) + 1e-30
        if name == "x":
            # LeakyReLU' jumps at z = 0: the recompute path scores an edge from the
            # Wh row it gathers (log2 units), the stored path from the projection's
            # s_src, and over 10.7M (edge, head) scores a few lie within that
            # rounding difference of 0, so their dz differs by the slope ratio.
            # That touches a handful of source rows of dx; everywhere else the
            # two paths agree to 1e-4.
            bad = ((a - b).abs() > 1e-4 * scale).any(dim=1)
            assert int(bad.sum()) <= 16, (name, int(bad.sum()))
            continue
        err = float((a - b).abs().max()) / scale
        # parameter gradients sum over all edges, the few kink edges included
        # (tools/kink_probe.py: 1-3 of the 10.7M scores lie within 1e-6 of 0,
        # depending on the projection's rounding), so they carry the same
        # ambiguity, diluted: 2e-4 of max |grad| measured, against O(1) for a
        # wrong gradient
        tol = 1e-3
        assert err < tol, (name, err)
