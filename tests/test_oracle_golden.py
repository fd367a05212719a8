"""The oracle (oracle/gat_oracle.py) against the golden vectors produced by
the reference's own GAT.py (tests/golden/make_golden.py), and against the
float64 closed form on the known-answer graphs.  CPU only."""
import pytest
import torch

from conftest import golden_names, load_golden
from oracle import closed_form_forward, gat_layer_forward_from_state, init_reference_params


@pytest.mark.parametrize("name", golden_names())
def test_oracle_matches_reference_fixture(name):
    g = load_golden(name)
    m = g["meta"]
    out = gat_layer_forward_from_state(g["state"], g["x"], g["edge_index"], m["H"], m["concat"])
    assert out.shape == g["out"].shape
    # same op sequence on the same CPU -> bit-identical
    assert torch.equal(out, g["out"])


@pytest.mark.parametrize("name", [n for n in golden_names() if n.startswith("kat_")])
def test_known_answer_closed_form(name):
    g = load_golden(name)
    m = g["meta"]
    cf = closed_form_forward(g["state"], g["x"], g["edge_index"], m["H"], m["concat"])
    torch.testing.assert_close(g["out"].double(), cf, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("name", golden_names())
def test_reference_init_order(name):
    """init_reference_params reproduces the reference constructor's RNG order."""
    g = load_golden(name)
    m = g["meta"]
    st = init_reference_params(m["Fin"], m["F"], m["H"], m["concat"], seed=m["seed"])
    assert list(st.keys()) == list(g["state"].keys())
    for k in st:
        assert torch.equal(st[k], g["state"][k]), k


def test_src_dst_convention():
    """attentions1 is the SOURCE term, attentions2 the TARGET term: swapping
    them changes the result on an asymmetric graph."""
    g = load_golden("kat_asym3")
    m = g["meta"]
    st = dict(g["state"])
    for h in range(m["H"]):
        st[f"attentions1.{h}.weight"], st[f"attentions2.{h}.weight"] = (
            st[f"attentions2.{h}.weight"], st[f"attentions1.{h}.weight"])
        st[f"attentions1.{h}.bias"], st[f"attentions2.{h}.bias"] = (
            st[f"attentions2.{h}.bias"], st[f"attentions1.{h}.bias"])
    swapped = gat_layer_forward_from_state(st, g["x"], g["edge_index"], m["H"], m["concat"])
    assert not torch.allclose(swapped, g["out"], atol=1e-4)


def test_differentiable_oracle_matches_fixture_and_has_grads():
    """gat_layer_forward_differentiable (the gradient oracle) equals the
    fixture-pinned forward, and autograd reaches every parameter."""
    import torch
    from oracle import gat_layer_forward_differentiable
    g = load_golden("grid_h4_f8_cat")
    meta = g["meta"]
    params = {k: v.double().requires_grad_(True) for k, v in g["state"].items()}
    out = gat_layer_forward_differentiable(params, g["x"].double(), g["edge_index"],
                                           meta["H"], meta["concat"])
    assert torch.allclose(out.float(), g["out"], atol=1e-5, rtol=0)
    out.sum().backward()
    assert all(p.grad is not None for p in params.values())


def test_dropout_mask_restatement_properties():
    import numpy as np
    from oracle import csr_positions, dropout_factors
    m = dropout_factors(np.arange(200000), 8, 0.6, 7)
    assert abs((m > 0).mean() - 0.4) < 0.005
    assert np.allclose(m[m > 0], 2.5)
    assert (dropout_factors(np.arange(1000), 4, 0.0, 7) == 1.0).all()
    assert (dropout_factors(np.arange(1000), 4, 1.0, 7) == 0.0).all()
    # different seeds and heads decorrelate
    m2 = dropout_factors(np.arange(200000), 8, 0.6, 8)
    assert abs(((m > 0) == (m2 > 0)).mean() - 0.52) < 0.01
    # CSR positions: by (target, source), equal pairs in input order
    import torch
    ei = torch.tensor([[1, 2, 0], [1, 0, 1]])
    # edges (src->dst): 1->1, 2->0, 0->1, loops 0->0, 1->1, 2->2
    # rows: 0: [0->0 (loop), 2->0]; 1: [0->1, 1->1 (input), 1->1 (loop)]; 2: [2->2]
    assert csr_positions(ei, 3).tolist() == [3, 1, 2, 0, 4, 5]


@pytest.mark.parametrize("concat,H", [(True, 8), (False, 4)])
def test_oracle_rows_equals_full_forward(concat, H):
    """gat_layer_forward_rows (the sampled-row oracle the Reddit-scale GPU
    tests use) gives exactly the full oracle's rows: same projection, and each
    row's in-edges in the same order with its self-loop last."""
    from oracle import gat_layer_forward_from_state, gat_layer_forward_rows, init_reference_params
    g = torch.Generator().manual_seed(3)
    n, e = 900, 20000
    ei = torch.stack([torch.randint(0, n, (e,), generator=g), torch.randint(0, n, (e,), generator=g)])
    ei[:, :50] = torch.tensor([[5] * 50, [5] * 50])  # pre-existing loops and multi-edges
    x = torch.randn(n, 20, generator=g)
    state = init_reference_params(20, 8, H, concat, seed=1)
    state["bias"] = torch.randn(state["bias"].shape, generator=g)
    full = gat_layer_forward_from_state(state, x, ei, H, concat)
    rows = torch.cat([torch.tensor([5, 0, n - 1, 5]), torch.randperm(n, generator=g)[:300]])
    part = gat_layer_forward_rows(state, x, ei, rows, H, concat, batch=128)
    torch.testing.assert_close(part, full[rows], atol=0, rtol=0)
