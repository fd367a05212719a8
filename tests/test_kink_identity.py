"""The identity behind the backward's edge-free pass 1 ("kink
sums"), checked in float64 on the CPU with autograd as the judge.

For one layer (GAT.py:53-67 with PyG's segmented softmax, GAT.py:60, and
attention dropout, GAT.py:61), target i and head h, with z_ij = s_dst[i] +
s_src[j], alpha = segment softmax of LeakyReLU(z), A = drop * alpha and
y_i = sum_j A_ij Wh_j:

    dL/ds_dst[i] = dy_i . Q_i - delta_i R_i,   delta_i = dy_i . y_i,
    Q_i = sum_j A_ij L'(z_ij) Wh_j,  R_i = sum_j alpha_ij L'(z_ij),

L' = 1 for z > 0, else the slope.  gat_edge_aggregate_train accumulates Q and
R in the forward and gat_bwd_table evaluates the right-hand side; here the
left-hand side comes from autograd through oracle.segment_softmax.
"""
import pytest
import torch

from oracle import segment_softmax


@pytest.mark.parametrize("slope", [0.2, 0.0, 1.0])
@pytest.mark.parametrize("p", [0.0, 0.5])
def test_ds_dst_equals_kink_sums(slope, p):
    g = torch.Generator().manual_seed(3)
    n, e, H, F = 40, 300, 4, 3
    src = torch.randint(0, n, (e,), generator=g)
    dst = torch.randint(0, n, (e,), generator=g)
    loops = torch.arange(n)
    src, dst = torch.cat([src, loops]), torch.cat([dst, loops])  # add_self_loops (GAT.py:38)
    wh = torch.randn(n, H, F, generator=g, dtype=torch.float64)
    s_src = torch.randn(n, H, generator=g, dtype=torch.float64)
    s_dst = torch.randn(n, H, generator=g, dtype=torch.float64).requires_grad_(True)
    keep = (torch.rand(src.numel(), H, generator=g) >= p).to(torch.float64)
    drop = keep / (1 - p)
    dy = torch.randn(n, H, F, generator=g, dtype=torch.float64)

    z = s_dst[dst] + s_src[src]
    e_ = torch.where(z > 0, z, slope * z)
    alpha = segment_softmax(e_, dst, n)
    a = alpha * drop
    y = torch.zeros(n, H, F, dtype=torch.float64).index_add_(0, dst, a.unsqueeze(-1) * wh[src])
    (y * dy).sum().backward()
    lhs = s_dst.grad

    with torch.no_grad():
        lk = torch.where(z > 0, torch.ones_like(z), torch.full_like(z, slope))
        q = torch.zeros(n, H, F, dtype=torch.float64).index_add_(
            0, dst, (a * lk).unsqueeze(-1) * wh[src])
        r = torch.zeros(n, H, dtype=torch.float64).index_add_(0, dst, alpha * lk)
        delta = (dy * y).sum(-1)
        rhs = (dy * q).sum(-1) - delta * r
    torch.testing.assert_close(rhs, lhs, rtol=1e-10, atol=1e-12)
