"""Seeded synthetic graphs of the shapes BASELINE.json names.

The reference trains on PyG datasets (Planetoid, Amazon, PPI, CIFAR10
superpixels) that need network access; these generators reproduce their
SHAPES only:

* ``uniform``: dst ~ U[0, N), src = (dst + 1 + U[0, N-1)) mod N — no
  self-loops in the input, multi-edges allowed (PPI-, arxiv-, Reddit-shape).
* ``powerlaw``: the degree-skew stress variant SURVEY.md §8d names for the
  Reddit shape: dst drawn with P(node of rank i) ~ (i + 1)^-0.5 over a seeded
  random ranking of the nodes, src uniform over the other nodes.  At Reddit's
  N and E the in-degrees run from ~250 to ~119k (mean 493).
* ``knn_batch``: ``run_gnn_benchmark.py``'s CIFAR10 superpixel batches —
  ``graphs`` graphs of n_g ~ U{85..150} nodes, pos ~ U[0,1)^2, 8-NN edges
  inside each graph (j -> i for the 8 nearest j of i), block-diagonal.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch


@dataclass(frozen=True)
class Workload:
    name: str
    kind: str  # "uniform" | "knn_batch"
    num_nodes: int
    num_edges: int  # input edges (before self-loops); knn_batch: graphs
    in_channels: int
    heads: int
    out_channels: int
    concat: bool = True


# BASELINE.json "configs", by index (0 is the reference's CPU plumbing case)
WORKLOADS = {
    "ppi": Workload("ppi", "uniform", 44_906, 1_226_368, 50, 8, 8, True),
    "ppi_h4": Workload("ppi_h4", "uniform", 44_906, 1_226_368, 50, 4, 8, True),
    "cifar": Workload("cifar", "knn_batch", 0, 512, 3, 4, 8, True),
    "cifar_h8": Workload("cifar_h8", "knn_batch", 0, 512, 3, 8, 8, True),
    "arxiv": Workload("arxiv", "uniform", 169_343, 1_166_243, 128, 8, 8, True),
    "reddit": Workload("reddit", "uniform", 232_965, 114_615_892, 602, 8, 8, True),
    "reddit_powerlaw": Workload("reddit_powerlaw", "powerlaw", 232_965, 114_615_892, 602, 8, 8,
                                True),
}


def uniform_graph(num_nodes: int, num_edges: int, seed: int = 2,
                  device: Optional[torch.device] = None) -> torch.Tensor:
    """edge_index [2, E] int64; generated in chunks to bound peak memory."""
    device = torch.device(device) if device is not None else torch.device("cpu")
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    out = torch.empty(2, num_edges, dtype=torch.int64, device=device)
    chunk = 1 << 24
    for s in range(0, num_edges, chunk):
        e = min(num_edges, s + chunk)
        dst = torch.randint(0, num_nodes, (e - s,), generator=g, device=device)
        off = torch.randint(0, max(num_nodes - 1, 1), (e - s,), generator=g, device=device)
        out[1, s:e] = dst
        out[0, s:e] = (dst + 1 + off) % num_nodes
    return out


def powerlaw_graph(num_nodes: int, num_edges: int, seed: int = 2, alpha: float = 0.5,
                   device: Optional[torch.device] = None) -> torch.Tensor:
    """edge_index [2, E] int64 with power-law in-degrees: target rank i drawn
    with probability ~ (i + 1)^-alpha (inverse-CDF sampling), ranks mapped to
    node ids by a seeded permutation; sources uniform, no self-loops."""
    device = torch.device(device) if device is not None else torch.device("cpu")
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    w = torch.arange(1, num_nodes + 1, dtype=torch.float64, device=device).pow(-alpha)
    cdf = w.cumsum(0)
    cdf /= cdf[-1].clone()
    perm = torch.randperm(num_nodes, generator=g, device=device)
    out = torch.empty(2, num_edges, dtype=torch.int64, device=device)
    chunk = 1 << 24
    for s in range(0, num_edges, chunk):
        e = min(num_edges, s + chunk)
        u = torch.rand(e - s, generator=g, dtype=torch.float64, device=device)
        rank = torch.searchsorted(cdf, u).clamp_(max=num_nodes - 1)
        dst = perm[rank]
        off = torch.randint(0, max(num_nodes - 1, 1), (e - s,), generator=g, device=device)
        out[1, s:e] = dst
        out[0, s:e] = (dst + 1 + off) % num_nodes
    return out


def knn_batch(graphs: int = 512, k: int = 8, seed: int = 3, nmin: int = 85, nmax: int = 150,
              device: Optional[torch.device] = None):
    """(edge_index [2, E] int64, batch [N] int64, num_nodes)."""
    device = torch.device(device) if device is not None else torch.device("cpu")
    g = torch.Generator(device="cpu")
    g.manual_seed(seed)
    sizes = torch.randint(nmin, nmax + 1, (graphs,), generator=g)
    srcs, dsts, batch = [], [], []
    base = 0
    for gi, n in enumerate(sizes.tolist()):
        pos = torch.rand(n, 2, generator=g)
        d = torch.cdist(pos, pos)
        d.fill_diagonal_(float("inf"))
        kk = min(k, n - 1)
        nbr = d.topk(kk, largest=False).indices  # [n, kk]
        dsts.append((torch.arange(n).unsqueeze(1).expand(n, kk) + base).reshape(-1))
        srcs.append((nbr + base).reshape(-1))
        batch.append(torch.full((n,), gi, dtype=torch.int64))
        base += n
    ei = torch.stack([torch.cat(srcs), torch.cat(dsts)]).to(device)
    return ei, torch.cat(batch).to(device), base


def make_inputs(w: Workload, device, x_seed: int = 1, edge_seed: int = 2):
    """(x [N, Fin] f32, edge_index [2, E] i64) for a workload."""
    device = torch.device(device)
    if w.kind in ("uniform", "powerlaw"):
        n = w.num_nodes
        gen = uniform_graph if w.kind == "uniform" else powerlaw_graph
        ei = gen(n, w.num_edges, seed=edge_seed, device=device)
        g = torch.Generator(device=device)
        g.manual_seed(x_seed)
        x = torch.randn(n, w.in_channels, generator=g, device=device)
    elif w.kind == "knn_batch":
        ei, _, n = knn_batch(w.num_edges, device=device)
        g = torch.Generator(device=device)
        g.manual_seed(x_seed)
        x = torch.rand(n, w.in_channels, generator=g, device=device)
    else:
        raise ValueError(w.kind)
    return x, ei
