"""Synthetic stand-ins for the datasets the run scripts load.

There is no network, so PyG's ``Planetoid`` / ``Amazon`` / ``GNNBenchmarkDataset``
downloads (``run_inductive.py:43-54``, ``run_gnn_benchmark.py:35-37``) are
replaced by seeded graphs with the same node / edge / feature / class counts,
class-correlated features and homophilous edges (so training has a signal to
learn), and the same splits and transforms:

* Planetoid ``split="public"``: 20 training nodes per class, 500 validation,
  1000 test; ``NormalizeFeatures`` (row-normalise to sum 1) for Cora/Citeseer
  (``run_inductive.py:62-63``);
* Amazon: ``RandomNodeSplit("test_rest", num_val=0.1, num_train_per_class=20)``
  (``run_inductive.py:60-61``);
* CIFAR10 superpixels: graphs of 85-150 nodes, 8-NN edges over 2-D positions,
  3 colour features, 10 classes; a loader that collates ``batch_size`` graphs
  into one block-diagonal graph plus a ``batch`` vector (PyG ``DataLoader``,
  ``run_gnn_benchmark.py:38-40``).

Accuracies on these graphs say nothing about the real datasets; they exist so
the loops, the layer's training path and the checkpoints run end to end.
"""
from __future__ import annotations

from typing import Iterator, List, NamedTuple, Optional

import torch

from .gatnet import GraphData

__all__ = ["DATASET_SHAPES", "synthetic_node_dataset", "SyntheticGraph",
           "synthetic_cifar_graphs", "collate", "GraphLoader"]


class _Shape(NamedTuple):
    nodes: int
    edges: int  # directed edges (both directions of each undirected edge), as PyG stores them
    features: int
    classes: int
    split: str  # "public" | "random" | "none"
    normalize: bool


# PyG statistics of the datasets the scripts name (run_inductive.py:17)
DATASET_SHAPES = {
    "Cora": _Shape(2708, 10556, 1433, 7, "public", True),
    "Citeseer": _Shape(3327, 9104, 3703, 6, "public", True),
    "Pubmed": _Shape(19717, 88648, 500, 3, "public", False),
    "AmazonComp": _Shape(13752, 491722, 767, 10, "random", False),
    "AmazonPhotos": _Shape(7650, 238162, 745, 8, "random", False),
    # the PPI shape of BASELINE config 1 (44,906 nodes over the 24 PPI graphs)
    "PPI": _Shape(44906, 1226368, 50, 121, "random", False),
}


def _split_masks(y: torch.Tensor, classes: int, kind: str, g: torch.Generator):
    n = y.numel()
    perm = torch.randperm(n, generator=g)
    train = torch.zeros(n, dtype=torch.bool)
    for c in range(classes):
        idx = perm[y[perm] == c][:20]
        train[idx] = True
    rest = perm[~train[perm]]
    val = torch.zeros(n, dtype=torch.bool)
    test = torch.zeros(n, dtype=torch.bool)
    if kind == "public":  # 500 validation, 1000 test (fewer on a scaled-down graph)
        nv = min(500, rest.numel() // 3)
        val[rest[:nv]] = True
        test[rest[nv:nv + 1000]] = True
    else:  # RandomNodeSplit("test_rest", num_val=0.1)
        nv = int(round(0.1 * n))
        val[rest[:nv]] = True
        test[rest[nv:]] = True
    return train, val, test


def synthetic_node_dataset(name: str, seed: int = 0, homophily: float = 0.8,
                           scale: float = 1.0) -> GraphData:
    """One seeded graph with ``name``'s shape (``scale`` < 1 shrinks nodes and
    edges for quick tests).  Features: sparse binary bag-of-words with a
    class-specific block of more frequent words; edges: a fraction
    ``homophily`` within the class, both directions stored."""
    if name not in DATASET_SHAPES:
        raise ValueError(f"unknown dataset {name!r}; one of {sorted(DATASET_SHAPES)}")
    sh = DATASET_SHAPES[name]
    g = torch.Generator().manual_seed(seed)
    n = max(int(sh.nodes * scale), 20 * sh.classes + 50)
    half = max(int(sh.edges * scale) // 2, 1)
    fin, C = sh.features, sh.classes
    y = torch.randint(0, C, (n,), generator=g)
    # features: background rate + a class block
    block = max(fin // C, 1)
    x = (torch.rand(n, fin, generator=g) < 0.01).float()
    cols = (y.unsqueeze(1) * block + torch.randint(0, block, (n, 8), generator=g)) % fin
    x.scatter_(1, cols, 1.0)
    if sh.normalize:
        x = x / x.sum(1, keepdim=True).clamp(min=1.0)
    # homophilous undirected edges: pick a same-class partner with prob `homophily`
    src = torch.randint(0, n, (half,), generator=g)
    order = torch.argsort(y)
    counts = torch.bincount(y, minlength=C)
    starts = torch.cumsum(counts, 0) - counts
    same = torch.rand(half, generator=g) < homophily
    ys = y[src]
    pick = (torch.rand(half, generator=g) * counts[ys].clamp(min=1)).long()
    partner_same = order[starts[ys] + pick.clamp(max=counts[ys] - 1)]
    partner_any = torch.randint(0, n, (half,), generator=g)
    dst = torch.where(same, partner_same, partner_any)
    keep = src != dst
    src, dst = src[keep], dst[keep]
    edge_index = torch.stack([torch.cat([src, dst]), torch.cat([dst, src])])
    train, val, test = _split_masks(y, C, sh.split, g)
    return GraphData(x, edge_index, y, train, val, test)


class SyntheticGraph(NamedTuple):
    x: torch.Tensor  # [n, 3]
    edge_index: torch.Tensor  # [2, n*k]
    y: int


def synthetic_cifar_graphs(num_graphs: int, seed: int = 0, k: int = 8, nmin: int = 85,
                           nmax: int = 150) -> List[SyntheticGraph]:
    """CIFAR10-superpixel-shaped graphs (``GNNBenchmarkDataset('CIFAR10')``):
    n ~ U{85..150} nodes, 8-NN edges (source = neighbour, target = node), RGB
    features whose mean depends on the class."""
    g = torch.Generator().manual_seed(seed)
    centres = torch.rand(10, 3, generator=g)
    out = []
    for _ in range(num_graphs):
        n = int(torch.randint(nmin, nmax + 1, (1,), generator=g))
        label = int(torch.randint(0, 10, (1,), generator=g))
        pos = torch.rand(n, 2, generator=g)
        d = torch.cdist(pos, pos)
        d.fill_diagonal_(float("inf"))
        kk = min(k, n - 1)
        nbr = d.topk(kk, largest=False).indices
        dst = torch.arange(n).unsqueeze(1).expand(n, kk).reshape(-1)
        x = (centres[label] + 0.25 * torch.randn(n, 3, generator=g)).clamp(0, 1)
        out.append(SyntheticGraph(x, torch.stack([nbr.reshape(-1), dst]), label))
    return out


def collate(graphs: List[SyntheticGraph]) -> GraphData:
    """Block-diagonal batch (PyG ``Batch.from_data_list``): node ids offset per
    graph, ``batch[n]`` = graph of node n, ``y`` one label per graph."""
    xs, eis, batch, ys = [], [], [], []
    base = 0
    for gi, gr in enumerate(graphs):
        n = gr.x.size(0)
        xs.append(gr.x)
        eis.append(gr.edge_index + base)
        batch.append(torch.full((n,), gi, dtype=torch.int64))
        ys.append(gr.y)
        base += n
    return GraphData(torch.cat(xs), torch.cat(eis, 1), torch.tensor(ys, dtype=torch.int64),
                     batch=torch.cat(batch), num_graphs=len(graphs))


class GraphLoader:
    """``torch_geometric.loader.DataLoader`` over a list of graphs: batches of
    ``batch_size`` collated graphs, reshuffled each epoch when ``shuffle``."""

    def __init__(self, graphs: List[SyntheticGraph], batch_size: int, shuffle: bool = False,
                 seed: int = 0):
        self.graphs = graphs
        self.batch_size = batch_size
        self.shuffle = shuffle
        self._g = torch.Generator().manual_seed(seed)

    def __len__(self) -> int:
        return (len(self.graphs) + self.batch_size - 1) // self.batch_size

    def __iter__(self) -> Iterator[GraphData]:
        idx = (torch.randperm(len(self.graphs), generator=self._g).tolist() if self.shuffle
               else list(range(len(self.graphs))))
        for s in range(0, len(idx), self.batch_size):
            yield collate([self.graphs[i] for i in idx[s:s + self.batch_size]])
