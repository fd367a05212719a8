"""The reference's callers of the layer: ``GATNet`` (``GATNet.py:12-87``), the
activation/heads/params experiment models, a ``Data``-like container and the
graph-batch readout — so the run-script loops (``run.py``) drive the MI355X
layer exactly as the reference scripts drive ``GAT.py``.

Only ``model_name='GAT'`` is built: the reference's ``'GCN'`` branch uses PyG's
``GCNConv`` (``GATNet.py:39-58``), which is outside this hot path.
``'PPI'`` is an addition: the PPI-shape configuration BASELINE.json config 1
names, which the reference's ``GATNet`` lacks (SURVEY.md §8d note).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from .layer import GraphAttentionLayer, GraphAttentionLayerActivationTest

__all__ = ["GraphData", "GATNet", "GATModel", "GATActivationModel", "segment_mean",
           "GATNET_CONFIGS"]


class GraphData:
    """The fields of PyG's ``Data`` / ``Batch`` the scripts read (``x``,
    ``edge_index``, ``y``, the split masks, ``batch``), with ``.to(device)``."""

    _FIELDS = ("x", "edge_index", "y", "train_mask", "val_mask", "test_mask", "batch")

    def __init__(self, x, edge_index, y=None, train_mask=None, val_mask=None, test_mask=None,
                 batch=None, num_graphs: Optional[int] = None):
        self.x, self.edge_index, self.y = x, edge_index, y
        self.train_mask, self.val_mask, self.test_mask = train_mask, val_mask, test_mask
        self.batch = batch
        self.num_graphs = num_graphs

    @property
    def num_nodes(self) -> int:
        return int(self.x.size(0))

    @property
    def num_node_features(self) -> int:
        return int(self.x.size(1))

    def to(self, device) -> "GraphData":
        kw = {k: (v.to(device) if isinstance(v, torch.Tensor) else v)
              for k, v in ((f, getattr(self, f)) for f in self._FIELDS)}
        return GraphData(num_graphs=self.num_graphs, **kw)


def segment_mean(x: torch.Tensor, batch: torch.Tensor, num_segments: Optional[int] = None):
    """``torch_scatter.scatter_mean(x, batch, dim=0)`` (``GATNet.py:73``): the
    per-graph mean readout; empty segments give 0, as scatter_mean does."""
    if num_segments is None:
        num_segments = int(batch.max().item()) + 1 if batch.numel() else 0
    total = torch.zeros(num_segments, x.size(1), dtype=x.dtype, device=x.device)
    total = total.index_add(0, batch, x)
    count = torch.bincount(batch, minlength=num_segments).clamp_(min=1).to(x.dtype)
    return total / count.unsqueeze(1)


# dataset -> (conv1 kwargs after num_features, conv2 args), GATNet.py:17-37
GATNET_CONFIGS = {
    "CIFAR10": (dict(out=8, heads=8, concat=True, dropout=0.0),
                dict(inp=64, out=8, heads=8, concat=True, dropout=0.0)),
    "Cora": (dict(out=8, heads=8, concat=True, dropout=0.6),
             dict(inp=64, out=7, heads=1, concat=False, dropout=0.6)),
    "Citeseer": (dict(out=8, heads=8, concat=True, dropout=0.6),
                 dict(inp=64, out=6, heads=1, concat=False, dropout=0.6)),
    "Pubmed": (dict(out=8, heads=8, concat=True, dropout=0.6),
               dict(inp=64, out=3, heads=8, concat=False, dropout=0.6)),
    "AmazonComp": (dict(out=8, heads=8, concat=True, dropout=0.6),
                   dict(inp=64, out=10, heads=8, concat=False, dropout=0.6)),
    "AmazonPhotos": (dict(out=8, heads=8, concat=True, dropout=0.6),
                     dict(inp=64, out=8, heads=8, concat=False, dropout=0.6)),
    # PPI shape (BASELINE config 1): conv1 = the (4, 8) pair of run_heads_experiment.py:52
    "PPI": (dict(out=8, heads=4, concat=True, dropout=0.6),
            dict(inp=32, out=121, heads=1, concat=False, dropout=0.6)),
}


class GATNet(torch.nn.Module):
    """``GATNet.py:12`` with ``model_name='GAT'``: two attention layers;
    node classification: dropout 0.6 -> conv1 -> ELU -> dropout 0.6 -> conv2 ->
    log_softmax (``GATNet.py:77-87``); CIFAR10 graph classification: conv1 ->
    ELU -> conv2 -> ELU -> per-graph mean -> Linear+ReLU -> Linear ->
    log_softmax (``GATNet.py:61-76``)."""

    def __init__(self, model_name, dataset_name, num_features):
        super().__init__()
        self.dataset_name = dataset_name
        self.model_name = model_name
        if model_name != "GAT":
            raise NotImplementedError(
                f"model_name={model_name!r}: only 'GAT' runs on the MI355X layer (the "
                "reference's 'GCN' branch uses PyG GCNConv, outside this build)")
        if dataset_name not in GATNET_CONFIGS:
            raise ValueError(f"unknown dataset_name {dataset_name!r}; one of "
                             f"{sorted(GATNET_CONFIGS)}")
        c1, c2 = GATNET_CONFIGS[dataset_name]
        self.conv1 = GraphAttentionLayer(num_features, c1["out"], num_heads=c1["heads"],
                                         concat=c1["concat"], dropout=c1["dropout"])
        self.conv2 = GraphAttentionLayer(c2["inp"], c2["out"], num_heads=c2["heads"],
                                         concat=c2["concat"], dropout=c2["dropout"])
        if dataset_name == "CIFAR10":
            self.lin1 = torch.nn.Linear(64, 64)
            self.lin2 = torch.nn.Linear(64, 10)

    def forward(self, data):
        x, edge_index = data.x, data.edge_index
        if self.dataset_name == "CIFAR10":
            x = F.elu(self.conv1(x, edge_index))
            x = F.elu(self.conv2(x, edge_index))
            x = segment_mean(x, data.batch, getattr(data, "num_graphs", None))
            x = F.relu(self.lin1(x))
            return F.log_softmax(self.lin2(x), dim=1)
        x = F.dropout(x, p=0.6, training=self.training)
        x = F.elu(self.conv1(x, edge_index))
        x = F.dropout(x, p=0.6, training=self.training)
        x = self.conv2(x, edge_index)
        return F.log_softmax(x, dim=1)


class GATModel(torch.nn.Module):
    """The heads / hidden-size experiment model (``run_heads_experiment.py:16-31``,
    ``run_params_experiment.py:14-29``)."""

    def __init__(self, num_input_features, num_output_features, num_heads, num_classes):
        super().__init__()
        self.conv1 = GraphAttentionLayer(num_input_features, num_output_features,
                                         num_heads=num_heads, concat=True)
        self.conv2 = GraphAttentionLayer(num_output_features * num_heads, num_classes,
                                         num_heads=1)

    def forward(self, data):
        x, edge_index = data.x, data.edge_index
        x = F.dropout(x, p=0.6, training=self.training)
        x = F.elu(self.conv1(x, edge_index))
        x = F.dropout(x, p=0.6, training=self.training)
        x = self.conv2(x, edge_index)
        return F.log_softmax(x, dim=1)


class GATActivationModel(torch.nn.Module):
    """The activation experiment model (``run_act_func_experiment.py:76-93``)."""

    def __init__(self, num_input_features, num_output_features, num_heads, num_classes,
                 activation_function=None):
        super().__init__()
        if activation_function is None:
            activation_function = torch.nn.LeakyReLU(negative_slope=0.2)
        self.conv1 = GraphAttentionLayerActivationTest(
            num_input_features, num_output_features, num_heads=num_heads, concat=True,
            activation_function=activation_function)
        self.conv2 = GraphAttentionLayerActivationTest(
            num_output_features * num_heads, num_classes, num_heads=1,
            activation_function=activation_function)

    def forward(self, data):
        x, edge_index = data.x, data.edge_index
        x = F.dropout(x, p=0.6, training=self.training)
        x = F.elu(self.conv1(x, edge_index))
        x = F.dropout(x, p=0.6, training=self.training)
        x = self.conv2(x, edge_index)
        return F.log_softmax(x, dim=1)
