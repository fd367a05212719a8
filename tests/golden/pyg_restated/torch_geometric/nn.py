"""Restated ``torch_geometric.nn.MessagePassing`` (PyG 2.0.x): the parts
GAT.py uses — ``__collect__`` lifting for ``_i``/``_j`` arguments (tuple element
0 -> ``_j``, element 1 -> ``_i``), ``index``, and ``aggr='add'`` aggregation
into ``dim_size = size[i]``."""
import inspect

import torch

from .utils import _scatter


class MessagePassing(torch.nn.Module):
    def __init__(self, aggr="add", flow="source_to_target", node_dim=-2):
        super().__init__()
        self.aggr = aggr
        self.flow = flow
        self.node_dim = node_dim
        self._msg_args = list(inspect.signature(self.message).parameters)

    def propagate(self, edge_index, size=None, **kwargs):
        i, j = (1, 0) if self.flow == "source_to_target" else (0, 1)
        size = [None, None]
        args = {}
        for arg in self._msg_args:
            if arg[-2:] in ("_i", "_j"):
                dim = 0 if arg[-2:] == "_j" else 1
                data = kwargs[arg[:-2]]
                if isinstance(data, (tuple, list)):
                    other = data[1 - dim]
                    if isinstance(other, torch.Tensor):
                        size[1 - dim] = other.size(self.node_dim)
                    data = data[dim]
                size[dim] = data.size(self.node_dim)
                args[arg] = data.index_select(self.node_dim, edge_index[j if dim == 0 else i])
            elif arg == "index":
                args[arg] = edge_index[i]
            else:
                args[arg] = kwargs.get(arg)
        out = self.message(**args)
        dim_size = size[i] if size[i] is not None else size[j]
        assert self.aggr == "add"
        return _scatter(out, edge_index[i], self.node_dim, dim_size, "sum")

    def message(self, x_j):
        return x_j
