"""Restated ``torch_geometric.utils.add_self_loops`` and ``softmax`` (PyG 2.0.x)."""
import torch


def _scatter(src, index, dim, dim_size, reduce):
    # torch_scatter.scatter semantics for a 1-D index broadcast along ``dim``.
    shape = list(src.shape)
    shape[dim] = dim_size
    view = [1] * src.dim()
    view[dim] = -1
    idx = index.view(view).expand_as(src)
    if reduce == "sum":
        return torch.zeros(shape, dtype=src.dtype).scatter_add_(dim, idx, src)
    if reduce == "max":
        out = torch.zeros(shape, dtype=src.dtype)
        return out.scatter_reduce(dim, idx, src, reduce="amax", include_self=False)
    raise ValueError(reduce)


def add_self_loops(edge_index, edge_attr=None, fill_value=None, num_nodes=None):
    n = int(edge_index.max()) + 1 if num_nodes is None else num_nodes
    loop_index = torch.arange(0, n, dtype=torch.long, device=edge_index.device)
    loop_index = loop_index.unsqueeze(0).repeat(2, 1)
    # fill_value only affects edge_attr, which is None at GAT.py:38.
    return torch.cat([edge_index, loop_index], dim=1), edge_attr


def softmax(src, index=None, ptr=None, num_nodes=None, dim=0):
    n = int(index.max()) + 1 if num_nodes is None else num_nodes
    src_max = _scatter(src, index, dim, n, "max").index_select(dim, index)
    out = (src - src_max).exp()
    out_sum = _scatter(out, index, dim, n, "sum").index_select(dim, index)
    return out / (out_sum + 1e-16)
