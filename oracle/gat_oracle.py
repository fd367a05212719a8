"""CPU oracle for the GAT attention-layer forward — TEST INFRASTRUCTURE ONLY.

This module is a checker, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` may
import it; the product path (``atmlgraphattentionnetworks_amd``) never does and
fails loudly when its HIP library is missing.

What it restates
----------------
The forward of ``GraphAttentionLayer`` in the reference
(``/root/reference/GAT.py:37-67``), op for op, on CPU PyTorch:

* ``GAT.py:38``  ``torch_geometric.utils.add_self_loops`` (PyG 2.0.x, not
  vendored in the reference, restated in :func:`add_self_loops`): appends the
  ``N`` loops ``(n, n)`` at the END of ``edge_index``; existing self-loops and
  multi-edges are kept; ``fill_value`` only touches ``edge_attr`` (None here).
* ``GAT.py:42-52`` the per-head ``Linear`` loop, ``stack``/``transpose`` and the
  attention ``Linear`` terms (``attentions1`` = source term,
  ``attentions2`` = target term).
* ``GAT.py:53`` PyG ``MessagePassing.propagate`` with ``aggr='add'``,
  ``node_dim=0``, ``flow='source_to_target'`` (restated in :func:`propagate`):
  ``x_j``/``*_j`` are lifted with ``edge_index[0]``, ``*_i`` with
  ``edge_index[1]``; for the tuple argument ``attention_vals=(a1, a2)`` element
  0 feeds ``_j`` and element 1 feeds ``_i``; messages are summed into the
  target with ``dim_size = N``.
* ``GAT.py:56-67`` ``message``: ``LeakyReLU_0.2(a_i + a_j)``, PyG
  ``utils.softmax`` (restated in :func:`segment_softmax`: scatter-max, gather,
  ``exp``, scatter-sum, gather, divide by ``sum + 1e-16``), dropout (identity
  in eval), ``x_j * alpha``, then head-major reshape (concat) or head mean.
* ``GAT.py:54`` ``+ self.bias``.

Pinning
-------
The reference cannot run unchanged here (``torch_geometric`` is not installed).
``tests/golden/make_golden.py`` runs the reference's own ``GAT.py`` with the
three PyG entry points restated in ``tests/golden/pyg_restated`` and commits its
outputs as fixtures; ``tests/test_oracle_golden.py`` checks this oracle against
them, and its ``test_known_answer_closed_form`` checks both against a float64
pure-Python closed form on the hand-checkable graphs.  The PyG semantics themselves are restated, not run: see
DESIGN.md "Oracle and parity".
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Sequence

import torch

__all__ = [
    "add_self_loops",
    "segment_softmax",
    "propagate",
    "gat_layer_forward",
    "gat_layer_forward_from_state",
    "gat_layer_forward_rows",
    "closed_form_forward",
    "init_reference_params",
    "gat_layer_forward_differentiable",
    "dropout_factors",
    "csr_positions",
]


def add_self_loops(edge_index: torch.Tensor, num_nodes: int) -> torch.Tensor:
    """PyG 2.0.x ``utils.add_self_loops`` as called at ``GAT.py:38``.

    ``cat([edge_index, arange(N).repeat(2, 1)], dim=1)`` — loops appended at
    the end, duplicates kept.
    """
    loop = torch.arange(num_nodes, dtype=torch.long, device=edge_index.device)
    loop = loop.unsqueeze(0).repeat(2, 1)
    return torch.cat([edge_index, loop], dim=1)


def segment_softmax(src: torch.Tensor, index: torch.Tensor, num_nodes: int) -> torch.Tensor:
    """PyG 2.0.x ``utils.softmax(src, index)`` as called at ``GAT.py:60``.

    Per target ``index[k]`` and head: ``exp(src - max) / (sum exp + 1e-16)``.
    """
    idx = index.view(-1, *([1] * (src.dim() - 1))).expand_as(src)
    src_max = torch.full((num_nodes,) + tuple(src.shape[1:]), float("-inf"), dtype=src.dtype)
    src_max = src_max.scatter_reduce(0, idx, src, reduce="amax", include_self=False)
    out = (src - src_max.index_select(0, index)).exp()
    out_sum = torch.zeros((num_nodes,) + tuple(src.shape[1:]), dtype=src.dtype)
    out_sum = out_sum.scatter_add(0, idx, out)
    return out / (out_sum.index_select(0, index) + 1e-16)


def propagate(edge_index: torch.Tensor, x: torch.Tensor, attention_vals, num_nodes: int,
              concat: bool, negative_slope: float = 0.2,
              drop: Optional[torch.Tensor] = None, activation=None) -> torch.Tensor:
    """PyG ``MessagePassing.propagate`` (``aggr='add'``, ``node_dim=0``) around
    ``GAT.py:56-67``'s ``message``.  ``drop`` ([E, H] multipliers, 0 or
    1/(1-p)) applies ``GAT.py:61``'s training-mode dropout with a given mask;
    None is eval mode.  ``activation`` replaces ``LeakyReLU(negative_slope)``
    as the score activation module (``run_act_func_experiment.py:38,58``)."""
    src, dst = edge_index[0], edge_index[1]
    # __collect__: _j lifts with edge_index[0] and takes tuple element 0,
    #              _i lifts with edge_index[1] and takes tuple element 1.
    x_j = x.index_select(0, src)
    att_j = attention_vals[0].index_select(0, src)
    att_i = attention_vals[1].index_select(0, dst)
    # message (GAT.py:57-66)
    e = att_i + att_j
    if activation is None:
        e = torch.nn.functional.leaky_relu(e, negative_slope)
    else:
        e = activation(e)
    alpha = segment_softmax(e, dst, num_nodes)
    if drop is not None:
        alpha = alpha * drop
    out = x_j * alpha.view(alpha.shape[0], alpha.shape[1], 1)
    if concat:
        out = out.reshape(out.shape[0], -1)
    else:
        out = torch.mean(out, dim=1)
    # aggregate: scatter-add into the target, dim_size = N
    agg = torch.zeros((num_nodes,) + tuple(out.shape[1:]), dtype=out.dtype)
    agg.index_add_(0, dst, out)
    return agg


def _project_heads(x, ws_weight, ws_bias, att1_weight, att1_bias, att2_weight, att2_bias):
    """``GAT.py:42-52``: the head loop of Linears, stack/transpose."""
    transformed, a1s, a2s = [], [], []
    for h in range(len(ws_weight)):
        t = torch.nn.functional.linear(x, ws_weight[h], ws_bias[h])
        transformed.append(t)
        a1s.append(torch.nn.functional.linear(t, att1_weight[h], att1_bias[h]))
        a2s.append(torch.nn.functional.linear(t, att2_weight[h], att2_bias[h]))
    transformed = torch.transpose(torch.stack(transformed), 0, 1)
    a1 = torch.stack(a1s).squeeze(-1).T
    a2 = torch.stack(a2s).squeeze(-1).T
    return transformed, a1, a2


def gat_layer_forward(x: torch.Tensor, edge_index: torch.Tensor,
                      ws_weight: Sequence[torch.Tensor], ws_bias: Sequence[torch.Tensor],
                      att1_weight: Sequence[torch.Tensor], att1_bias: Sequence[torch.Tensor],
                      att2_weight: Sequence[torch.Tensor], att2_bias: Sequence[torch.Tensor],
                      bias: torch.Tensor, concat: bool, negative_slope: float = 0.2) -> torch.Tensor:
    """``GraphAttentionLayer.forward`` (``GAT.py:37-54``) in eval mode."""
    with torch.no_grad():
        n = x.size(0)
        edge_ind = add_self_loops(edge_index, n)
        transformed, a1, a2 = _project_heads(x, ws_weight, ws_bias, att1_weight, att1_bias,
                                             att2_weight, att2_bias)
        return propagate(edge_ind, transformed, (a1, a2), n, concat, negative_slope) + bias


def _state_params(state: Dict[str, torch.Tensor], H: int):
    g = lambda k: state[k].detach().cpu()
    return ([g(f"ws.{h}.weight") for h in range(H)], [g(f"ws.{h}.bias") for h in range(H)],
            [g(f"attentions1.{h}.weight") for h in range(H)],
            [g(f"attentions1.{h}.bias") for h in range(H)],
            [g(f"attentions2.{h}.weight") for h in range(H)],
            [g(f"attentions2.{h}.bias") for h in range(H)])


def gat_layer_forward_from_state(state: Dict[str, torch.Tensor], x: torch.Tensor,
                                 edge_index: torch.Tensor, num_heads: int, concat: bool,
                                 negative_slope: float = 0.2) -> torch.Tensor:
    """Same as :func:`gat_layer_forward`, parameters taken from a reference
    ``state_dict`` (keys ``ws.{h}.weight`` … ``bias``, ``GAT.py:16-35``)."""
    return gat_layer_forward(x.detach().cpu(), edge_index.detach().cpu(),
                             *_state_params(state, num_heads), state["bias"].detach().cpu(),
                             concat, negative_slope)


def gat_layer_forward_rows(state: Dict[str, torch.Tensor], x: torch.Tensor,
                           edge_index: torch.Tensor, rows: torch.Tensor, num_heads: int,
                           concat: bool, negative_slope: float = 0.2,
                           batch: int = 1024) -> torch.Tensor:
    """``GAT.py:37-67`` for the target rows ``rows`` only, in batches: the
    projection (``GAT.py:42-52``) over all N nodes, as the reference does, then
    per batch the message / segmented softmax / scatter-add (``GAT.py:53-67``)
    over exactly those rows' in-edges, in ``edge_index`` order, each followed
    by the row's self-loop (``add_self_loops`` appends every node's loop after
    all original edges, ``GAT.py:38``, so a row's loop is its last in-edge).
    A row's output depends only on its own in-edges, so this equals
    ``gat_layer_forward_from_state(...)[rows]`` with the same per-row op
    order, while holding [E_batch, H, F] instead of the [E', H, F] message
    tensor (29 GB at Reddit scale).  Returns [len(rows), width]."""
    with torch.no_grad():
        x = x.detach().cpu()
        ei = edge_index.detach().cpu()
        rows = rows.detach().cpu().long()
        n = x.size(0)
        transformed, a1, a2 = _project_heads(x, *_state_params(state, num_heads))
        bias = state["bias"].detach().cpu()
        # every sampled row's in-edges in one pass over edge_index (order kept),
        # then each batch selects from that much smaller set
        ei = ei[:, torch.isin(ei[1], rows)]
        outs = []
        for b0 in range(0, rows.numel(), batch):
            rb = rows[b0:b0 + batch]
            sub = ei[:, torch.isin(ei[1], rb)]
            loops = rb.unique().unsqueeze(0).repeat(2, 1)
            agg = propagate(torch.cat([sub, loops], dim=1), transformed, (a1, a2), n, concat,
                            negative_slope)
            outs.append(agg[rb] + bias)
        return torch.cat(outs)


def closed_form_forward(state: Dict[str, torch.Tensor], x, edge_index, num_heads: int,
                        concat: bool, negative_slope: float = 0.2):
    """Pure-Python float64 loops over the closed form of SURVEY.md §8a —
    small cases only (known-answer tests).

    y[i,h] = sum_{(j->i) in E+loops} softmax_j(LReLU(s_dst[i,h] + s_src[j,h])) * Wh[j,h]
    """
    H = num_heads
    xs = [[float(v) for v in row] for row in x.tolist()]
    n = len(xs)
    src = list(edge_index[0].tolist()) + list(range(n))
    dst = list(edge_index[1].tolist()) + list(range(n))
    W = [state[f"ws.{h}.weight"].double().tolist() for h in range(H)]
    b = [state[f"ws.{h}.bias"].double().tolist() for h in range(H)]
    a1 = [state[f"attentions1.{h}.weight"].double().tolist()[0] for h in range(H)]
    c1 = [float(state[f"attentions1.{h}.bias"].double().item()) for h in range(H)]
    a2 = [state[f"attentions2.{h}.weight"].double().tolist()[0] for h in range(H)]
    c2 = [float(state[f"attentions2.{h}.bias"].double().item()) for h in range(H)]
    bias = state["bias"].double().tolist()
    F = len(b[0])
    wh = [[[sum(W[h][f][k] * xs[nn][k] for k in range(len(xs[nn]))) + b[h][f] for f in range(F)]
           for h in range(H)] for nn in range(n)]
    s_src = [[sum(wh[nn][h][f] * a1[h][f] for f in range(F)) + c1[h] for h in range(H)] for nn in range(n)]
    s_dst = [[sum(wh[nn][h][f] * a2[h][f] for f in range(F)) + c2[h] for h in range(H)] for nn in range(n)]
    out = []
    for i in range(n):
        ks = [k for k in range(len(dst)) if dst[k] == i]
        y = [[0.0] * F for _ in range(H)]
        for h in range(H):
            es = []
            for k in ks:
                z = s_dst[i][h] + s_src[src[k]][h]
                es.append(z if z > 0 else negative_slope * z)
            m = max(es)
            ps = [math.exp(e - m) for e in es]
            tot = sum(ps)
            for k, p in zip(ks, ps):
                for f in range(F):
                    y[h][f] += p / tot * wh[src[k]][h][f]
        if concat:
            out.append([y[h][f] + bias[h * F + f] for h in range(H) for f in range(F)])
        else:
            out.append([sum(y[h][f] for h in range(H)) / H + bias[f] for f in range(F)])
    return torch.tensor(out, dtype=torch.float64)


def init_reference_params(input_channels: int, output_channels: int, num_heads: int,
                          concat: bool, seed: Optional[int] = None) -> Dict[str, torch.Tensor]:
    """Parameters drawn in the reference constructor's RNG order
    (``GAT.py:19-35``): per head ``Linear(Fin,F)``, ``Linear(F,1)`` x2, then
    Xavier-uniform on the three weights; layer bias zeros.  Returned in the
    reference ``state_dict`` key order (``bias`` first: direct parameters
    precede child modules)."""
    if seed is not None:
        torch.manual_seed(seed)
    ws, a1, a2 = [], [], []
    for _ in range(num_heads):
        t = torch.nn.Linear(input_channels, output_channels)
        p = torch.nn.Linear(output_channels, 1)
        q = torch.nn.Linear(output_channels, 1)
        torch.nn.init.xavier_uniform_(t.weight)
        torch.nn.init.xavier_uniform_(p.weight)
        torch.nn.init.xavier_uniform_(q.weight)
        ws.append(t)
        a1.append(p)
        a2.append(q)
    width = output_channels * num_heads if concat else output_channels
    state = {"bias": torch.zeros(width)}
    for name, mods in (("ws", ws), ("attentions1", a1), ("attentions2", a2)):
        for h, m in enumerate(mods):
            state[f"{name}.{h}.weight"] = m.weight.detach().clone()
            state[f"{name}.{h}.bias"] = m.bias.detach().clone()
    return state


def gat_layer_forward_differentiable(params: Dict[str, torch.Tensor], x: torch.Tensor,
                                     edge_index: torch.Tensor, num_heads: int, concat: bool,
                                     negative_slope: float = 0.2,
                                     drop: Optional[torch.Tensor] = None,
                                     activation=None) -> torch.Tensor:
    """``GAT.py:37-67`` with autograd left on (the reference trains through
    it with ``loss.backward()``): the gradient oracle.  ``params`` uses the
    reference ``state_dict`` keys; ``drop`` is the dropout multiplier per
    (edge in add_self_loops order, head)."""
    H = num_heads
    n = x.size(0)
    edge_ind = add_self_loops(edge_index, n)
    transformed, a1s, a2s = [], [], []
    for h in range(H):
        t = torch.nn.functional.linear(x, params[f"ws.{h}.weight"], params[f"ws.{h}.bias"])
        transformed.append(t)
        a1s.append(torch.nn.functional.linear(t, params[f"attentions1.{h}.weight"],
                                              params[f"attentions1.{h}.bias"]))
        a2s.append(torch.nn.functional.linear(t, params[f"attentions2.{h}.weight"],
                                              params[f"attentions2.{h}.bias"]))
    transformed = torch.transpose(torch.stack(transformed), 0, 1)
    a1 = torch.stack(a1s).squeeze(-1).T
    a2 = torch.stack(a2s).squeeze(-1).T
    return propagate(edge_ind, transformed, (a1, a2), n, concat, negative_slope,
                     drop, activation) + params["bias"]


def _mix32(x):
    import numpy as np
    x = x.astype(np.uint32)
    x ^= x >> np.uint32(16)
    x *= np.uint32(0x7FEB352D)
    x ^= x >> np.uint32(15)
    x *= np.uint32(0x846CA68B)
    x ^= x >> np.uint32(16)
    return x


def dropout_factors(positions, num_heads: int, p: float, seed: int):
    """The HIP library's attention-dropout mask, restated in numpy (its
    ``drop_factor``: keep (k, h) iff mix(seed, k*H + h) >= round(p * 2^32)).
    ``positions`` are CSR edge positions; returns float64 [len, H] of 0 or
    1/(1-p).  The mask itself is a design choice of this library (the
    reference draws it from torch's RNG, GAT.py:61), so parity of a dropout
    step is checked against this mask, not the reference's draw."""
    import numpy as np
    k = np.asarray(positions, dtype=np.uint64)[:, None]
    h = np.arange(num_heads, dtype=np.uint64)[None, :]
    idx = k * np.uint64(num_heads) + h
    lo = (idx & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    hi = (idx >> np.uint64(32)).astype(np.uint32)
    seed_lo = np.uint32(seed & 0xFFFFFFFF)
    seed_hi = np.uint32((seed >> 32) & 0xFFFFFFFF)
    a = _mix32(lo ^ seed_lo)
    with np.errstate(over="ignore"):
        b = _mix32((hi + seed_hi).astype(np.uint32))
    r = _mix32(a ^ b)
    thresh = min(max(math.floor(p * 4294967296.0 + 0.5), 0), 4294967295)
    scale = 1.0 if p <= 0 else (0.0 if p >= 1 else
                                 float(np.float32(1.0) / (np.float32(1.0) - np.float32(p))))
    return np.where(r >= np.uint32(thresh), scale, 0.0)


def csr_positions(edge_index: torch.Tensor, num_nodes: int):
    """CSR position of each edge of ``add_self_loops(edge_index)`` in the HIP
    library's CSR (sorted by (target, source); equal pairs in input order)."""
    import numpy as np
    dst = np.concatenate([edge_index[1].cpu().numpy(), np.arange(num_nodes)])
    src = np.concatenate([edge_index[0].cpu().numpy(), np.arange(num_nodes)])
    order = np.lexsort((src, dst))
    pos = np.empty_like(order)
    pos[order] = np.arange(order.size)
    return pos
