"""Training path of the layer: forward with attention dropout and the HIP
backward pass, as one ``torch.autograd.Function``.

The reference trains ``GraphAttentionLayer`` through PyTorch autograd over
PyG's gather/scatter ops (``run_inductive.py:83-90``, ``run_*_experiment.py``:
``loss.backward(); optimizer.step()``).  Here the gradient of
``GAT.py:37-67`` is computed by three library calls and two plain GEMMs:

  forward   gat_project, then gat_edge_aggregate_ex (dropout GAT.py:61 from a
            counter-based hash; any score activation; also stores lse and the
            per-head aggregation y)
  backward  1. gat_edge_backward_rows (per target row: dropout, softmax and
               LeakyReLU backward -> ds_dst, and per-edge A / dz in CSC order)
            2. gat_src_backward (per source row: dWh = sum A * dy + the score
               terms; per-wave partials of da/dc -- deterministic, no atomics)
            3. dW = dWh^T x, db = sum dWh, dx = dWh W (hipBLASLt via torch.mm:
               plain library GEMMs), dbias = sum of the incoming gradient.

The packed parameters (W = cat of ws[h].weight, ...) are built with
differentiable ``torch.cat`` by the caller, so the gradients land on each
head's ``Linear`` exactly where the reference's would.
"""
from __future__ import annotations

import torch

from . import _lib
from .graph import CSRGraph, get_csc

__all__ = ["GATFunction", "gat_train_forward", "new_dropout_seed"]

# rows of per-wave partials written by gat_src_backward
_MAX_PARTS = 8192


def new_dropout_seed() -> int:
    """A fresh 62-bit dropout seed from torch's default generator, so that
    ``torch.manual_seed`` makes training runs reproducible."""
    return int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())


class GATFunction(torch.autograd.Function):
    """Layer forward (training) and backward on prepared inputs."""

    @staticmethod
    def forward(ctx, x, w, b, a_src, c_src, a_dst, c_dst, bias, csr: CSRGraph, heads: int,
                f: int, concat: bool, act: int, act_param: float, p: float, seed: int):
        lib = _lib.load()
        n, fin = x.shape
        hf = heads * f
        hfp = (hf + 3) // 4 * 4
        dev = x.device
        stream = torch._C._cuda_getCurrentRawStream(dev.index)
        wh = torch.empty(n, hfp, dtype=torch.float32, device=dev)
        s_src = torch.empty(n, heads, dtype=torch.float32, device=dev)
        s_dst = torch.empty(n, heads, dtype=torch.float32, device=dev)
        _lib.check(lib.gat_project(x.data_ptr(), n, fin, w.data_ptr(), b.data_ptr(),
                                   a_src.data_ptr(), c_src.data_ptr(), a_dst.data_ptr(),
                                   c_dst.data_ptr(), heads, f, wh.data_ptr(), hfp,
                                   s_src.data_ptr(), heads, s_dst.data_ptr(), stream),
                   "gat_project")
        out = torch.empty(n, hf if concat else f, dtype=torch.float32, device=dev)
        lse = torch.empty(n, heads, dtype=torch.float32, device=dev)
        y = torch.empty(n, hf, dtype=torch.float32, device=dev)
        order = csr.order
        _lib.check(lib.gat_edge_aggregate_ex(
            csr.rowptr.data_ptr(), csr.col.data_ptr(), 0 if order is None else order.data_ptr(),
            0, n, wh.data_ptr(), hfp, s_src.data_ptr(), heads, a_src.data_ptr(),
            c_src.data_ptr(), s_dst.data_ptr(), heads, f, int(concat), int(act),
            float(act_param), float(p), int(seed), bias.data_ptr(), out.data_ptr(),
            lse.data_ptr(), y.data_ptr(), csr.num_edges // max(n, 1), stream),
            "gat_edge_aggregate_ex")
        ctx.save_for_backward(x, w, a_src, a_dst, wh, s_src, s_dst, lse, y)
        ctx.csr = csr
        ctx.cfg = (heads, f, bool(concat), int(act), float(act_param), float(p), int(seed))
        return out

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, g):
        x, w, a_src, a_dst, wh, s_src, s_dst, lse, y = ctx.saved_tensors
        heads, f, concat, act, act_param, p, seed = ctx.cfg
        csr = ctx.csr
        lib = _lib.load()
        g = g.contiguous()
        if g.dtype != torch.float32:
            g = g.float()
        n, fin = x.shape
        hf = heads * f
        hfp = wh.size(1)
        dev = x.device
        stream = torch._C._cuda_getCurrentRawStream(dev.index)
        csc = get_csc(csr)
        nnz = csr.num_edges
        ds_dst = torch.empty(n, heads, dtype=torch.float32, device=dev)
        alpha = torch.empty(max(nnz, 1), heads, dtype=torch.float32, device=dev)
        dz = torch.empty(max(nnz, 1), heads, dtype=torch.float32, device=dev)
        order = csr.order
        _lib.check(lib.gat_edge_backward_rows(
            csr.rowptr.data_ptr(), csr.col.data_ptr(), 0 if order is None else order.data_ptr(),
            0, n, csc.csr_to_csc.data_ptr(), wh.data_ptr(), hfp, s_src.data_ptr(), heads,
            s_dst.data_ptr(), lse.data_ptr(), y.data_ptr(), g.data_ptr(), heads, f, int(concat),
            act, act_param, p, seed, ds_dst.data_ptr(), alpha.data_ptr(), dz.data_ptr(), stream),
            "gat_edge_backward_rows")
        parts = max(1, min(n, _MAX_PARTS))
        dwh = torch.empty(n, hf, dtype=torch.float32, device=dev)
        part = torch.empty(parts, 2 * hf + 2 * heads, dtype=torch.float32, device=dev)
        _lib.check(lib.gat_src_backward(
            csc.ptr.data_ptr(), csc.dst.data_ptr(), n, wh.data_ptr(), hfp, g.data_ptr(),
            alpha.data_ptr(), dz.data_ptr(), ds_dst.data_ptr(), a_src.data_ptr(),
            a_dst.data_ptr(), heads, f, int(concat), dwh.data_ptr(), hf, 0, part.data_ptr(),
            parts, stream), "gat_src_backward")
        ps = part.sum(0)
        need = ctx.needs_input_grad
        dx = torch.mm(dwh, w) if need[0] else None
        dw = torch.mm(dwh.t(), x) if need[1] else None
        db = dwh.sum(0) if need[2] else None
        da_src = ps[:hf] if need[3] else None
        dc_src = ps[2 * hf:2 * hf + heads] if need[4] else None
        da_dst = ps[hf:2 * hf] if need[5] else None
        dc_dst = ps[2 * hf + heads:] if need[6] else None
        dbias = g.sum(0) if need[7] else None
        return (dx, dw, db, da_src, dc_src, da_dst, dc_dst, dbias,
                None, None, None, None, None, None, None, None)


def packed_params_differentiable(layer):
    """cat of the per-head parameters, recorded by autograd (GAT.py:19-22)."""
    H = layer.num_heads
    ws = list(layer.ws._modules.values())
    a1 = list(layer.attentions1._modules.values())
    a2 = list(layer.attentions2._modules.values())
    w = torch.cat([m.weight for m in ws], 0)
    b = torch.cat([m.bias for m in ws], 0)
    a_src = torch.cat([m.weight.reshape(-1) for m in a1])
    c_src = torch.cat([m.bias.reshape(-1) for m in a1])
    a_dst = torch.cat([m.weight.reshape(-1) for m in a2])
    c_dst = torch.cat([m.bias.reshape(-1) for m in a2])
    assert w.size(0) == H * layer.output_channels
    return w, b, a_src, c_src, a_dst, c_dst


def gat_train_forward(layer, x: torch.Tensor, csr: CSRGraph, p: float, seed: int):
    w, b, a_src, c_src, a_dst, c_dst = packed_params_differentiable(layer)
    act, act_param = layer.score_activation()
    return GATFunction.apply(x, w, b, a_src, c_src, a_dst, c_dst, layer.bias, csr,
                             layer.num_heads, layer.output_channels, layer.concat,
                             act, act_param, p, seed)
