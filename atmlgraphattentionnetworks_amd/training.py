"""Training path of the layer: forward with attention dropout and the HIP
backward pass, as one ``torch.autograd.Function``.

The reference trains ``GraphAttentionLayer`` through PyTorch autograd over
PyG's gather/scatter ops (``run_inductive.py:83-90``, ``run_*_experiment.py``:
``loss.backward(); optimizer.step()``).  Here the gradient of
``GAT.py:37-67`` is computed by three library calls and two plain GEMMs:

  forward   gat_project, then gat_edge_aggregate_train (LeakyReLU, HF = 64:
            also the per-head kink sums Q, R) or gat_edge_aggregate_ex (dropout
            GAT.py:61 from a counter-based hash; any score activation; also
            stores lse and the per-head aggregation y)
  backward  1. gat_bwd_table after gat_edge_aggregate_train (elementwise:
               ds_dst = dy.Q - delta R), else gat_bwd_targets (per target row
               over the in-edges: dropout, softmax and LeakyReLU backward ->
               ds_dst); both write the per-target table [g | s_dst, lse, delta]
            2. gat_bwd_sources (per source row over the CSC: recomputes each
               edge's coefficient from the table, dWh = sum A * dy + the score
               terms; per-wave partials of da/dc/db/dbias -- deterministic, no
               atomics), gat_sum_partials
            (other score activations or head widths: gat_edge_backward_rows,
            which stores (A, dz) per edge in CSC order, + gat_src_backward)
            3. gat_weight_grad: dW = dWh^T x (split-K fp32 MFMA)
            4. gat_input_grad: dx = dWh W (fp32 matrix cores), only when x
               needs a gradient.

The per-head parameters are views into the packed buffers the kernels read
(``GraphAttentionLayer._bind_packed``), so the gradients come back as views of
the packed gradients and land on each head's ``Linear`` exactly where the
reference's autograd would put them.
"""
from __future__ import annotations

import torch

from . import _lib
from .graph import CSRGraph, get_csc

__all__ = ["GATFunction", "gat_train_forward", "new_dropout_seed", "next_seed_slot"]

# rows of per-wave partials written by gat_src_backward
_MAX_PARTS = 8192


def new_dropout_seed() -> int:
    """A fresh 62-bit dropout seed from torch's default generator, so that
    ``torch.manual_seed`` makes training runs reproducible."""
    return int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())


def next_seed_slot(owner, device: torch.device) -> torch.Tensor:
    """A device int64[1] holding this call's dropout seed, written on the
    current stream by ``gat_dropout_seed_next`` from a per-owner device counter
    (started from torch's default generator, so ``torch.manual_seed`` fixes the
    sequence).  Because the seed is produced on the GPU, a training step
    captured in a HIP graph draws a fresh mask on every replay.  The counter is
    a plain attribute, not a buffer: the state_dict keys stay the reference's."""
    if device.index is None:
        device = torch.device(device.type, torch.cuda.current_device())
    counters = owner.__dict__.setdefault("_dropout_counters", {})
    ctr = counters.get(device)
    if ctr is None:
        ctr = torch.tensor([new_dropout_seed()], dtype=torch.int64, device=device)
        counters[device] = ctr
    slot = torch.empty(1, dtype=torch.int64, device=device)
    _lib.check(_lib.load().gat_dropout_seed_next(
        ctr.data_ptr(), slot.data_ptr(), torch._C._cuda_getCurrentRawStream(device.index)),
        "gat_dropout_seed_next")
    return slot


class GATFunction(torch.autograd.Function):
    """Layer forward (training) and backward on prepared inputs.

    ``params`` are the layer's 6H per-head leaves, in ``_param_list`` order;
    they only route gradients — the kernels read the packed buffers ``pp``
    they are views of (``GraphAttentionLayer._bind_packed``)."""

    @staticmethod
    def forward(ctx, x, bias, cfg, csr: CSRGraph, pp, seed_slot, *params):
        heads, f, concat, act, act_param, p, seed = cfg
        p_seed = 0 if seed_slot is None else seed_slot.data_ptr()
        lib = _lib.load()
        n, fin = x.shape
        hf = heads * f
        hfp = (hf + 3) // 4 * 4
        dev = x.device
        stream = torch._C._cuda_getCurrentRawStream(dev.index)
        # one workspace: Wh | s_src | s_dst | lse | y | Q | R (Q, R: kink sums)
        kink = act == _lib.GAT_ACT_LEAKY_RELU
        ws = torch.empty(n * (hfp + 3 * heads + hf + (hf + heads if kink else 0)),
                         dtype=torch.float32, device=dev)
        # raw pointers into it (no per-call slice views: host cost of small graphs)
        p_wh = ws.data_ptr()
        p_ss = p_wh + 4 * n * hfp
        p_sd, p_lse, p_y = p_ss + 4 * n * heads, p_ss + 8 * n * heads, p_ss + 12 * n * heads
        from .layer import project_workspace
        pws = project_workspace(dev, fin, heads, f)
        rc = lib.gat_project_ex(x.data_ptr(), n, fin, pp.w.data_ptr(), pp.b.data_ptr(),
                                pp.a_src.data_ptr(), pp.c_src.data_ptr(), pp.a_dst.data_ptr(),
                                pp.c_dst.data_ptr(), heads, f, 1, p_wh, hfp,
                                p_ss, heads, p_sd, 0, 0,
                                0 if pws is None else pws.data_ptr(),
                                0 if pws is None else pws.numel(), stream)
        if rc:
            _lib.check(rc, "gat_project_ex")
        out = torch.empty(n, hf if concat else f, dtype=torch.float32, device=dev)
        order = csr.order
        if kink:
            p_q = p_y + 4 * n * hf
            rc = lib.gat_edge_aggregate_train(
                csr.rowptr.data_ptr(), csr.col.data_ptr(), 0 if order is None else order.data_ptr(),
                0, n, p_wh, hfp, pp.a_src.data_ptr(), pp.c_src.data_ptr(),
                p_sd, heads, f, int(concat), act_param, p, seed, p_seed,
                bias.data_ptr(), out.data_ptr(), p_lse, p_y, p_q,
                p_q + 4 * n * hf, csr.kernel_hint(), stream)
            if rc and rc != _lib.GAT_EUNSUPPORTED:
                _lib.check(rc, "gat_edge_aggregate_train")
            kink = rc == 0  # GAT_EUNSUPPORTED: another head shape, or GAT_BWD_KINK=0
        if not kink:
            rc = lib.gat_edge_aggregate_ex(
                csr.rowptr.data_ptr(), csr.col.data_ptr(),
                0 if order is None else order.data_ptr(), 0, n, p_wh, hfp,
                p_ss, heads, pp.a_src.data_ptr(), pp.c_src.data_ptr(),
                p_sd, heads, f, int(concat), act, act_param, p, seed, p_seed,
                bias.data_ptr(), out.data_ptr(), p_lse, p_y,
                csr.kernel_hint(), stream)
            if rc:
                _lib.check(rc, "gat_edge_aggregate_ex")
        ctx.save_for_backward(x, ws)
        ctx.csr, ctx.pp, ctx.cfg, ctx.seed_slot = csr, pp, cfg, seed_slot
        ctx.kink = kink
        return out

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, g):
        x, ws = ctx.saved_tensors
        heads, f, concat, act, act_param, p, seed = ctx.cfg
        csr, pp = ctx.csr, ctx.pp
        g = g.contiguous()
        if g.dtype != torch.float32:
            g = g.float()
        n, fin = x.shape
        hf = heads * f
        dev = x.device
        stream = torch._C._cuda_getCurrentRawStream(dev.index)
        csc = get_csc(csr)
        dwh, ps = _backward_recompute(ctx, g, ws, csc, stream)
        if dwh is None:
            dwh, ps = _backward_stored(ctx, g, ws, csc, stream)
        need = ctx.needs_input_grad
        dx = None
        if need[0]:  # dx = dWh W (gat_input_grad: fp32 matrix cores, hf <= 128)
            dx = torch.empty(n, fin, dtype=torch.float32, device=dev)
            rc = _lib.load().gat_input_grad(dwh.data_ptr(), dwh.stride(0), n, hf,
                                            pp.w.data_ptr(), fin, dx.data_ptr(), fin, stream)
            if rc == _lib.GAT_EUNSUPPORTED:
                dx = torch.mm(dwh, pp.w)  # wider tables than any reference configuration
            elif rc:
                _lib.check(rc, "gat_input_grad")
        dbias = ps[3 * hf + 2 * heads:] if need[1] else None
        grads = [None] * (6 * heads)
        if any(need[5:]):
            lib = _lib.load()
            dw = torch.empty(hf, fin, dtype=torch.float32, device=dev)
            wsz = _lib.weight_grad_workspace_size(n, fin, hf)
            wws = torch.empty(max(wsz // 4, 1), dtype=torch.float32, device=dev)
            rc = lib.gat_weight_grad(x.data_ptr(), n, fin, dwh.data_ptr(), hf, hf, dw.data_ptr(),
                                     wws.data_ptr(), wsz, stream)
            if rc:
                _lib.check(rc, "gat_weight_grad")
            H = heads
            grads[0:H] = dw.view(H, f, fin).unbind(0)
            grads[H:2 * H] = ps[2 * hf + 2 * H:3 * hf + 2 * H].view(H, f).unbind(0)
            grads[2 * H:3 * H] = ps[:hf].view(H, 1, f).unbind(0)
            grads[3 * H:4 * H] = ps[2 * hf:2 * hf + H].view(H, 1).unbind(0)
            grads[4 * H:5 * H] = ps[hf:2 * hf].view(H, 1, f).unbind(0)
            grads[5 * H:6 * H] = ps[2 * hf + H:2 * hf + 2 * H].view(H, 1).unbind(0)
        return (dx, dbias, None, None, None, None, *grads)


def _line_up(floats: int) -> int:
    """``floats`` rounded up to a whole 128-B line (32 floats)."""
    return (floats + 31) // 32 * 32


def _seed_ptr(ctx) -> int:
    return 0 if ctx.seed_slot is None else ctx.seed_slot.data_ptr()


def _sums_tensor(pw: int, device) -> torch.Tensor:
    """The per-parameter gradient sums get their own small allocation: the
    bias / attention gradients handed to autograd are views of it, and views
    of the backward workspace would keep that workspace (per-edge
    coefficients on the stored path: 8 B per edge and head) alive for as long
    as the gradients are."""
    return torch.empty(pw, dtype=torch.float32, device=device)


def _saved_layout(ctx, ws):
    """Pointers into the forward workspace: Wh | s_src | s_dst | lse | y."""
    heads, f = ctx.cfg[0], ctx.cfg[1]
    n = ctx.csr.num_nodes
    hfp = (heads * f + 3) // 4 * 4
    p_wh = ws.data_ptr()
    p_ss = p_wh + 4 * n * hfp
    return hfp, p_wh, p_ss, p_ss + 4 * n * heads, p_ss + 8 * n * heads, p_ss + 12 * n * heads


def _backward_recompute(ctx, g, ws, csc, stream):
    """gat_bwd_targets + gat_bwd_sources (no per-edge intermediates); returns
    (None, None) when the shape or activation needs the stored-coefficient path."""
    heads, f, concat, act, act_param, p, seed = ctx.cfg
    if act != _lib.GAT_ACT_LEAKY_RELU:
        return None, None
    csr, pp = ctx.csr, ctx.pp
    lib = _lib.load()
    n = csr.num_nodes
    hf = heads * f
    ldg = hf if concat else f
    pw = 3 * hf + 2 * heads + ldg
    ld_t = _lib.bwd_table_layout(heads, f, concat)
    parts = _lib.bwd_sources_parts(n, heads, f)
    sws = (parts + 255) // 256 * pw if parts > 256 else 0
    hfp, p_wh, p_ss, p_sd, p_lse, p_y = _saved_layout(ctx, ws)
    # one workspace: ds_dst | target table | dwh | partials | sums | scratch; the
    # table starts on a 128-B line (its rows are whole lines: a row gathered per
    # out-edge in pass 2 then touches 3 lines, not 4), and so does dwh
    o_t = _line_up(n * heads)
    o_dwh = _line_up(o_t + n * ld_t)
    o_part = o_dwh + n * hf
    o_ps = o_part + parts * pw
    bw = torch.empty(o_ps + pw + sws, dtype=torch.float32, device=g.device)
    base = bw.data_ptr()
    order = csr.order
    hint = csr.kernel_hint()
    if ctx.kink:
        # the forward stored the kink sums Q | R after y: no pass over the in-edges
        p_q = p_y + 4 * n * hf
        rc = lib.gat_bwd_table(p_sd, p_lse, p_y, p_q, p_q + 4 * n * hf, g.data_ptr(), n, heads,
                               f, int(concat), base, base + 4 * o_t, ld_t, stream)
        name = "gat_bwd_table"
    else:
        rc = lib.gat_bwd_targets(
            csr.rowptr.data_ptr(), csr.col.data_ptr(), 0 if order is None else order.data_ptr(),
            0, n, p_wh, hfp, pp.a_src.data_ptr(), pp.c_src.data_ptr(), p_sd, p_lse, p_y,
            g.data_ptr(), heads, f, int(concat), act_param, p, seed, _seed_ptr(ctx), base,
            base + 4 * o_t, ld_t, hint, stream)
        name = "gat_bwd_targets"
    if rc == _lib.GAT_EUNSUPPORTED:
        return None, None
    if rc:
        _lib.check(rc, name)
    rc = lib.gat_bwd_sources(
        csc.ptr.data_ptr(), csc.dst.data_ptr(), csc.eid.data_ptr(), n, p_wh, hfp,
        base + 4 * o_t, ld_t, base, pp.a_src.data_ptr(), pp.c_src.data_ptr(),
        pp.a_dst.data_ptr(), heads, f, int(concat), act_param, p, seed, _seed_ptr(ctx),
        base + 4 * o_dwh, hf, base + 4 * o_part, parts, hint, stream)
    if rc:
        _lib.check(rc, "gat_bwd_sources")
    ps = _sums_tensor(pw, g.device)
    rc = lib.gat_sum_partials(base + 4 * o_part, parts, pw, ps.data_ptr(),
                              base + 4 * (o_ps + pw), 4 * sws, stream)
    if rc:
        _lib.check(rc, "gat_sum_partials")
    return bw[o_dwh:o_part].view(n, hf), ps


def _backward_stored(ctx, g, ws, csc, stream):
    """gat_edge_backward_rows (per-edge (A, dz) stored in CSC order) +
    gat_src_backward: any score activation, any head width."""
    heads, f, concat, act, act_param, p, seed = ctx.cfg
    csr, pp = ctx.csr, ctx.pp
    lib = _lib.load()
    n = csr.num_nodes
    hf = heads * f
    nnz = csr.num_edges
    ldg = hf if concat else f
    parts = max(1, min(n, _MAX_PARTS))
    pw = 3 * hf + 2 * heads + ldg
    sws = (parts + 255) // 256 * pw if parts > 256 else 0
    hfp, p_wh, p_ss, p_sd, p_lse, p_y = _saved_layout(ctx, ws)
    # one workspace: ds_dst | (A, dz) per edge and head | dwh | partials | sums | scratch
    m = 2 * max(nnz, 1) * heads
    o_dwh = _line_up(n * heads + m)
    o_part = o_dwh + n * hf
    o_ps = o_part + parts * pw
    bw = torch.empty(o_ps + pw + sws, dtype=torch.float32, device=g.device)
    p_dsd = bw.data_ptr()
    p_az = p_dsd + 4 * n * heads
    p_part = bw.data_ptr() + 4 * o_part
    order = csr.order
    rc = lib.gat_edge_backward_rows(
        csr.rowptr.data_ptr(), csr.col.data_ptr(), 0 if order is None else order.data_ptr(),
        0, n, csc.csr_to_csc.data_ptr(), p_wh, hfp, p_ss, heads, pp.a_src.data_ptr(),
        pp.c_src.data_ptr(), p_sd, p_lse, p_y, g.data_ptr(), heads, f, int(concat), act,
        act_param, p, seed, _seed_ptr(ctx), p_dsd, p_az, nnz // max(n, 1), stream)
    if rc:
        _lib.check(rc, "gat_edge_backward_rows")
    rc = lib.gat_src_backward(
        csc.ptr.data_ptr(), csc.dst.data_ptr(), n, p_wh, hfp, g.data_ptr(), p_az, p_dsd,
        pp.a_src.data_ptr(), pp.a_dst.data_ptr(), heads, f, int(concat),
        bw.data_ptr() + 4 * o_dwh, hf, 0, p_part, parts, stream)
    if rc:
        _lib.check(rc, "gat_src_backward")
    ps = _sums_tensor(pw, g.device)
    rc = lib.gat_sum_partials(p_part, parts, pw, ps.data_ptr(),
                              bw.data_ptr() + 4 * (o_ps + pw), 4 * sws, stream)
    if rc:
        _lib.check(rc, "gat_sum_partials")
    return bw[o_dwh:o_part].view(n, hf), ps


def gat_train_forward(layer, x: torch.Tensor, csr: CSRGraph, p: float, seed: int,
                      act: int = None, act_param: float = None, seed_slot=None):
    """``seed_slot`` (a device int64[1], ``next_seed_slot``) overrides ``seed``."""
    from .layer import _param_list
    if act is None:
        act, act_param = layer.score_activation()
    pp = layer.packed()
    cfg = (layer.num_heads, layer.output_channels, bool(layer.concat), int(act),
           float(act_param), float(p), int(seed))
    return GATFunction.apply(x, layer.bias, cfg, csr, pp, seed_slot, *_param_list(layer))
