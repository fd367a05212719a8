#!/usr/bin/env python3
"""Interleaved A/B of edge-kernel variants in the layer's own table layout
(sliced planes where the layer uses them), in ONE process.  A variant is a set
of GAT_* knobs, e.g. ``base`` (no knobs) or ``GAT_EDGE_U=8,GAT_EDGE_SPLIT=1``.
Outputs are compared against the first variant (max |diff|).

    python tools/edge_ab.py --workload reddit --rounds 5 \
        --variants "base;GAT_EDGE_U=8;GAT_EDGE_PIPE=0"

``--only K`` runs variant K alone, ``--iters`` times, eagerly (for rocprofv3
--pmc passes: every launch of the kernel is then that variant).
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from atmlgraphattentionnetworks_amd import tuning  # noqa: E402

from timing import time_fn  # noqa: E402

KNOBS = ("GAT_EDGE_U", "GAT_EDGE_V", "GAT_EDGE_PIPE", "GAT_EDGE_SPLIT", "GAT_EDGE_ROWCOL",
         "GAT_EDGE_XPROJ", "GAT_WH_SLICES", "GAT_HUB_SPLIT", "GAT_HUB_SEG", "GAT_EDGE_SCHED")


def parse(spec):
    """knobs of a variant; the pseudo-knob ``passes=W`` runs the edge work as W
    source-window passes (gat_edge_aggregate_seg, online-softmax state carried
    in memory between passes)."""
    if spec in ("", "base"):
        return {}
    return dict(kv.split("=", 1) for kv in spec.split(","))


def window_segments(csr, windows):
    """[windows + 1, N] int32: pass c covers CSR positions [seg[c], seg[c+1]) of
    each row, the in-edges whose source lies in window c of the node range."""
    n = csr.num_nodes
    rp = csr.rowptr.to(torch.int64)
    deg = rp[1:] - rp[:-1]
    row_id = torch.repeat_interleave(torch.arange(n, device=rp.device), deg)
    blk = (n + windows - 1) // windows
    ch = csr.col.to(torch.int64) // blk
    cnt = torch.zeros(n * windows, dtype=torch.int64, device=rp.device)
    cnt.index_add_(0, row_id * windows + ch, torch.ones_like(ch))
    del row_id, ch
    seg = torch.empty(windows + 1, n, dtype=torch.int32, device=rp.device)
    seg[0] = rp[:-1].to(torch.int32)
    seg[1:] = (rp[:-1].unsqueeze(1) + cnt.view(n, windows).cumsum(1)).t().to(torch.int32)
    return seg


def apply(env):
    for k in KNOBS:
        os.environ.pop(k, None)
    os.environ.update(env)
    tuning.reload()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="reddit")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--variants", default="base")
    ap.add_argument("--only", type=int, default=-1)
    ap.add_argument("--layer", action="store_true", help="also time the whole layer forward")
    args = ap.parse_args()
    from atmlgraphattentionnetworks_amd import GraphAttentionLayer, get_csr
    from atmlgraphattentionnetworks_amd.layer import ForwardPlan, gat_forward
    from atmlgraphattentionnetworks_amd import _lib
    from atmlgraphattentionnetworks_amd.synthetic import WORKLOADS, make_inputs

    lib = _lib.load()
    dev = torch.device("cuda", 0)
    w = WORKLOADS[args.workload]
    x, ei = make_inputs(w, dev)
    n = x.size(0)
    torch.manual_seed(0)
    layer = GraphAttentionLayer(w.in_channels, w.out_channels, num_heads=w.heads,
                                concat=w.concat).to(dev).eval()
    csr = get_csr(ei, n)
    del ei
    pp = layer.packed()
    bias = layer.bias.detach()
    specs = [s.strip() for s in args.variants.split(";") if s.strip()]
    envs = [parse(s) for s in specs]
    knob_envs = [{k: v for k, v in e.items() if k not in ("passes", "sched", "hubseg", "hublast")}
                 for e in envs]

    plan_out = {}
    H, F = w.heads, w.out_channels
    hf = H * F

    class Passes:
        """The edge work as W source-window passes over the plan's table."""

        def __init__(self, plan, windows):
            self.plan, self.windows = plan, windows
            self.seg = window_segments(csr, windows)
            self.st_acc = torch.empty(n, (hf + 3) // 4 * 4, device=dev)
            self.st_ml = torch.empty(n, 2 * H, device=dev)

        def edge(self, lib, csr_, pp_, bias_, out):
            p = self.plan
            stream = torch._C._cuda_getCurrentRawStream(dev.index)
            ld = hf // p.slices if p.slices > 1 else p.hfp
            for c in range(self.windows):
                flags = (_lib.GAT_SEG_LOAD if c > 0 else 0) | \
                    (_lib.GAT_SEG_STORE if c < self.windows - 1 else 0)
                rc = lib.gat_edge_aggregate_seg(
                    self.seg[c].data_ptr(), self.seg[c + 1].data_ptr(), 0, csr.col.data_ptr(),
                    csr.order.data_ptr(), 0, n, p.p_wh, ld, n, p.slices, pp.a_src.data_ptr(),
                    pp.c_src.data_ptr(), p.p_sd, H, F, 1, 0.2, self.st_acc.data_ptr(),
                    self.st_ml.data_ptr(), flags, 0, bias.data_ptr(), out.data_ptr(), p.hint,
                    stream)
                _lib.check(rc, "seg pass")
            return out

        def kernel_name(self):
            return f"{self.windows} source-window passes: " + self.plan.kernel_name()

    class Sched:
        """The edge kernel over a SCHEDULED copy of the CSR: rows laid out in
        the degree order the kernel walks them (positions by_pos), so a lane
        group's row bounds come from one load independent of order[pos], and
        the rows sharing a wave read adjacent col ranges."""

        def __init__(self, plan):
            self.plan = plan
            rp = csr.rowptr.to(torch.int64)
            order = csr.order.to(torch.int64)
            deg = (rp[1:] - rp[:-1])[order]
            sptr = torch.zeros(n + 1, dtype=torch.int64, device=dev)
            sptr[1:] = deg.cumsum(0)
            e = int(sptr[-1])
            offs = torch.arange(e, device=dev) - torch.repeat_interleave(sptr[:-1], deg)
            idx = torch.repeat_interleave(rp[order], deg) + offs
            self.col = csr.col[idx].contiguous()
            self.sb = sptr[:-1].to(torch.int32).contiguous()
            self.se = sptr[1:].to(torch.int32).contiguous()

        def edge(self, lib, csr_, pp_, bias_, out):
            p = self.plan
            stream = torch._C._cuda_getCurrentRawStream(dev.index)
            ld = hf // p.slices if p.slices > 1 else p.hfp
            rc = lib.gat_edge_aggregate_seg(
                self.sb.data_ptr(), self.se.data_ptr(), 1, self.col.data_ptr(),
                csr.order.data_ptr(), 0, n, p.p_wh, ld, n, p.slices, pp.a_src.data_ptr(),
                pp.c_src.data_ptr(), p.p_sd, H, F, int(w.concat), 0.2, 0, 0, 0, 0,
                bias.data_ptr(), out.data_ptr(), p.khint, stream)
            _lib.check(rc, "scheduled CSR")
            return out

        def kernel_name(self):
            return "scheduled CSR: " + self.plan.kernel_name()

    class HubSeg:
        """The default plan over a copy of the CSR whose hub rows are split at
        a different segment length (graph.hub_plan(seg_len=...)) and the
        variant's GAT_HUB_ORDER / GAT_ROW_ORDER."""

        def __init__(self, seg_len):
            from atmlgraphattentionnetworks_amd.graph import hub_plan
            self.csr = csr._replace(
                hubs=hub_plan(csr.rowptr, csr.order, csr.num_edges, seg_len=seg_len, col=csr.col))
            self.plan = ForwardPlan(x, self.csr, w.heads, w.out_channels, w.concat, 0.2)
            self.plan.project(lib, x, pp)
            self.seg_len = seg_len

        def edge(self, lib, csr_, pp_, bias_, out):
            return self.plan.edge(lib, self.csr, pp_, bias_, out)

        def kernel_name(self):
            h = self.csr.hubs
            return (f"hub segments of {self.seg_len} ({0 if h is None else h.n_hub} hubs, "
                    f"{0 if h is None else h.n_vrows} segments): " + self.plan.kernel_name())

    class HubLast:
        """Hub rows split as the default plan, but the whole rows run FIRST and
        the hub segments after them (two launches of the same schedule's
        position ranges), then the merge."""

        def __init__(self, plan):
            self.plan = plan

        def edge(self, lib, csr_, pp_, bias_, out):
            p = self.plan
            hubs = csr.hubs
            stream = torch._C._cuda_getCurrentRawStream(dev.index)
            hf4 = (hf + 3) // 4 * 4
            nv = hubs.n_vrows
            st = torch.empty(nv * (hf4 + 2 * H), dtype=torch.float32, device=dev)
            p_acc = st.data_ptr()
            p_ml = p_acc + 4 * nv * hf4
            n_pos = hubs.sched_row.numel()
            ld = hf // p.slices if p.slices > 1 else p.hfp
            for lo, hi in ((nv, n_pos), (0, nv)):
                rc = lib.gat_edge_aggregate_seg(
                    hubs.sched_b.data_ptr(), hubs.sched_e.data_ptr(), 1, csr.col.data_ptr(),
                    hubs.sched_row.data_ptr(), lo, hi, p.p_wh, ld, n, p.slices,
                    pp.a_src.data_ptr(), pp.c_src.data_ptr(), p.p_sd, H, F, int(w.concat), 0.2,
                    p_acc, p_ml, 0, nv, bias.data_ptr(), out.data_ptr(), p.khint, stream)
                _lib.check(rc, "hub-last seg")
            # the segment slot map (GAT_HUB_ORDER=src reorders the segments)
            slot = 0 if hubs.seg_slot is None else hubs.seg_slot.data_ptr()
            rc = lib.gat_edge_merge_ex(hubs.hub_rows.data_ptr(), hubs.hub_vptr.data_ptr(), slot,
                                       hubs.n_hub, p_acc, p_ml, H, F, int(w.concat),
                                       bias.data_ptr(), out.data_ptr(), 0, 0, stream)
            _lib.check(rc, "merge")
            return out

        def kernel_name(self):
            return "hub segments last: " + self.plan.kernel_name()

    def plan_for(env):
        env = dict(env)
        from atmlgraphattentionnetworks_amd import graph as _graph
        _graph._sched_cache.clear()  # the scheduled copy is built under each variant's knobs
        _graph._rot_cache.clear()  # and the rotated col
        if int(env.pop("hublast", "0")):
            apply(env)
            plan = ForwardPlan(x, csr, w.heads, w.out_channels, w.concat, 0.2)
            plan.project(lib, x, pp)
            plan = HubLast(plan)
            plan_out[id(plan)] = torch.empty(n, hf if w.concat else F, device=dev)
            return plan
        windows = int(env.pop("passes", "0"))
        sched = int(env.pop("sched", "0"))
        hubseg = int(env.pop("hubseg", "0"))
        apply(env)
        if hubseg:
            plan = HubSeg(hubseg)
            plan_out[id(plan)] = torch.empty(n, hf if w.concat else F, device=dev)
            return plan
        plan = ForwardPlan(x, csr, w.heads, w.out_channels, w.concat, 0.2)
        plan.project(lib, x, pp)
        if windows > 1:
            plan = Passes(plan, windows)
        elif sched:
            plan = Sched(plan)
        plan_out[id(plan)] = torch.empty(n, hf if w.concat else F, device=dev)
        return plan

    with torch.no_grad():
        if args.only >= 0:
            plan = plan_for(envs[args.only])
            apply(knob_envs[args.only])
            for _ in range(args.iters):
                plan.edge(lib, csr, pp, bias, plan_out[id(plan)])
            torch.cuda.synchronize()
            print(json.dumps({"variant": specs[args.only], "kernel": plan.kernel_name()}))
            return
        plans = [plan_for(e) for e in envs]
        res = {s: [] for s in specs}
        lres = {s: [] for s in specs}
        outs = {}
        for _ in range(args.rounds):
            for s, env, plan in zip(specs, knob_envs, plans):
                apply(env)
                o = plan_out[id(plan)]
                res[s].append(time_fn(lambda: plan.edge(lib, csr, pp, bias, o), args.iters))
                outs[s] = o.clone()
                if args.layer:
                    lres[s].append(time_fn(
                        lambda: gat_forward(x, csr, pp, bias, w.heads, w.out_channels, w.concat,
                                            0.2), args.iters))
        apply({})
    ref = outs[specs[0]]
    summary = {}
    for s in specs:
        med = statistics.median(res[s])
        d = {"edge_median_ms": round(med, 5), "edge_min_ms": round(min(res[s]), 5),
             "edges_per_s": csr.num_edges / med * 1e3,
             "max_abs_diff_vs_first": float((outs[s] - ref).abs().max()),
             "kernel": plans[specs.index(s)].kernel_name()}
        if args.layer:
            d["layer_median_ms"] = round(statistics.median(lres[s]), 5)
        summary[s] = d
    print(json.dumps({"workload": args.workload, "N": n, "E'": csr.num_edges,
                      "max_abs_ref": float(ref.abs().max()), "results": summary}, indent=1))


if __name__ == "__main__":
    main()
