#!/usr/bin/env python3
"""Timing probe for a target-blocked backward source pass: the CSC split into
B sub-CSCs by target block (targets [b*N/B, (b+1)*N/B)), so that each launch
of gat_bwd_sources gathers from 1/B of the per-target table, against one
launch over the whole CSC.  Inputs are random (only the time is read); the
sum of the B launches leaves out the carry of each row's partial sums from
block to block that a real blocked pass would add.

    python tools/bwd_block_probe.py [workload] [B list, comma separated] [prep]

prep (before each timed repetition, outside the timed region): "none";
"writeT" rewrites the whole table (as gat_bwd_targets does just before the
source pass in a training step); "flush" streams 1 GiB through the caches.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    from atmlgraphattentionnetworks_amd import _lib
    from atmlgraphattentionnetworks_amd.graph import build_csr, get_csc
    from atmlgraphattentionnetworks_amd.synthetic import WORKLOADS, make_inputs
    name = sys.argv[1] if len(sys.argv) > 1 else "reddit"
    blocks = [int(b) for b in (sys.argv[2] if len(sys.argv) > 2 else "1,4,8,16,24").split(",")]
    prep = sys.argv[3] if len(sys.argv) > 3 else "none"
    w = WORKLOADS[name]
    dev = torch.device("cuda", 0)
    x, ei = make_inputs(w, dev)
    n = x.size(0)
    del x
    csr = build_csr(ei, n)
    del ei
    csc = get_csc(csr)
    H, F = w.heads, w.out_channels
    hf = H * F
    lib = _lib.load()
    ld_t = _lib.bwd_table_layout(H, F, True)
    parts = _lib.bwd_sources_parts(n, H, F)
    pw = 3 * hf + 2 * H + hf
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    T = 0.1 * torch.randn(n, ld_t, device=dev, generator=g)
    wh = torch.randn(n, hf, device=dev, generator=g)
    ds_dst = torch.randn(n * H, device=dev, generator=g)
    a_src, a_dst = torch.randn(hf, device=dev), torch.randn(hf, device=dev)
    c_src = torch.randn(H, device=dev)
    dwh = torch.empty(n, hf, device=dev)
    part = torch.empty(parts * pw, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    T2 = T.clone()
    junk = torch.empty(1 << 28, device=dev) if prep == "flush" else None

    def do_prep():
        if prep == "writeT":
            T.copy_(T2)
        elif prep == "flush":
            junk.fill_(1.0)
        elif prep != "none":
            raise SystemExit("prep: none | writeT | flush")

    src = torch.repeat_interleave(torch.arange(n, device=dev),
                                  (csc.ptr[1:] - csc.ptr[:-1]).long())

    def launch(ptr, dst, eid, hint):
        rc = lib.gat_bwd_sources(ptr.data_ptr(), dst.data_ptr(), eid.data_ptr(), n,
                                 wh.data_ptr(), hf, T.data_ptr(), ld_t, ds_dst.data_ptr(),
                                 a_src.data_ptr(), c_src.data_ptr(), a_dst.data_ptr(), H, F, 1,
                                 0.2, 0.6, 1234, None, dwh.data_ptr(), hf, part.data_ptr(),
                                 parts, hint, stream)
        _lib.check(rc, "gat_bwd_sources")

    out = {"workload": name, "prep": prep, "N": n, "E_prime": csr.num_edges, "results": {}}
    for B in blocks:
        subs = []
        if B == 1:
            subs.append((csc.ptr, csc.dst, csc.eid, csr.num_edges // n))
        else:
            blk = (csc.dst.long() * B) // n
            for b in range(B):
                m = blk == b
                cnt = torch.bincount(src[m], minlength=n)
                ptr = torch.zeros(n + 1, dtype=torch.int32, device=dev)
                ptr[1:] = torch.cumsum(cnt, 0).int()
                subs.append((ptr, csc.dst[m].contiguous(), csc.eid[m].contiguous(),
                             int(m.sum().item()) // n))
            del blk
        for s in subs:
            launch(*s)
        torch.cuda.synchronize()
        times = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            do_prep()
            e0.record()
            for s in subs:
                launch(*s)
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1))
        times.sort()
        out["results"][str(B)] = {"ms_median": times[2], "ms_min": times[0]}
        print(json.dumps({"B": B, "ms": times[2]}), file=sys.stderr, flush=True)
        del subs
        torch.cuda.empty_cache()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
