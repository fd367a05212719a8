#!/usr/bin/env python3
"""Training-step cost of one GraphAttentionLayer (forward with dropout +
backward) on a synthetic workload: wall time per step with torch events, and
— under rocprofv3 --kernel-trace --stats — the per-kernel split.

    python tools/train_probe.py [workload] [steps] [dropout]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    from atmlgraphattentionnetworks_amd import GraphAttentionLayer
    from atmlgraphattentionnetworks_amd.synthetic import WORKLOADS, make_inputs
    name = sys.argv[1] if len(sys.argv) > 1 else "ppi"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    p = float(sys.argv[3]) if len(sys.argv) > 3 else 0.6
    w = WORKLOADS[name]
    dev = torch.device("cuda", 0)
    x, ei = make_inputs(w, dev)
    torch.manual_seed(0)
    layer = GraphAttentionLayer(w.in_channels, w.out_channels, num_heads=w.heads,
                                concat=w.concat, dropout=p).to(dev).train()
    gout = torch.randn(x.size(0), w.heads * w.out_channels if w.concat else w.out_channels,
                       device=dev)

    def step():
        layer.zero_grad(set_to_none=True)
        out = layer(x, ei)
        out.backward(gout)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        step()
    e1.record()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    gpu = e0.elapsed_time(e1) / steps * 1e-3
    # forward-only (training mode, no grad) for the ratio
    with torch.no_grad():
        for _ in range(3):
            layer(x, ei)
        e0.record()
        for _ in range(steps):
            layer(x, ei)
        e1.record()
        torch.cuda.synchronize()
    fwd = e0.elapsed_time(e1) / steps * 1e-3
    n_edges = w.num_edges + x.size(0) if w.kind == "uniform" else ei.size(1) + x.size(0)
    if os.environ.get("TRAIN_PROBE_PROFILE"):
        import cProfile
        import io
        import pstats
        pr = cProfile.Profile()
        torch.cuda.synchronize()
        pr.enable()
        for _ in range(steps):
            step()
        pr.disable()
        torch.cuda.synchronize()
        buf = io.StringIO()
        pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(30)
        print(buf.getvalue(), file=sys.stderr)
    if os.environ.get("TRAIN_PROBE_TORCHPROF"):
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CPU]) as prof:
            for _ in range(steps):
                step()
            torch.cuda.synchronize()
        print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=40),
              file=sys.stderr)
    print(json.dumps({"workload": name, "dropout": p, "steps": steps,
                      "train_step_ms": round(gpu * 1e3, 4), "wall_ms": round(wall * 1e3, 4),
                      "forward_train_ms": round(fwd * 1e3, 4),
                      "train_edges_per_s": n_edges / gpu}))


if __name__ == "__main__":
    main()
