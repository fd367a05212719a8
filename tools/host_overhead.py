#!/usr/bin/env python3
"""Host-side cost of one GraphAttentionLayer forward (enqueue only) vs its
GPU time, and a cProfile of the enqueue path."""
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    from atmlgraphattentionnetworks_amd import GraphAttentionLayer
    from atmlgraphattentionnetworks_amd.synthetic import WORKLOADS, make_inputs
    w = WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "ppi"]
    dev = torch.device("cuda", 0)
    x, ei = make_inputs(w, dev)
    layer = GraphAttentionLayer(w.in_channels, w.out_channels, num_heads=w.heads,
                                concat=w.concat).to(dev).eval()
    with torch.no_grad():
        for _ in range(5):
            layer(x, ei)
        torch.cuda.synchronize()
        n = 200
        t0 = time.perf_counter()
        for _ in range(n):
            layer(x, ei)
        t_enq = (time.perf_counter() - t0) / n
        torch.cuda.synchronize()
        t_all = (time.perf_counter() - t0) / n
        print(f"host enqueue per forward: {t_enq * 1e6:.1f} us; wall per forward (GPU-bound "
              f"if larger): {t_all * 1e6:.1f} us")
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(n):
            layer(x, ei)
        pr.disable()
        torch.cuda.synchronize()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
        print(s.getvalue())


if __name__ == "__main__":
    main()
