"""Shared timing helper for the tools' interleaved A/Bs."""
import torch


def time_fn(fn, iters, reps=3):
    """Average GPU time per call: `iters` calls captured in one HIP graph and
    replayed, so host launch overhead does not leak into short kernels."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        g.replay()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / (iters * reps)
