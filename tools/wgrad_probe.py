#!/usr/bin/env python3
"""dW = dWh^T x (K = N rows) formulations, timed with events: hipBLASLt
picks poorly for the very long K of a weight gradient."""
import sys
import torch


def t(fn, it=50):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


for n, hf, fin in [(44906, 64, 50), (232965, 64, 602), (169343, 64, 128), (2708, 64, 1433)]:
    dwh = torch.randn(n, hf, device="cuda")
    x = torch.randn(n, fin, device="cuda")
    ref = dwh.t().mm(x)
    res = {"mm(dwh.t, x)": t(lambda: dwh.t().mm(x)),
           "mm(x.t, dwh).t": t(lambda: x.t().mm(dwh))}
    for s in (16, 64, 256):
        m = (n + s - 1) // s * s
        dp = torch.zeros(m, hf, device="cuda"); dp[:n] = dwh
        xp = torch.zeros(m, fin, device="cuda"); xp[:n] = x
        f = lambda: torch.bmm(dp.view(s, m // s, hf).transpose(1, 2), xp.view(s, m // s, fin)).sum(0)
        assert torch.allclose(f(), ref, rtol=1e-3, atol=1e-2)
        res[f"bmm split {s}"] = t(f)
    print(n, hf, fin, {k: round(v, 1) for k, v in res.items()}, flush=True)
