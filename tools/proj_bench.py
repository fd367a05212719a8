#!/usr/bin/env python3
"""Projection kernel timing over shapes x knob variants (gat_project_ex with its
workspace; interleaved rounds, each measurement a captured HIP graph of --iters launches), outputs checked
bitwise against the first variant (or within 1e-5 of it when a variant
changes the arithmetic, e.g. another kernel).

Shapes: a workload name (synthetic.WORKLOADS) or NAME@ROWS for its first
ROWS rows (a rank's share of the partitioned step, e.g. reddit@29120 at P = 8).
The table layout is the eval forward's (2 column planes at >= 16 edges/row).

    python tools/proj_bench.py --shapes "reddit,reddit@29120,arxiv,ppi" \
        --variants "base" --out gpurun_out/proj_bench.json
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def parse(spec: str) -> dict:
    if spec == "base":
        return {}
    return dict(kv.split("=", 1) for kv in spec.split(",") if kv)


def apply(env: dict, knobs) -> None:
    from atmlgraphattentionnetworks_amd import tuning
    for k in knobs:
        os.environ.pop(k, None)
    os.environ.update(env)
    tuning.reload()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="reddit,reddit@29120,arxiv,ppi")
    ap.add_argument("--variants", default="base")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from atmlgraphattentionnetworks_amd import GraphAttentionLayer, _lib
    from atmlgraphattentionnetworks_amd.synthetic import WORKLOADS, make_inputs
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    specs = [s.strip() for s in args.variants.split(";") if s.strip()]
    envs = [parse(s) for s in specs]
    knobs = sorted({k for e in envs for k in e})
    result = {}
    for shape in [s for s in args.shapes.split(",") if s]:
        name, _, rows = shape.partition("@")
        w = WORKLOADS[name]
        x_full, ei = make_inputs(w, dev)
        del ei
        n_full = x_full.size(0)
        n = int(rows) if rows else n_full
        x = x_full[:n].contiguous()
        del x_full
        torch.manual_seed(0)
        layer = GraphAttentionLayer(w.in_channels, w.out_channels, num_heads=w.heads,
                                    concat=w.concat).to(dev).eval()
        pp = layer.packed()
        H, F = w.heads, w.out_channels
        hf = H * F
        epr = w.num_edges // n_full + 1
        slices = 2 if (hf == 64 and epr >= 16 and w.concat) else 1
        stream = torch.cuda.current_stream()  # (timing events; launches use the current one)
        outs = []
        for e in envs:
            wh = torch.empty(n * ((hf + 3) // 4 * 4), device=dev)
            sd = torch.empty(n * H, device=dev)
            ss = torch.empty(n * H, device=dev)
            outs.append((wh, sd, ss))

        from atmlgraphattentionnetworks_amd.layer import project_workspace
        pws = project_workspace(dev, w.in_channels, H, F)
        wsa = (0, 0) if pws is None else (pws.data_ptr(), pws.numel())

        def launch(i):
            wh, sd, ss = outs[i]
            st = torch.cuda.current_stream().cuda_stream  # the capture stream inside a graph
            args = (x.data_ptr(), n, w.in_channels, pp.w.data_ptr(), pp.b.data_ptr(),
                    pp.a_src.data_ptr(), pp.c_src.data_ptr(), pp.a_dst.data_ptr(),
                    pp.c_dst.data_ptr(), H, F)
            if slices > 1:
                rc = lib.gat_project_ex(*args, slices, wh.data_ptr(), n, 0, H, sd.data_ptr(),
                                        0, 0, *wsa, st)
            else:
                rc = lib.gat_project_ex(*args, 1, wh.data_ptr(), (hf + 3) // 4 * 4,
                                        ss.data_ptr(), H, sd.data_ptr(), 0, 0, *wsa, st)
            if rc:
                raise RuntimeError(f"projection rc={rc}")

        graphs = []
        for i, e in enumerate(envs):
            apply(e, knobs)
            launch(i)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(args.iters):
                    launch(i)
            graphs.append(g)
        torch.cuda.synchronize()
        # correctness against variant 0
        check = {}
        for i in range(1, len(envs)):
            d = max(float((outs[i][k] - outs[0][k]).abs().max()) for k in (0, 1))
            scale = float(outs[0][0].abs().max())
            check[specs[i]] = d
            if not d <= 1e-5 * max(1.0, scale):
                raise RuntimeError(f"{shape} {specs[i]}: max |diff| {d:.3e} vs base")
        times = {s: [] for s in specs}
        for _ in range(args.rounds):
            for i, s in enumerate(specs):
                ev0 = torch.cuda.Event(enable_timing=True)
                ev1 = torch.cuda.Event(enable_timing=True)
                graphs[i].replay()
                ev0.record(stream)
                graphs[i].replay()
                ev1.record(stream)
                ev1.synchronize()
                times[s].append(ev0.elapsed_time(ev1) * 1e3 / args.iters)
        nbytes = 4 * (n * w.in_channels + n * hf + n * H)
        res = {}
        for s in specs:
            us = statistics.median(times[s])
            res[s] = {"us": round(us, 2), "min_us": round(min(times[s]), 2),
                      "TBps": round(nbytes / us / 1e6, 3)}
        result[shape] = {"n": n, "fin": w.in_channels, "slices": slices, "bytes": nbytes,
                         "variants": res, "max_abs_diff_vs_first": check}
        print(json.dumps({shape: result[shape]}), flush=True)
        del graphs, outs, x
        torch.cuda.empty_cache()
    if args.out:
        with open(args.out, "w") as f:
            json.dump(result, f, indent=1)


if __name__ == "__main__":
    main()
