#!/usr/bin/env python3
"""One-line summaries of A/B result files (edge_ab / proj_ab / emu_probe JSON,
tolerating non-JSON lines before the object)."""
import json
import sys


def load(path):
    txt = open(path).read()
    return json.loads(txt[txt.index("{"):])


for path in sys.argv[1:]:
    try:
        d = load(path)
    except (OSError, ValueError) as exc:
        print(path, "unreadable:", exc)
        continue
    res = d.get("results", {})
    parts = []
    for k, v in res.items():
        if "edge_median_ms" in v:
            parts.append(f"{k}: {v['edge_median_ms'] * 1e3:.2f} us (diff {v['max_abs_diff_vs_first']:.1e})")
        elif "median_ms" in v:
            parts.append(f"{k}: {v['median_ms'] * 1e3:.2f} us")
        elif "max_edge_passes_us" in v:
            parts.append(f"{k}: proj {v['max_project_us']:.1f} edge {v['max_edge_passes_us']:.1f}")
        else:
            parts.append(f"{k}: {v}")
    print(path.split("/")[-1], "|", d.get("workload", ""))
    for p in parts:
        print("   ", p)
