#!/usr/bin/env python3
"""Accuracy of a 120k-edge hub row: ours (split / unsplit) and the reference's
own fp32 path (the oracle) against float64."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from atmlgraphattentionnetworks_amd import tuning  # noqa: E402
from oracle import gat_layer_forward_from_state  # noqa: E402
from test_gpu_hubs import _hub_case, _layer  # noqa: E402

DEV = torch.device("cuda", 0)
from atmlgraphattentionnetworks_amd.graph import csr_cache  # noqa: E402

x, ei, state = _hub_case(4000, 80000, [(17, 120_000)], 50, 8, 8, True, seed=11)
layer = _layer(state, 50, 8, 8, True)
with torch.no_grad():
    out = layer(x.to(DEV), ei.to(DEV)).cpu()
os.environ["GAT_HUB_SPLIT"] = "0"
tuning.reload()
csr_cache.clear()
with torch.no_grad():
    out_nosplit = layer(x.to(DEV), ei.to(DEV)).cpu()
ref32 = gat_layer_forward_from_state(state, x, ei, 8, True)
st64 = {k: v.double() for k, v in state.items()}
ref64 = gat_layer_forward_from_state(st64, x.double(), ei, 8, True)
for name, t in [("split", out), ("unsplit", out_nosplit), ("ref32", ref32)]:
    d = (t.double() - ref64).abs()
    print(f"{name:8s} row17 max|err| vs f64 {float(d[17].max()):.3e}  other rows {float(d[torch.arange(4000) != 17].max()):.3e}")
print("row17 |ref64| max", float(ref64[17].abs().max()))
