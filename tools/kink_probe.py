import sys, os, torch
sys.path.insert(0, os.getcwd())
from atmlgraphattentionnetworks_amd import GraphAttentionLayer, _lib, tuning
from atmlgraphattentionnetworks_amd.graph import get_csr
from atmlgraphattentionnetworks_amd.synthetic import WORKLOADS, make_inputs
w = WORKLOADS["arxiv"]; dev = torch.device("cuda", 0)
x, ei = make_inputs(w, dev); torch.manual_seed(0)
layer = GraphAttentionLayer(w.in_channels, w.out_channels, num_heads=w.heads, concat=w.concat).to(dev)
csr = get_csr(ei, x.size(0)); pp = layer.packed(); lib = _lib.load()
n = x.size(0); H, F = w.heads, w.out_channels; hf = H * F
for x3 in ("0", "1"):
    os.environ["GAT_PROJ_X3"] = x3; tuning.reload()
    wh = torch.empty(n, hf, device=dev); ss = torch.empty(n, H, device=dev); sd = torch.empty(n, H, device=dev)
    rc = lib.gat_project(x.data_ptr(), n, w.in_channels, pp.w.data_ptr(), pp.b.data_ptr(), pp.a_src.data_ptr(), pp.c_src.data_ptr(), pp.a_dst.data_ptr(), pp.c_dst.data_ptr(), H, F, wh.data_ptr(), hf, ss.data_ptr(), H, sd.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ss_re = (wh.view(n, H, F) * pp.a_src.view(1, H, F)).sum(-1) + pp.c_src.view(1, H)
    rp = csr.rowptr.long(); deg = rp[1:] - rp[:-1]
    tgt = torch.repeat_interleave(torch.arange(n, device=dev), deg); src = csr.col.long()
    z1 = sd[tgt] + ss[src]; z2 = sd[tgt] + ss_re[src]
    flips = int(((z1 > 0) != (z2 > 0)).sum())
    print("x3", x3, "max|ss-ss_re|", float((ss - ss_re).abs().max()), "sign flips", flips,
          "|z|<1e-6:", int((z1.abs() < 1e-6).sum()), flush=True)
