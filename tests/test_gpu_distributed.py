"""The sharded (node-range partitioned) forward's HIP path on ONE GPU: P
ShardedGAT ranks in one process, the all-gather emulated by copying every
rank's projected slot into every rank's packed table.  Covers the kernels on
the packed [Wh | s_src] layout with remapped (table-row) column ids and row
slices; the RCCL collective itself runs in bench.py --gpus N."""
import pytest
import torch

from oracle import gat_layer_forward_from_state, init_reference_params

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("P", [2, 4, 8])
@pytest.mark.parametrize("exchange", ["allgather", "replicate"])
@pytest.mark.parametrize("concat", [True, False])
def test_sharded_hip_path_matches_single_gpu(P, exchange, concat):
    from atmlgraphattentionnetworks_amd import GraphAttentionLayer, get_csr
    from atmlgraphattentionnetworks_amd.distributed import ShardedGAT
    from atmlgraphattentionnetworks_amd.synthetic import uniform_graph
    dev = torch.device("cuda", 0)
    n, e, fin, H, F = 3000, 60000, 50, 8, 8
    state = init_reference_params(fin, F, H, concat, seed=1)
    state["bias"] = torch.randn(state["bias"].shape)
    layer = GraphAttentionLayer(fin, F, num_heads=H, concat=concat)
    layer.load_state_dict(state)
    layer = layer.to(dev).eval()
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    x = torch.randn(n, fin, generator=g, device=dev)
    ei = uniform_graph(n, e, seed=4, device=dev)
    csr = get_csr(ei, n)
    with torch.no_grad():
        ranks = [ShardedGAT(layer, csr, P, r, exchange=exchange) for r in range(P)]
        for sh in ranks:
            sh.phase_project(sh.local_x(x))
        if exchange == "allgather":
            m = ranks[0].rows_per_part
            for dst in ranks:
                for src in ranks:
                    sl = slice(src.rank * m, (src.rank + 1) * m)
                    dst.table.buf[sl] = src.table.buf[sl]
        outs = [sh.phase_edges().clone() for sh in ranks]
    full = torch.cat(outs).cpu()
    ref = gat_layer_forward_from_state(state, x.cpu(), ei.cpu(), H, concat)
    torch.testing.assert_close(full, ref, atol=1e-5, rtol=1e-5)
