"""The node-partitioned forward's HIP kernels (distributed.py)
on ONE GPU: ``distributed.emulate`` runs P ranks in one process — every
rank's projection into its blocks of its own table, the all-gather emulated
by block copies, every rank's edge passes with the softmax state carried
between passes (gat_edge_aggregate_seg) — and the concatenated output must
match the oracle (small graphs, BASELINE.json's configs in partitioned form)
or the single-GPU forward (full size; that forward is itself checked against
the oracle in test_gpu_parity.py / test_gpu_fullsize.py).

Bar: |sharded - ref| <= 1e-5 + 1e-5 |ref| (fp32; the passes change the
summation order only).  RCCL with N > 1 needs distinct GPUs: the
multi-process path is rehearsed here with two ranks on cuda:0 exchanging
through gloo (test_bench_two_ranks_shared_gpu); the RCCL exchange itself
(CollectiveExchange: async in-place all_gather_into_tensor per chunk, then
wait) runs over a one-rank RCCL group (test_rccl_exchange_one_rank,
test_bench_dist_one_rank_rccl), and over N GPUs in the driver's multi-GPU
bench.
"""
import pytest
import torch

from oracle import gat_layer_forward_from_state, gat_layer_forward_rows, init_reference_params

pytestmark = pytest.mark.gpu

ATOL = RTOL = 1e-5
DEV = torch.device("cuda", 0)


def _layer(fin, F, H, concat, state, act=None):
    from atmlgraphattentionnetworks_amd import GraphAttentionLayer
    from atmlgraphattentionnetworks_amd.layer import GraphAttentionLayerActivationTest
    if act is None:
        layer = GraphAttentionLayer(fin, F, num_heads=H, concat=concat)
    else:
        layer = GraphAttentionLayerActivationTest(fin, F, num_heads=H, concat=concat,
                                                  activation_function=act)
    layer.load_state_dict(state)
    return layer.to(DEV).eval()


def _small_case(concat, n=3000, e=60000, fin=50, H=8, F=8, seed=1):
    from atmlgraphattentionnetworks_amd.synthetic import uniform_graph
    state = init_reference_params(fin, F, H, concat, seed=seed)
    state["bias"] = torch.randn(state["bias"].shape)
    g = torch.Generator(device=DEV)
    g.manual_seed(seed)
    x = torch.randn(n, fin, generator=g, device=DEV)
    ei = uniform_graph(n, e, seed=4, device=DEV)
    return state, x, ei


@pytest.mark.parametrize("P", [2, 4, 8])
@pytest.mark.parametrize("exchange", ["allgather", "replicate"])
@pytest.mark.parametrize("concat", [True, False])
@pytest.mark.parametrize("table", ["default", "row_major"])
@pytest.mark.parametrize("chunks", [1, 3])
def test_sharded_hip_path_matches_oracle(P, exchange, concat, table, chunks, monkeypatch):
    """table=default: at 21 edges per row the concat table is 2 column planes;
    row_major: GAT_WH_SLICES=1 (Wh-only rows).  chunks=3: the all-gather in 3
    chunks and 3 edge passes carrying (m, l, acc)."""
    if table == "row_major":
        monkeypatch.setenv("GAT_WH_SLICES", "1")
    else:
        monkeypatch.delenv("GAT_WH_SLICES", raising=False)
    if exchange == "replicate" and chunks > 1:
        pytest.skip("replicate has no collective to overlap")
    from atmlgraphattentionnetworks_amd import get_csr
    from atmlgraphattentionnetworks_amd.distributed import ShardedGAT, emulate
    state, x, ei = _small_case(concat)
    layer = _layer(50, 8, 8, concat, state)
    csr = get_csr(ei, x.size(0))
    with torch.no_grad():
        sh = ShardedGAT(layer, csr, P, 0, exchange=exchange, chunks=chunks)
        assert sh.slices == (2 if concat and table == "default" else 1)
        if exchange == "allgather":
            assert sh.chunks == chunks
        full = emulate(layer, csr, x, P, exchange=exchange, chunks=chunks).cpu()
    ref = gat_layer_forward_from_state(state, x.cpu(), ei.cpu(), 8, concat)
    torch.testing.assert_close(full, ref, atol=ATOL, rtol=RTOL)


@pytest.mark.parametrize("split", ["1", "2", "4"])
@pytest.mark.parametrize("table", ["default", "row_major"])
@pytest.mark.parametrize("chunks", [1, 3])
def test_sharded_split_rows_match_oracle(split, table, chunks, monkeypatch):
    """GAT_EDGE_SPLIT: 1, 2 or 4 lane groups per row, merged in registers, in
    the segment passes that carry (m, l, acc) across all-gather chunks."""
    monkeypatch.setenv("GAT_EDGE_SPLIT", split)
    if table == "row_major":
        monkeypatch.setenv("GAT_WH_SLICES", "1")
    else:
        monkeypatch.delenv("GAT_WH_SLICES", raising=False)
    from atmlgraphattentionnetworks_amd import get_csr
    from atmlgraphattentionnetworks_amd.distributed import emulate
    state, x, ei = _small_case(True)
    layer = _layer(50, 8, 8, True, state)
    csr = get_csr(ei, x.size(0))
    with torch.no_grad():
        full = emulate(layer, csr, x, 4, exchange="allgather", chunks=chunks).cpu()
    ref = gat_layer_forward_from_state(state, x.cpu(), ei.cpu(), 8, True)
    torch.testing.assert_close(full, ref, atol=ATOL, rtol=RTOL)


@pytest.mark.parametrize("act_name,concat,chunks", [("lrelu0.3", True, 2), ("lrelu0.01", False, 3),
                                                    ("relu", True, 2), ("tanh", True, 1),
                                                    ("logsigmoid", False, 1)])
def test_sharded_score_activation(act_name, concat, chunks):
    """The layer's score activation reaches the shard kernels: LeakyReLU(0.3),
    LeakyReLU(0.01) and ReLU on the fused chunked path, Tanh / LogSigmoid on the
    packed [Wh | s_src] table (one pass)."""
    from atmlgraphattentionnetworks_amd import get_csr
    from atmlgraphattentionnetworks_amd.distributed import emulate
    from oracle import gat_layer_forward_differentiable
    act = {"lrelu0.3": torch.nn.LeakyReLU(0.3), "lrelu0.01": torch.nn.LeakyReLU(0.01),
           "relu": torch.nn.ReLU(), "tanh": torch.nn.Tanh(),
           "logsigmoid": torch.nn.LogSigmoid()}[act_name]
    state, x, ei = _small_case(concat, n=2000, e=40000)
    layer = _layer(50, 8, 8, concat, state, act)
    csr = get_csr(ei, x.size(0))
    with torch.no_grad():
        full = emulate(layer, csr, x, 4, chunks=chunks).cpu()
        ref = gat_layer_forward_differentiable(state, x.cpu(), ei.cpu(), 8, concat,
                                               activation=act)
    torch.testing.assert_close(full, ref, atol=ATOL, rtol=RTOL)


@pytest.mark.parametrize("P", [2, 4, 8])
@pytest.mark.parametrize("chunks", [1, 2])
def test_arxiv_full_size_partitioned(P, chunks):
    """BASELINE.json configs[3] (ogbn-arxiv scale: N=169,343, E=1,166,243,
    Fin=128, H=8, F=8) node-partitioned over P ranks, at full size: equals
    the single-GPU forward (which test_gpu_fullsize.py checks in full against
    the oracle)."""
    from atmlgraphattentionnetworks_amd import GraphAttentionLayer, get_csr
    from atmlgraphattentionnetworks_amd.distributed import emulate
    from atmlgraphattentionnetworks_amd.synthetic import WORKLOADS, make_inputs
    w = WORKLOADS["arxiv"]
    x, ei = make_inputs(w, DEV)
    torch.manual_seed(0)
    layer = GraphAttentionLayer(w.in_channels, w.out_channels, num_heads=w.heads,
                                concat=w.concat).to(DEV).eval()
    with torch.no_grad():
        layer.bias.normal_()
        one = layer(x, ei)
        full = emulate(layer, get_csr(ei, x.size(0)), x, P, chunks=chunks)
    torch.testing.assert_close(full, one, atol=ATOL, rtol=RTOL)


def test_reddit_scale_partitioned_p8():
    """BASELINE.json configs[4] (Reddit scale, 114.8M edges) node-partitioned
    over 8 ranks with the all-gather in 4 chunks: every row equals the
    single-GPU forward, and 4,096 sampled rows plus each rank's first and last
    row equal the oracle evaluated on their complete in-edge sets."""
    from atmlgraphattentionnetworks_amd import GraphAttentionLayer, get_csr
    from atmlgraphattentionnetworks_amd.distributed import ShardedGAT, emulate
    from atmlgraphattentionnetworks_amd.synthetic import WORKLOADS, make_inputs
    w = WORKLOADS["reddit"]
    x, ei = make_inputs(w, DEV)
    state = init_reference_params(w.in_channels, w.out_channels, w.heads, w.concat, seed=0)
    state["bias"] = torch.randn(state["bias"].shape)
    layer = GraphAttentionLayer(w.in_channels, w.out_channels, num_heads=w.heads,
                                concat=w.concat)
    layer.load_state_dict(state)
    layer = layer.to(DEV).eval()
    csr = get_csr(ei, x.size(0))
    with torch.no_grad():
        sh = ShardedGAT(layer, csr, 8, 3, chunks=4)
        assert sh.chunks == 4 and sh.slices == 2
        del sh
        one = layer(x, ei)
        full = emulate(layer, csr, x, 8, chunks=4)
    torch.testing.assert_close(full, one, atol=ATOL, rtol=RTOL)
    from atmlgraphattentionnetworks_amd.distributed import partition_rows
    bounds = partition_rows(csr.rowptr, 8)
    edges_rows = [b for b0 in bounds[:-1] for b in (b0, max(b0 - 1, 0))] + [x.size(0) - 1]
    g = torch.Generator(device="cpu")
    g.manual_seed(321)
    rows = torch.cat([torch.randperm(x.size(0), generator=g)[:4096],
                      torch.tensor(edges_rows)]).unique()
    ref = gat_layer_forward_rows(state, x.cpu(), ei.cpu(), rows, w.heads, w.concat)
    torch.testing.assert_close(full[rows.to(DEV)].cpu(), ref, atol=ATOL, rtol=RTOL)


def _one_line(stdout: str, budget: int = 8000):
    """Exactly one non-empty stdout line, under the driver's parse budget."""
    import json
    lines = [ln for ln in stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, stdout[-2000:]
    assert len(lines[0].encode()) < budget, len(lines[0])
    return json.loads(lines[0])


def test_bench_two_ranks_shared_gpu(tmp_path):
    """bench.py --gpus 2 end to end with 2 torchrun ranks on cuda:0
    (GAT_BENCH_SHARE_GPU0; the all-gather staged through gloo because RCCL
    refuses two ranks on one device): the chunked shared-graph step, the
    max-over-ranks timing, the in-run check of the gathered output against the
    single-GPU forward, and exactly one JSON line on rank 0's stdout."""
    import json
    import os
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, GAT_BENCH_SHARE_GPU0="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
           "--dist-workloads", "ppi,arxiv", "--steps", "6", "--warmup", "2",
           "--detail-out", str(tmp_path / "detail.json")]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _one_line(r.stdout)
    assert line["n_gpus"] == 2 and line["scaling"] == "strong" and line["value"] > 0
    assert line["headline"]["check_max_abs_diff"] is not None
    d = json.load(open(tmp_path / "detail.json"))  # the full detail
    assert d["value"] == line["value"] or abs(d["value"] / line["value"] - 1) < 1e-3
    assert d["steps"] == 6 and d["unit"] == "edges/s"
    assert d["config"]["workload"].startswith("ppi:")  # BASELINE.json's metric workload
    head = d["headline_detail"]
    assert head["check"]["max_abs_diff_vs_one_gpu"] <= 1e-5 + 1e-5 * head["check"]["max_abs_ref"]
    assert set(head["strategy_trials_ms"]) == {"allgather_k1", "allgather_k2", "allgather_k4",
                                               "replicate"}
    # the headline is the north-star design: node-range partition + all-gather
    assert d["config"]["strategy"].startswith("allgather")
    assert head["exchange"] == "allgather" and head["collective_bytes_received_per_rank"] > 0
    rep = d["replicate"]  # reported beside it, never in its place
    assert rep is not None and rep["strategy"] == "replicate"
    assert rep["check"]["max_abs_diff_vs_one_gpu"] <= 1e-5 + 1e-5 * rep["check"]["max_abs_ref"]
    assert d["speedup_vs_one_gpu"] > 0 and d["one_gpu_same_workload"]["value"] > 0
    arx = d["workloads"]["arxiv"]
    assert arx["check"]["max_abs_diff_vs_one_gpu"] <= 1e-5 + 1e-5 * arx["check"]["max_abs_ref"]
    assert d["ppi_blocks_data_parallel"]["value"] > 0
    # the graph path's control flow at world 2: each rank captured its compute
    # (the host-staged exchange is not capturable), the ranks agreed, the
    # replay ran and its gathered output matched the one-GPU forward; a
    # rehearsal value never replaces the step's
    for w in (head, arx):
        g = w["graph"]
        assert g["ok"] and g["compute_only"], g
        assert g["check"]["max_abs_diff_vs_one_gpu"] <= 1e-5 + 1e-5 * g["check"]["max_abs_ref"]
        assert w.get("launch", "eager") == "eager"
    # the reported speed-up compares like with like
    assert d["speedup_launch_mode"] == "eager vs eager"
    assert d["one_gpu_same_workload"]["launch"] == "eager"
    assert d["one_gpu_same_workload"]["graph"]["ok"]


_RCCL_ONE_RANK = r"""
import json, os, sys
sys.path.insert(0, os.getcwd())
import torch, torch.distributed as dist
from atmlgraphattentionnetworks_amd import GraphAttentionLayer, get_csr
from atmlgraphattentionnetworks_amd.distributed import CollectiveExchange, ShardedGAT
from atmlgraphattentionnetworks_amd.synthetic import uniform_graph
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1)
torch.manual_seed(0)
layer = GraphAttentionLayer(50, 8, num_heads=8, concat=True).to(dev).eval()
with torch.no_grad():
    layer.bias.normal_()
x = torch.randn(3000, 50, device=dev)
ei = uniform_graph(3000, 60000, seed=4, device=dev)
csr = get_csr(ei, 3000)
res = {}
with torch.no_grad():
    one = layer(x, ei)
    for k in (1, 3):
        ex = CollectiveExchange(None)
        sh = ShardedGAT(layer, csr, 1, 0, chunks=k, exchanger=ex, force_exchange=True)
        hs = []
        xl = sh.local_x(x)
        for c in range(sh.chunks):
            sh.project_chunk(xl, c)
            hs.append(sh.exchange_start(c))
        assert all(h is not None for h in hs), "exchange_start short-circuited"
        for c in range(sh.chunks):
            sh.exchanger.wait(hs[c])
            sh.edge_pass(c)
        torch.cuda.synchronize()
        res[k] = float((sh.out - one).abs().max())
        res[f"chunks{k}"] = sh.chunks
        res[f"scale{k}"] = float(one.abs().max())
dist.destroy_process_group()
print(json.dumps(res))
"""


def test_rccl_exchange_one_rank():
    """CollectiveExchange over a real RCCL communicator (one rank: the GPU box
    has one GPU): ``new`` nccl process group, the asynchronous in-place
    all_gather_into_tensor of each table chunk, ``wait()`` ordering the edge
    passes after it on torch's stream — with 1 and 3 chunks.  The output must
    equal the single-GPU forward."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _RCCL_ONE_RANK], cwd=root, capture_output=True,
                       text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    for k in ("1", "3"):
        assert d[f"chunks{k}"] == int(k)
        assert d[k] <= 1e-5 + 1e-5 * d[f"scale{k}"], d


def test_bench_dist_one_rank_rccl(tmp_path):
    """``bench.py --dist`` at one rank (no torchrun): the multi-GPU bench path
    with its all-gather strategies issued over a one-rank RCCL group, the
    PPI-shape headline, and the check against the one-GPU forward."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("MASTER_ADDR", "MASTER_PORT", "RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "bench.py", "--dist", "--dist-workloads", "ppi",
                        "--no-weak", "--steps", "6", "--warmup", "2",
                        "--detail-out", str(tmp_path / "detail.json")], cwd=root, env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _one_line(r.stdout)
    for k in ("metric", "value", "ms_per_step", "unit", "scaling"):
        assert k in line, k
    assert line["scaling"] == "strong"
    d = json.load(open(tmp_path / "detail.json"))
    assert d["n_gpus"] == 1 and d["config"]["workload"].startswith("ppi:")
    assert "RCCL" in d["config"]["exchange"]
    head = d["headline_detail"]
    assert set(head["strategy_trials_ms"]) == {"allgather_k1", "allgather_k2", "replicate"}
    assert d["config"]["strategy"].startswith("allgather")
    assert head["collective_ms"] > 0
    assert head["check"]["max_abs_diff_vs_one_gpu"] <= 1e-5 + 1e-5 * head["check"]["max_abs_ref"]
    # the same all-gather step replayed from a captured graph (the RCCL
    # collective recorded in it): captured, timed and checked
    g = head["graph"]
    assert g["ok"], g
    assert g["check"]["max_abs_diff_vs_one_gpu"] <= 1e-5 + 1e-5 * g["check"]["max_abs_ref"]
    # the headline is the faster launch of the same strategy
    assert d["value"] >= g["value"] * (1 - 1e-9)
    og = d["one_gpu_same_workload"]
    assert og["launch"] == "eager" and og["graph"]["ok"]
    # both graph sides hold the same number of steps per replay
    assert g["launch"].startswith(og["graph"]["launch"]), (og["graph"]["launch"], g["launch"])
    if "eager" in head:  # the graph won: its speed-up is over the graphed one-GPU step
        assert d["value"] == g["value"] and d["config"]["launch"].startswith("hipGraph")
        assert d["speedup_launch_mode"] == "hipGraph vs hipGraph"
        assert abs(d["speedup_vs_one_gpu"] / (d["value"] / og["graph"]["value"]) - 1) < 1e-9
    else:
        assert d["speedup_launch_mode"] == "eager vs eager"
        assert abs(d["speedup_vs_one_gpu"] / (d["value"] / og["value"]) - 1) < 1e-9


def test_bench_single_gpu_line(tmp_path):
    """``bench.py`` at N = 1 (extra workloads, PMC, training and the rank
    emulation off, to keep it short): exactly one stdout line under the
    driver's 8 KB budget, carrying the required keys, ``roofline`` and
    ``cpu_baseline``; the full detail goes to the file (a 29.8 KB
    line was not parsed)."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "bench.py", "--workloads", "", "--no-pmc", "--no-train",
                        "--emulate-ranks", "", "--steps", "5", "--warmup", "2",
                        "--detail-out", str(tmp_path / "detail.json")], cwd=root,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _one_line(r.stdout)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in line, k
    assert line["n_gpus"] == 1 and line["steps"] == 5 and line["scaling"] == "strong"
    roof = line["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in roof, k
    assert 0 < roof["frac"] <= 1 and roof["unit"] == "GB/s"
    # SURVEY §8(d)'s no-reuse model beside the compulsory one, from the same kernel time
    assert roof["frac_8d"] > roof["frac"] and roof["achieved_8d"] > roof["achieved"]
    cb = line["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] == "port" and cb["sample"]
    d = json.load(open(tmp_path / "detail.json"))
    assert d["roofline"]["kernel_ms"] > 0


@pytest.mark.parametrize("P,chunks,fin", [(2, 3, 50), (8, 3, 50), (4, 4, 602), (8, 2, 128)])
def test_chunked_projection_equals_per_chunk_launches(P, chunks, fin):
    """gat_project_chunked (one launch for all of a rank's chunk blocks) writes
    exactly what one gat_project_sliced launch per chunk writes: every table
    block bit for bit, s_dst too (including the partial last chunk)."""
    from atmlgraphattentionnetworks_amd import get_csr
    from atmlgraphattentionnetworks_amd.distributed import ShardedGAT
    state, x, ei = _small_case(True, n=5000, e=100000, fin=fin)
    layer = _layer(fin, 8, 8, True, state)
    csr = get_csr(ei, x.size(0))
    with torch.no_grad():
        for rank in range(P):
            sh = ShardedGAT(layer, csr, P, rank, chunks=chunks, pingpong=False)
            assert sh.layout.kind == "planes" and sh.chunks == chunks
            xl = sh.local_x(x)
            sh.table.fill_(float("nan"))
            sh.project_all(xl)
            t1, s1 = sh.table.clone(), sh.s_dst.clone()
            sh.table.fill_(float("nan"))
            sh.s_dst.fill_(float("nan"))
            for c in range(sh.chunks):
                sh.project_chunk(xl, c)
            assert torch.equal(torch.nan_to_num(t1, nan=7.0), torch.nan_to_num(sh.table, nan=7.0))
            assert torch.equal(s1[:sh.n_local], sh.s_dst[:sh.n_local])
