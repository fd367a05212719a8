"""Parity of the HIP path (through the C-ABI) with the reference / oracle.

Bar: fp32, |ours - ref| <= 1e-5 + 1e-5 * |ref| ("within 1e-5
fp32"; summation order differs from the reference's CPU scatter, so the
check is magnitude-aware).  Integer work (the CSR) is bit-exact.
"""
import numpy as np
import pytest
import torch

from conftest import golden_names, load_golden
from oracle import gat_layer_forward_from_state

pytestmark = pytest.mark.gpu

ATOL = 1e-5
RTOL = 1e-5


def dev():
    assert torch.cuda.is_available(), "gpu tests need a ROCm device"
    return torch.device("cuda", 0)


# Every parity case runs on the default kernels AND under each knob the library
# keeps (atmlgraphattentionnetworks_amd/csrc/gat_abi.hip kKnobNames; tuning.PY_KNOBS):
# each forces a product path that a shape or a graph size also reaches, so the
# small cases cover the kernels the full-size graphs run.  The other kernel
# families (projection per Fin and head width, the gathered-score and generic
# edge kernels, odd lane groups) are reached by the shapes in CASES.
VARIANTS = {
    "fast": {},
    # one lane group per row (the full-size launches; row-batched ids where
    # rows average >= 16 in-edges), and four
    "split1": {"GAT_EDGE_SPLIT": "1"},
    "split4": {"GAT_EDGE_SPLIT": "4"},
    # edges per chunk 8 / 16, two float4s per lane, the pipelined long-row kernel
    "u8": {"GAT_EDGE_U": "8", "GAT_EDGE_SPLIT": "1"},
    "u16": {"GAT_EDGE_U": "16"},
    "u16_v2_pipe": {"GAT_EDGE_U": "16", "GAT_EDGE_V": "2"},
    "u16_v2_nopipe": {"GAT_EDGE_U": "16", "GAT_EDGE_V": "2", "GAT_EDGE_PIPE": "0"},
    "v2": {"GAT_EDGE_V": "2", "GAT_EDGE_SPLIT": "1"},
    # short-row col values one chunk ahead instead of 8 chunks per load; the
    # row-batched ids without the lean form's gathers one chunk ahead
    "no_rowcol": {"GAT_EDGE_ROWCOL": "0", "GAT_EDGE_SPLIT": "1"},
    "rowcol1": {"GAT_EDGE_ROWCOL": "1", "GAT_EDGE_SPLIT": "1"},
    # Fin <= 4: projection and edge kernel as two launches instead of the fused
    # small-Fin kernel (the default through gat_layer_forward)
    "no_xproj": {"GAT_EDGE_XPROJ": "0"},
    # the CSR-order launch (short rows take the scheduled copy by default), and
    # the scheduled copy without the staggered sweeps
    "nosched": {"GAT_EDGE_SCHED": "0"},
    "sched_plain": {"GAT_EDGE_SCHED": "plain"},
    # sliced node table (gat_*_sliced); shapes it does not take run row-major
    "sliced2": {"GAT_WH_SLICES": "2"},
}

KNOBS = ("GAT_EDGE_U", "GAT_EDGE_V", "GAT_EDGE_PIPE", "GAT_EDGE_SPLIT", "GAT_EDGE_ROWCOL",
         "GAT_EDGE_XPROJ", "GAT_BWD_KINK", "GAT_BWD_SL", "GAT_BWD_KERNEL", "GAT_WH_SLICES",
         "GAT_HUB_SPLIT", "GAT_HUB_SEG", "GAT_EDGE_SCHED")


@pytest.fixture(params=list(VARIANTS))
def variant(request, monkeypatch):
    for k in KNOBS:
        monkeypatch.delenv(k, raising=False)
    for k, v in VARIANTS[request.param].items():
        monkeypatch.setenv(k, v)
    return request.param


def layer_from_state(state, fin, F, H, concat):
    from atmlgraphattentionnetworks_amd import GraphAttentionLayer
    layer = GraphAttentionLayer(fin, F, num_heads=H, concat=concat)
    layer.load_state_dict(state)
    return layer.to(dev()).eval()


def run_layer(layer, x, ei):
    with torch.no_grad():
        return layer(x.to(dev()), ei.to(dev())).cpu()


@pytest.mark.parametrize("name", golden_names())
def test_golden_fixture(name, variant):
    g = load_golden(name)
    m = g["meta"]
    layer = layer_from_state(g["state"], m["Fin"], m["F"], m["H"], m["concat"])
    out = run_layer(layer, g["x"], g["edge_index"])
    torch.testing.assert_close(out, g["out"], atol=ATOL, rtol=RTOL)


def random_case(n, e, fin, H, F, concat, seed, kind="uniform"):
    from oracle import init_reference_params
    rng = np.random.default_rng(seed)
    if kind == "uniform":
        dst = rng.integers(0, n, size=e)
        src = rng.integers(0, n, size=e)
    elif kind == "hub":  # one node takes half the edges -> many chunks in one row
        dst = np.where(rng.random(e) < 0.5, 0, rng.integers(0, n, size=e))
        src = rng.integers(0, n, size=e)
    else:
        raise ValueError(kind)
    ei = torch.from_numpy(np.stack([src, dst]).astype(np.int64))
    x = torch.from_numpy(rng.standard_normal((n, fin)).astype(np.float32))
    state = init_reference_params(fin, F, H, concat, seed=seed)
    state["bias"] = torch.from_numpy(rng.standard_normal(state["bias"].shape).astype(np.float32))
    return x, ei, state


CASES = [
    # n, e, fin, H, F, concat, kind
    (500, 6000, 50, 8, 8, True, "uniform"),
    (500, 6000, 50, 8, 8, False, "uniform"),
    (300, 4000, 7, 64, 4, True, "uniform"),  # H = 64, HF = 256
    (300, 4000, 7, 64, 4, False, "uniform"),
    (300, 4000, 33, 1, 1, True, "uniform"),  # HF = 1
    (300, 4000, 33, 2, 100, False, "uniform"),  # F > 64 in mean mode
    (300, 4000, 17, 5, 7, True, "uniform"),  # odd H, odd F
    (300, 4000, 17, 16, 16, True, "uniform"),  # HF = 256
    (1000, 20000, 24, 8, 8, True, "hub"),  # ~10k-edge row
    (1000, 20000, 24, 32, 8, False, "hub"),
    (64, 0, 5, 4, 8, True, "uniform"),  # self-loops only
    (1, 0, 3, 2, 2, True, "uniform"),  # a single node
    (700, 9000, 602, 8, 8, True, "uniform"),  # Reddit's Fin
    # pre-split W (Fin > 128, HF 32 / 64): K tails, mean mode
    (500, 5000, 202, 4, 8, True, "uniform"),
    (321, 4000, 138, 8, 8, False, "uniform"),
    # the K-chunked projections (Fin > 128; Fin > 64 with heads of 1-16 columns, F a power of 2): K tails and
    # partial column tiles
    (400, 5000, 65, 4, 8, True, "uniform"),  # one-column tail chunk, NT = 2
    (400, 5000, 130, 2, 4, False, "uniform"),  # HF = 8, NT = 1
    (300, 3000, 129, 3, 8, True, "uniform"),  # HF = 24: a half-used tile
    (300, 3000, 200, 1, 16, True, "uniform"),  # one 16-wide head
    (257, 3000, 128, 8, 8, True, "uniform"),  # rows not a multiple of the 128-row block
    # k_project_wres (64 < Fin <= 128): partial 16-row tiles, NT = 1 / 4
    (333, 4000, 100, 8, 8, True, "uniform"),
    (50, 500, 66, 4, 4, False, "uniform"),
    (700, 9000, 0, 3, 4, True, "uniform"),  # Fin = 0: Wh = bias
    # fin 32 / 64 / 128 with NT = 1, 2, 4 and many tiles per wave (k_project_wres,
    # k_project_wg in the tools-only GAT_AB_KERNELS build)
    (333, 4000, 32, 2, 8, False, "uniform"),
    (1500, 20000, 64, 2, 16, True, "uniform"),
    (60000, 200000, 128, 8, 8, True, "uniform"),
    # k_project_wres with the LDS output tile (heads of 2 columns, 64 < Fin <= 128)
    (300, 3000, 80, 32, 2, True, "uniform"),
    # the K-tiled projection: Fin > 64 with heads of 7 (LDS epilogue) or HF = 128
    # (8 column tiles: shuffle epilogue)
    (300, 3000, 100, 5, 7, True, "uniform"),
    (300, 3000, 100, 8, 16, True, "uniform"),
    # the gathered-score edge kernel (a head's lanes not a power of two: F = 12, 24)
    (400, 8000, 20, 4, 12, True, "uniform"),
    (400, 8000, 20, 2, 24, True, "uniform"),
    # rows of ~40 and ~150 in-edges: U = 8 and the pipelined U = 16, V = 2 kernel by default
    (500, 20000, 40, 8, 8, True, "uniform"),
    (400, 60000, 24, 8, 8, True, "uniform"),
    (400, 60000, 24, 4, 16, True, "uniform"),
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "n%d_e%d_fin%d_h%d_f%d_%s_%s" % (
    c[0], c[1], c[2], c[3], c[4], "cat" if c[5] else "mean", c[6]))
def test_random_vs_oracle(case, variant):
    n, e, fin, H, F, concat, kind = case
    x, ei, state = random_case(n, e, fin, H, F, concat, seed=n + e + H, kind=kind)
    ref = gat_layer_forward_from_state(state, x, ei, H, concat)
    out = run_layer(layer_from_state(state, fin, F, H, concat), x, ei)
    torch.testing.assert_close(out, ref, atol=ATOL, rtol=RTOL)


@pytest.mark.parametrize("n,e,fin,H,F,concat,kind", [
    (3000, 84000, 50, 8, 8, True, "uniform"),    # PPI-like rows, 2 column planes, G = 8
    (5000, 40000, 128, 8, 8, True, "uniform"),   # arxiv-like rows: not row-batched (< 16)
    (2000, 30000, 20, 8, 8, False, "uniform"),   # head mean, row-major, G = 16
    (1500, 30000, 3, 4, 8, True, "uniform"),     # small Fin: the fused projection
    (1500, 60000, 24, 2, 16, True, "hub"),       # a hub row split into segments, U = 8
    (2000, 400000, 24, 8, 8, True, "uniform"),   # ~200 per row: pipelined, not row-batched
])
def test_rowcol_bitwise(n, e, fin, H, F, concat, kind, monkeypatch):
    """Col values loaded 8 chunks per round trip (k_edge_grp RC, the default at
    U = 4 for rows of >= 16 in-edges on average) walk the same chunks with the
    same ids in the same order as the one-chunk-ahead form (GAT_EDGE_ROWCOL=0):
    bitwise equal outputs; and so does the default for rows < 1024
    (GAT_HINT_SHORT: the lean form with the gathers one chunk ahead)."""
    from atmlgraphattentionnetworks_amd import tuning
    from atmlgraphattentionnetworks_amd.graph import csr_cache
    x, ei, state = random_case(n, e, fin, H, F, concat, seed=n + fin, kind=kind)
    outs = []
    arms = ({"GAT_EDGE_ROWCOL": "1"}, {"GAT_EDGE_ROWCOL": "0"}, {})
    for env in arms:
        monkeypatch.delenv("GAT_EDGE_ROWCOL", raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        tuning.reload()
        csr_cache.clear()
        outs.append(run_layer(layer_from_state(state, fin, F, H, concat), x, ei))
    csr_cache.clear()
    assert torch.equal(outs[0], outs[1])  # row-batched ids == one chunk ahead, bit for bit
    # the default (rows < 1024: the lean form with the gathers one chunk ahead)
    # walks the same chunks in the same order; its instance may contract an
    # FMA differently (1 ulp at PPI scale), so it is held to the ulp level
    torch.testing.assert_close(outs[2], outs[0], atol=1e-6, rtol=1e-6)
    if kind == "uniform":  # (a 30k-200k-edge hub row: tests/test_gpu_hubs.py's bar)
        ref = gat_layer_forward_from_state(state, x, ei, H, concat)
        torch.testing.assert_close(outs[0], ref, atol=ATOL, rtol=RTOL)


@pytest.mark.parametrize("n,e", [(3000, 84000)])
def test_rowcol_training_bitwise(n, e, monkeypatch):
    """The training forward (kink sums, k_edge_grp KINK) with the row-batched
    ids (PPI-like rows) against the one-chunk-ahead form: outputs and input
    gradients bitwise equal (no dropout, so both runs draw nothing)."""
    from atmlgraphattentionnetworks_amd import tuning
    from atmlgraphattentionnetworks_amd.graph import csr_cache
    x, ei, state = random_case(n, e, 24, 8, 8, True, seed=n, kind="uniform")
    g = torch.randn(n, 64, generator=torch.Generator().manual_seed(3))
    res = []
    for env in ({}, {"GAT_EDGE_ROWCOL": "0"}):
        monkeypatch.delenv("GAT_EDGE_ROWCOL", raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        tuning.reload()
        csr_cache.clear()
        layer = layer_from_state(state, 24, 8, 8, True)
        xd = x.to(dev()).requires_grad_(True)
        y = layer(xd, ei.to(dev()))
        y.backward(g.to(dev()))
        res.append((y.detach().cpu(), xd.grad.cpu()))
    csr_cache.clear()
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1])


def test_edge_order_invariance_and_determinism():
    x, ei, state = random_case(800, 12000, 20, 8, 8, True, seed=5)
    layer = layer_from_state(state, 20, 8, 8, True)
    a = run_layer(layer, x, ei)
    a2 = run_layer(layer, x, ei.clone())  # fresh CSR build: bitwise reproducible
    assert torch.equal(a, a2)
    perm = torch.from_numpy(np.random.default_rng(0).permutation(ei.size(1)))
    b = run_layer(layer, x, ei[:, perm].contiguous())
    torch.testing.assert_close(a, b, atol=ATOL, rtol=RTOL)


def test_csr_bit_exact():
    from atmlgraphattentionnetworks_amd import build_csr
    rng = np.random.default_rng(7)
    n, e = 5000, 80000
    src = rng.integers(0, n, size=e)
    dst = rng.integers(0, n, size=e)
    ei = torch.from_numpy(np.stack([src, dst]).astype(np.int64))
    csr = build_csr(ei.to(dev()), n)
    # expected: the edges of add_self_loops (loops appended), sorted by (target,
    # source), equal pairs in input order (stable)
    s_all = np.concatenate([src, np.arange(n)])
    d_all = np.concatenate([dst, np.arange(n)])
    order = np.lexsort((s_all, d_all))
    exp_col = s_all[order].astype(np.int32)
    exp_rowptr = np.concatenate([[0], np.cumsum(np.bincount(d_all, minlength=n))]).astype(np.int32)
    assert np.array_equal(csr.rowptr.cpu().numpy(), exp_rowptr)
    assert np.array_equal(csr.col.cpu().numpy(), exp_col)
    assert csr.num_edges == e + n
    # schedule: rows by descending in-degree, ties in row order
    deg = np.diff(exp_rowptr)
    exp_order = np.lexsort((np.arange(n), -deg)).astype(np.int32)
    assert np.array_equal(csr.order.cpu().numpy(), exp_order)


def test_out_of_range_edge_raises():
    from atmlgraphattentionnetworks_amd import GraphAttentionLayer
    layer = GraphAttentionLayer(4, 2, num_heads=2).to(dev()).eval()
    x = torch.randn(5, 4, device=dev())
    bad = torch.tensor([[0, 5], [1, 2]], device=dev())
    with torch.no_grad(), pytest.raises(ValueError):
        layer(x, bad)
    neg = torch.tensor([[0, -1], [1, 2]], device=dev())
    with torch.no_grad(), pytest.raises(ValueError):
        layer(x, neg)


def test_wrong_dtype_and_shape_raise():
    from atmlgraphattentionnetworks_amd import GraphAttentionLayer
    layer = GraphAttentionLayer(4, 2, num_heads=2).to(dev()).eval()
    ei = torch.tensor([[0, 1], [1, 2]], device=dev())
    with torch.no_grad():
        with pytest.raises(ValueError):
            layer(torch.randn(5, 4, device=dev(), dtype=torch.float64), ei)
        with pytest.raises(ValueError):
            layer(torch.randn(5, 3, device=dev()), ei)


def test_csr_cache_reuse():
    from atmlgraphattentionnetworks_amd.graph import csr_cache, get_csr
    csr_cache.clear()
    ei = torch.randint(0, 100, (2, 500), device=dev())
    a = get_csr(ei, 100)
    b = get_csr(ei, 100)
    assert a is b
    ei[0, 0] = (ei[0, 0] + 1) % 100  # in-place edit bumps the version -> rebuild
    c = get_csr(ei, 100)
    assert c is not a


@pytest.mark.parametrize("graph", ["uniform", "hubs"])
def test_cached_plan_pingpong_repeated_forwards(graph):
    """The layer's cached plan alternates two workspaces (layer.ForwardPlan
    pingpong): back-to-back forwards with different x give each x's own
    result, bitwise equal whenever x repeats, and equal to the oracle."""
    from atmlgraphattentionnetworks_amd.synthetic import powerlaw_graph, uniform_graph
    from oracle import init_reference_params
    torch.manual_seed(5)
    n, fin, H, F = 3000, 50, 8, 8
    if graph == "uniform":
        ei = uniform_graph(n, 60_000, seed=4, device=dev())
    else:
        ei = powerlaw_graph(n, 60_000, seed=4, device=dev())
    state = init_reference_params(fin, F, H, True, seed=1)
    layer = layer_from_state(state, fin, F, H, True)
    xa, xb = torch.randn(n, fin, device=dev()), torch.randn(n, fin, device=dev())
    with torch.no_grad():
        outs = [layer(x, ei).clone() for x in (xa, xb, xa, xb, xa)]
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[2]) and torch.equal(outs[0], outs[4])
    assert torch.equal(outs[1], outs[3])
    for x, out in ((xa, outs[0]), (xb, outs[1])):
        ref = gat_layer_forward_from_state(state, x.cpu(), ei.cpu(), H, True)
        torch.testing.assert_close(out.cpu(), ref, atol=ATOL, rtol=RTOL)


def test_ppi_shape_full_size_vs_oracle():
    """BASELINE config 2 at full size (N=44,906, E=1,226,368, Fin=50, H=8, F=8)."""
    from atmlgraphattentionnetworks_amd.synthetic import WORKLOADS, make_inputs
    from oracle import init_reference_params
    w = WORKLOADS["ppi"]
    x, ei = make_inputs(w, dev())
    state = init_reference_params(w.in_channels, w.out_channels, w.heads, w.concat, seed=0)
    out = run_layer(layer_from_state(state, w.in_channels, w.out_channels, w.heads, w.concat),
                    x, ei)
    ref = gat_layer_forward_from_state(state, x.cpu(), ei.cpu(), w.heads, w.concat)
    torch.testing.assert_close(out, ref, atol=ATOL, rtol=RTOL)


@pytest.mark.parametrize("slices,H,F,fin", [(2, 8, 8, 50), (2, 8, 8, 602), (8, 8, 8, 50),
                                            (4, 8, 8, 50), (2, 4, 8, 3), (4, 4, 8, 128),
                                            (8, 8, 8, 602), (3, 3, 8, 20), (4, 4, 16, 50),
                                            (2, 16, 4, 50), (2, 4, 16, 128)])
def test_sliced_table_equals_row_major(slices, H, F, fin, monkeypatch):
    """gat_project_sliced + gat_edge_aggregate_sliced take this shape (status 0,
    checked directly) and give the row-major path's output bit for bit: the
    same per-lane arithmetic on a different table layout."""
    from atmlgraphattentionnetworks_amd import _lib
    from atmlgraphattentionnetworks_amd.layer import wh_slices
    n, e = 1500, 30000
    x, ei, state = random_case(n, e, fin, H, F, True, seed=slices * 100 + H)
    layer = layer_from_state(state, fin, F, H, True)
    # one lane group per row in both layouts (the two-group split of small
    # launches applies to some lane-group widths only, and regroups the sums)
    monkeypatch.setenv("GAT_EDGE_SPLIT", "1")
    # planes narrower than 16 columns run lane groups of 1-2 lanes, which the
    # library instantiates at 8 edges per chunk only: the row-major run then
    # takes 8 too (the same chunks, so still bit for bit)
    if H * F // slices < 16:
        monkeypatch.setenv("GAT_EDGE_U", "8")
    # the row-batched ids of the non-lean instances (the lean default's
    # instance may contract an FMA differently: DESIGN.md §3.2)
    monkeypatch.setenv("GAT_EDGE_ROWCOL", "1")
    monkeypatch.setenv("GAT_WH_SLICES", str(slices))
    assert wh_slices(H, F, True, 0.2) == slices
    pp = layer.packed()
    xd = x.to(dev())
    wh = torch.empty(n * H * F, device=dev())
    ss = torch.empty(n * H, device=dev())
    sd = torch.empty(n * H, device=dev())
    lib = _lib.load()
    rc = lib.gat_project_sliced(xd.data_ptr(), n, fin, pp.w.data_ptr(), pp.b.data_ptr(),
                                pp.a_src.data_ptr(), pp.c_src.data_ptr(), pp.a_dst.data_ptr(),
                                pp.c_dst.data_ptr(), H, F, slices, wh.data_ptr(), n,
                                ss.data_ptr(), H, sd.data_ptr(),
                                torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    a = run_layer(layer, x, ei)
    monkeypatch.setenv("GAT_WH_SLICES", "1")
    b = run_layer(layer, x, ei)
    assert torch.equal(a, b)
    ref = gat_layer_forward_from_state(state, x, ei, H, True)
    torch.testing.assert_close(a, ref, atol=ATOL, rtol=RTOL)
    # the planes hold the row-major table's columns
    wh_rm = torch.empty(n, H * F, device=dev())
    rc = lib.gat_project(xd.data_ptr(), n, fin, pp.w.data_ptr(), pp.b.data_ptr(),
                         pp.a_src.data_ptr(), pp.c_src.data_ptr(), pp.a_dst.data_ptr(),
                         pp.c_dst.data_ptr(), H, F, wh_rm.data_ptr(), H * F, ss.data_ptr(), H,
                         sd.data_ptr(), torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    sw = H * F // slices
    planes = wh.view(slices, n, sw)
    for g in range(slices):
        assert torch.equal(planes[g], wh_rm[:, g * sw:(g + 1) * sw])


def test_sliced_entry_points_reject_unsupported_shapes():
    from atmlgraphattentionnetworks_amd import _lib
    lib = _lib.load()
    st = torch.cuda.current_stream().cuda_stream
    buf = torch.zeros(4096, device=dev())
    p = buf.data_ptr()
    # hf % slices != 0, slices < 2, plane width not a multiple of 4
    assert lib.gat_edge_aggregate_sliced(p, p, 0, 0, 1, p, 1, 3, p, p, p, 2, 8, 0.2, p, p, 0,
                                         st) == _lib.GAT_EINVAL
    assert lib.gat_edge_aggregate_sliced(p, p, 0, 0, 1, p, 1, 1, p, p, p, 2, 8, 0.2, p, p, 0,
                                         st) == _lib.GAT_EINVAL
    assert lib.gat_project_sliced(p, 1, 4, p, p, p, p, p, p, 4, 2, 4, p, 1, p, 4, p,
                                  st) == _lib.GAT_EINVAL
    # planes shorter than the rows written
    assert lib.gat_project_sliced(p, 8, 4, p, p, p, p, p, p, 8, 8, 2, p, 4, p, 8, p,
                                  st) == _lib.GAT_EINVAL
    # planes splitting a head (sw % f != 0) and a slope outside [0, 1]
    assert lib.gat_edge_aggregate_sliced(p, p, 0, 0, 1, p, 1, 4, p, p, p, 2, 8, 0.2, p, p, 0,
                                         st) == _lib.GAT_EUNSUPPORTED
    assert lib.gat_edge_aggregate_sliced(p, p, 0, 0, 1, p, 1, 2, p, p, p, 2, 8, -0.5, p, p, 0,
                                         st) == _lib.GAT_EUNSUPPORTED
    # fin > 64 needs the pipelined projection: f a power of two <= 16, hf <= 64
    assert lib.gat_project_sliced(p, 1, 100, p, p, p, p, p, p, 8, 12, 2, p, 1, p, 8, p,
                                  st) == _lib.GAT_EUNSUPPORTED


def test_sliced_default_with_unaligned_x_view():
    """x as a row view that starts off a 16-B boundary (fin = 50): the whole-K
    projection that writes the sliced table needs 16-B aligned rows, so the
    layer falls back to the row-major path; results still match the oracle."""
    from atmlgraphattentionnetworks_amd import _lib
    n, e, fin, H, F = 1500, 30000, 50, 8, 8
    x, ei, state = random_case(n + 1, e, fin, H, F, True, seed=11)
    layer = layer_from_state(state, fin, F, H, True)
    xd = x.to(dev())[1:]                 # 200-B offset
    assert xd.data_ptr() % 16 != 0
    ei = ei[:, (ei[0] >= 1) & (ei[1] >= 1)] - 1
    with torch.no_grad():
        out = layer(xd, ei.to(dev())).cpu()
    ref = gat_layer_forward_from_state(state, x[1:], ei, H, True)
    torch.testing.assert_close(out, ref, atol=ATOL, rtol=RTOL)
    # the sliced projection itself refuses the unaligned rows (nothing launched)
    pp = layer.packed()
    wh = torch.empty(2 * n * 32, device=dev())
    sd = torch.empty(n * H, device=dev())
    lib = _lib.load()
    rc = lib.gat_project_sliced(xd.data_ptr(), n, fin, pp.w.data_ptr(), pp.b.data_ptr(),
                                pp.a_src.data_ptr(), pp.c_src.data_ptr(), pp.a_dst.data_ptr(),
                                pp.c_dst.data_ptr(), H, F, 2, wh.data_ptr(), n, None, H,
                                sd.data_ptr(), torch.cuda.current_stream().cuda_stream)
    assert rc == _lib.GAT_EUNSUPPORTED


@pytest.mark.parametrize("fin,heads", [(602, 8), (138, 4), (202, 8), (200, 8), (201, 4)])
@pytest.mark.parametrize("chunks", [1, 3])
def test_projection_presplit_bitwise(fin, heads, chunks):
    """gat_project_ex with its workspace (W split once per launch into bf16
    planes, k_split_w: 2-float x rows, 2 or 4 column tiles) equals the
    per-workgroup split bitwise (the same exact 3-term split), for row-major
    and planes tables, one launch over row chunks included; without a
    workspace, or with one too small, it takes the per-workgroup split.
    4-float rows (200) and 1-float rows (201) never pre-split: all four calls
    run the same kernel."""
    from atmlgraphattentionnetworks_amd import GraphAttentionLayer, _lib
    from atmlgraphattentionnetworks_amd.layer import project_workspace
    d = dev()
    torch.manual_seed(1)
    F, n = 8, 1000
    hf = heads * F
    layer = GraphAttentionLayer(fin, F, num_heads=heads, concat=True).to(d).eval()
    pp = layer.packed()
    x = torch.randn(n, fin, device=d)
    ws = project_workspace(d, fin, heads, F)
    assert ws is not None and ws.numel() == 3 * hf * ((fin + 63) // 64 * 64) * 2
    lib = _lib.load()
    for slices in (1, 2):
        if chunks > 1 and slices == 1:
            continue  # row chunks are a planes-table form
        crows = ((n + chunks - 1) // chunks + 63) // 64 * 64 if chunks > 1 else 0
        outs = []
        for wsa in ((ws.data_ptr(), ws.numel()), (0, 0), (ws.data_ptr(), ws.numel() - 16)):
            # row chunk c of ``crows`` rows goes to block c of (n rounded) rows
            blk = crows if crows else n
            nblk = (n + blk - 1) // blk
            wh = torch.full((nblk * blk * hf + 64,), float("nan"), device=d)
            ss = torch.full((n * heads,), float("nan"), device=d)
            sd = torch.full((n * heads,), float("nan"), device=d)
            ld = blk if slices > 1 else hf
            jump = blk * hf if crows else 0
            rc = lib.gat_project_ex(x.data_ptr(), n, fin, pp.w.data_ptr(), pp.b.data_ptr(),
                                    pp.a_src.data_ptr(), pp.c_src.data_ptr(), pp.a_dst.data_ptr(),
                                    pp.c_dst.data_ptr(), heads, F, slices, wh.data_ptr(), ld,
                                    0 if slices > 1 else ss.data_ptr(), heads, sd.data_ptr(),
                                    crows, jump, *wsa, torch.cuda.current_stream().cuda_stream)
            _lib.check(rc, "gat_project_ex")
            torch.cuda.synchronize()
            outs.append((wh.cpu(), sd.cpu(), ss.cpu()))
        for o in outs[1:]:
            for a, b in zip(outs[0], o):
                assert torch.equal(a.nan_to_num(7.0), b.nan_to_num(7.0))
        if slices == 1 and crows == 0:
            # and it is the reference's per-head fp32 Linears (GAT.py:43-45)
            with torch.no_grad():
                ref = torch.cat([torch.nn.functional.linear(x, layer.ws[h].weight,
                                                            layer.ws[h].bias)
                                 for h in range(heads)], 1).cpu()
            torch.testing.assert_close(outs[0][0][:n * hf].view(n, hf), ref,
                                       atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("fin,H,F,unaligned", [
    (50, 8, 8, False),    # k_project_wk (direct epilogue)
    (50, 8, 8, True),     # k_project (K-tiled: x not 16-B aligned)
    (128, 8, 8, False),   # k_project_wres_d
    (100, 8, 8, False),
    (200, 8, 8, False),   # k_project_x3, 4-float rows
    (602, 8, 8, False),   # k_project_x3 on pre-split W
    (130, 8, 8, True),    # K-tiled, Fin > 128
    (128, 32, 2, False),  # k_project_wres (LDS output tile)
    (100, 32, 2, False),
], ids=["wk", "tiled50", "wres_d128", "wres_d100", "x3_200", "x3_602", "tiled130", "wres128",
        "wres100"])
def test_projection_non_finite_inputs(fin, H, F, unaligned):
    """Non-finite x (include/gat_amd.h, gat_project): rows without a
    non-finite value are unaffected (no leak into other rows through clamped
    or padded loads), and the rows with one equal the reference's fp32
    ``Linear`` (GAT.py:43-45) — +Inf, -Inf and NaN in the same places, for the
    fp32-MFMA kernels (fin <= 64, the K-tiled one) and the split-bf16 ones
    (fin > 64), whose correction products of an infinite x are dropped
    (split_sum)."""
    from atmlgraphattentionnetworks_amd import GraphAttentionLayer
    from atmlgraphattentionnetworks_amd.layer import alloc_table, project
    d = dev()
    torch.manual_seed(0)
    n = 700
    layer = GraphAttentionLayer(fin, F, num_heads=H, concat=True).to(d).eval()
    x = torch.randn(n, fin, device=d)
    clean = x.clone()
    if unaligned:  # views 4 bytes past a 256-B boundary: the library takes k_project
        x = torch.empty(n * fin + 1, device=d)[1:].view(n, fin).copy_(x)
        clean = torch.empty(n * fin + 1, device=d)[1:].view(n, fin).copy_(clean)
    bad_rows = [0, 17, 351, 500, n - 1]
    x[0, 3] = float("inf")
    x[17, fin - 1] = float("-inf")
    x[351, fin // 2] = float("nan")
    x[500, 1] = float("inf")
    x[500, fin - 2] = float("-inf")  # Inf - Inf: NaN in the reference
    x[n - 1, 0] = float("inf")
    pp = layer.packed()
    with torch.no_grad():
        t_bad, sd_bad = project(x, pp, H, F, table=alloc_table(n, H, F, d))
        t_ok, sd_ok = project(clean, pp, H, F, table=alloc_table(n, H, F, d))
    good = torch.ones(n, dtype=torch.bool, device=d)
    good[bad_rows] = False
    assert torch.equal(t_bad.wh[good], t_ok.wh[good])
    assert torch.equal(sd_bad[good], sd_ok[good])
    # the reference's own per-head Linears on the host, fp32 (GAT.py:43-45)
    lin = torch.nn.functional.linear
    xc = x.cpu()

    def host(p):
        return p.detach().cpu()
    with torch.no_grad():
        wh_ref = torch.cat([lin(xc, host(layer.ws[h].weight), host(layer.ws[h].bias))
                            for h in range(H)], 1)
        sd_ref = torch.cat([lin(wh_ref[:, h * F:(h + 1) * F], host(layer.attentions2[h].weight),
                                host(layer.attentions2[h].bias)) for h in range(H)], 1)
    ours = t_bad.wh[:, :H * F].cpu()
    for r in bad_rows:
        assert not bool(torch.isfinite(wh_ref[r]).any())
        torch.testing.assert_close(ours[r], wh_ref[r], equal_nan=True, atol=0, rtol=0)
        # s_dst: non-finite in the same places with the same infinities
        a, b = sd_bad[r].cpu(), sd_ref[r]
        assert torch.equal(torch.isnan(a), torch.isnan(b)), (r, a, b)
        assert torch.equal(a[torch.isinf(b)], b[torch.isinf(b)]), (r, a, b)


@pytest.mark.parametrize("edges", [60000, 400000])
def test_layer_copy_and_pickle_after_eval_forward(edges):
    """the eval forward's cached plans (workspaces, raw device
    pointers, the bound ctypes call) live in a side table keyed weakly by the
    layer, not in its __dict__: deepcopy and pickle of a layer that has run
    work, the copies own their workspaces (the original freed first), and a
    cached plan does not keep the graph alive.  Short rows (the bound
    gat_layer_forward call) and long rows (the sliced table)."""
    import copy
    import gc
    import pickle
    import weakref
    from atmlgraphattentionnetworks_amd import GraphAttentionLayer, get_csr
    from atmlgraphattentionnetworks_amd.layer import _eval_plans
    from atmlgraphattentionnetworks_amd.synthetic import uniform_graph
    d = dev()
    torch.manual_seed(0)
    n = 3000
    layer = GraphAttentionLayer(50, 8, num_heads=8, concat=True).to(d).eval()
    with torch.no_grad():
        layer.bias.normal_()
    x = torch.randn(n, 50, device=d)
    ei = uniform_graph(n, edges, seed=4, device=d)
    with torch.no_grad():
        y0 = layer(x, ei)
        y0b = layer(x, ei)  # the second workspace of the ping-pong pair
    assert torch.equal(y0, y0b)
    assert "_eval_plans" not in layer.__dict__ and len(_eval_plans[layer]) == 1
    cp = copy.deepcopy(layer)
    blob = pickle.dumps(layer)  # our own bytes, loaded back below
    del layer
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    junk = torch.full((64 << 20,), float("nan"), device=d)  # reuse the freed memory
    ld = pickle.loads(blob)
    with torch.no_grad():
        for m in (cp, ld):
            for _ in range(3):
                assert torch.equal(m(x, ei), y0)
    del junk
    # a cached plan holds the graph weakly: dropping the graph frees it
    csr_ref = weakref.ref(get_csr(ei, n, d).rowptr)
    del ei
    gc.collect()
    assert csr_ref() is None


def test_csr_max_degree():
    """build_csr records the longest row (order[0]'s in-degree, self-loop
    included), read with the range flag in one device -> host copy."""
    from atmlgraphattentionnetworks_amd.graph import build_csr
    d = dev()
    rng = np.random.default_rng(5)
    for hub_deg in (0, 1023, 5000):
        n, e = 3000, 20000
        dst = rng.integers(0, n, size=e)
        if hub_deg:
            dst = np.concatenate([dst, np.full(hub_deg, 7)])
        src = rng.integers(0, n, size=dst.size)
        ei = torch.from_numpy(np.stack([src, dst]).astype(np.int64)).to(d)
        csr = build_csr(ei, n)
        deg = np.bincount(dst, minlength=n) + 1  # + the self-loop
        assert csr.max_degree == int(deg.max())


@pytest.mark.parametrize("fin", [1, 3, 4, 5, 8])
@pytest.mark.parametrize("hfc", [(4, 8, True), (8, 8, True), (8, 8, False), (16, 4, True),
                                 (4, 4, False)],
                         ids=["H4F8_cat", "H8F8_cat", "H8F8_mean", "H16F4_cat", "H4F4_mean"])
def test_small_fin_fused_forward(fin, hfc, monkeypatch):
    """Fin <= 4 (CIFAR's 3): gat_layer_forward fuses the projection into the
    edge kernel, which gathers x rows and projects them in registers
    (k_edge_grp<..., XF>).  Against the oracle at the parity bar, and against
    the two-kernel path (GAT_EDGE_XPROJ=0) with non-finite x in a few rows:
    the same Inf / NaN pattern."""
    from atmlgraphattentionnetworks_amd import tuning
    H, F, concat = hfc
    x, ei, state = random_case(700, 8000, fin, H, F, concat, seed=31 * fin + H)
    ref = gat_layer_forward_from_state(state, x, ei, H, concat)
    outs = {}
    xb = x.clone()
    xb[5, 0] = float("inf")
    xb[77, fin - 1] = float("nan")
    xb[300, 0] = float("-inf")
    for xproj in ("1", "0"):
        monkeypatch.setenv("GAT_EDGE_XPROJ", xproj)
        tuning.reload()
        layer = layer_from_state(state, fin, F, H, concat)
        outs[xproj] = run_layer(layer, x, ei)
        outs[xproj + "_bad"] = run_layer(layer, xb, ei)
    torch.testing.assert_close(outs["1"], ref, atol=ATOL, rtol=RTOL)
    torch.testing.assert_close(outs["1"], outs["0"], atol=ATOL, rtol=RTOL)
    assert torch.equal(torch.isnan(outs["1_bad"]), torch.isnan(outs["0_bad"]))
    assert torch.equal(torch.isinf(outs["1_bad"]), torch.isinf(outs["0_bad"]))
    fin_rows = torch.isfinite(outs["0_bad"]).all(1)
    torch.testing.assert_close(outs["1_bad"][fin_rows], outs["0_bad"][fin_rows], atol=ATOL,
                               rtol=RTOL)
