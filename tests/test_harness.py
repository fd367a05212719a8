"""Host-side harness on CPU: the GATNet module tree, the synthetic datasets
and collation, the per-graph readout, and the run-loop control flow
(early stopping, checkpoint, test of the best checkpoint) driven by a torch-only
stand-in model — the GPU layer itself is exercised in test_gpu_gatnet.py."""
import pytest
import torch

from atmlgraphattentionnetworks_amd.datasets import (DATASET_SHAPES, GraphLoader, collate,
                                                     synthetic_cifar_graphs,
                                                     synthetic_node_dataset)
from atmlgraphattentionnetworks_amd.gatnet import GATNET_CONFIGS, GATNet, segment_mean
from atmlgraphattentionnetworks_amd.run import (TrainConfig, summarize,
                                                train_graph_classification,
                                                train_node_classification)


@pytest.mark.parametrize("name", ["Cora", "Citeseer", "Pubmed", "AmazonComp"])
def test_gatnet_module_tree_matches_reference(name):
    torch.manual_seed(0)
    fin = DATASET_SHAPES[name].features
    m = GATNet("GAT", name, fin)
    c1, c2 = GATNET_CONFIGS[name]
    assert m.conv1.num_heads == c1["heads"] and m.conv1.concat is True
    assert m.conv1.dropout_val == c1["dropout"]
    assert m.conv2.output_channels == c2["out"] and m.conv2.num_heads == c2["heads"]
    assert m.conv2.concat is False
    keys = list(m.state_dict())
    assert keys[0] == "conv1.bias" and "conv2.attentions2.0.bias" in keys


def test_gatnet_cifar_has_readout_mlp_and_gcn_is_out_of_scope():
    m = GATNet("GAT", "CIFAR10", 3)
    assert m.lin1.in_features == 64 and m.lin2.out_features == 10
    assert m.conv2.input_channels == 64 and m.conv2.concat is True
    with pytest.raises(NotImplementedError):
        GATNet("GCN", "Cora", 1433)
    with pytest.raises(ValueError):
        GATNet("GAT", "Reddit", 602)


def test_segment_mean_matches_loop():
    x = torch.randn(10, 3)
    batch = torch.tensor([0, 0, 1, 1, 1, 3, 3, 3, 3, 3])
    out = segment_mean(x, batch, 5)
    for g in range(5):
        sel = x[batch == g]
        ref = sel.mean(0) if len(sel) else torch.zeros(3)
        assert torch.allclose(out[g], ref, atol=1e-6)


@pytest.mark.parametrize("name", sorted(DATASET_SHAPES))
def test_synthetic_node_dataset_shapes_and_splits(name):
    sh = DATASET_SHAPES[name]
    d = synthetic_node_dataset(name, seed=1, scale=0.05)
    assert d.x.size(1) == sh.features and d.edge_index.size(0) == 2
    assert int(d.edge_index.max()) < d.num_nodes
    assert not bool((d.train_mask & d.val_mask).any())
    assert not bool((d.train_mask & d.test_mask).any())
    assert not bool((d.val_mask & d.test_mask).any())
    per_class = torch.bincount(d.y[d.train_mask], minlength=sh.classes)
    assert int(per_class.max()) <= 20
    if sh.normalize:
        s = d.x.sum(1)
        assert torch.allclose(s[s > 0], torch.ones_like(s[s > 0]), atol=1e-5)


def test_full_size_public_split():
    d = synthetic_node_dataset("Cora", seed=0)
    assert d.num_nodes == 2708
    assert int(d.train_mask.sum()) == 140 and int(d.val_mask.sum()) == 500
    assert int(d.test_mask.sum()) == 1000


def test_collate_block_diagonal():
    gs = synthetic_cifar_graphs(5, seed=2)
    b = collate(gs)
    sizes = [g.x.size(0) for g in gs]
    assert b.x.size(0) == sum(sizes) and b.num_graphs == 5
    assert torch.equal(torch.bincount(b.batch), torch.tensor(sizes))
    # every edge stays inside its graph
    assert torch.equal(b.batch[b.edge_index[0]], b.batch[b.edge_index[1]])
    loader = GraphLoader(gs, 2, shuffle=True, seed=0)
    assert len(loader) == 3
    assert sum(bt.num_graphs for bt in loader) == 5


class _CpuNodeModel(torch.nn.Module):
    """Stand-in for GATNet in the loop tests (CPU, no graph op)."""

    def __init__(self, fin, classes):
        super().__init__()
        self.lin = torch.nn.Linear(fin, classes)

    def forward(self, data):
        return torch.log_softmax(self.lin(torch.nn.functional.dropout(
            data.x, 0.2, self.training)), dim=1)


def test_node_loop_early_stopping_and_checkpoint(tmp_path):
    torch.manual_seed(0)
    d = synthetic_node_dataset("Cora", seed=0, scale=0.3)
    m = _CpuNodeModel(d.x.size(1), 7)
    ck = str(tmp_path / "model" / "cur_model.pt")
    cfg = TrainConfig(forced_epochs=5, early_stopping_patience=15, num_epochs=400,
                      checkpoint=ck, learning_rate=0.05)
    res = train_node_classification(m, d, cfg)
    assert res.epochs < 400  # stopped early
    assert len(res.val_accs) == res.epochs - cfg.forced_epochs + 1
    assert res.test_acc > 0.3  # chance is 1/7
    # the test accuracy is that of the saved checkpoint
    state = torch.load(ck, weights_only=True)
    m2 = _CpuNodeModel(d.x.size(1), 7)
    m2.load_state_dict(state)
    m2.eval()
    pred = m2(d).argmax(1)
    acc = float((pred[d.test_mask] == d.y[d.test_mask]).float().mean())
    assert acc == pytest.approx(res.test_acc)


def test_node_loop_without_early_stopping_runs_num_epochs():
    d = synthetic_node_dataset("Citeseer", seed=0, scale=0.1)
    m = _CpuNodeModel(d.x.size(1), 6)
    res = train_node_classification(m, d, TrainConfig(use_early_stopping=False, num_epochs=25,
                                                       logging_frequency=10))
    assert res.epochs == 25 and len(res.train_losses) == 25
    assert len(res.val_accs) == 2  # epochs 10 and 20


class _CpuGraphModel(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.lin = torch.nn.Linear(3, 10)

    def forward(self, data):
        return torch.log_softmax(self.lin(segment_mean(data.x, data.batch, data.num_graphs)), 1)


def test_graph_loop_runs_and_checkpoints(tmp_path):
    torch.manual_seed(0)
    tr = GraphLoader(synthetic_cifar_graphs(64, seed=0), 16, shuffle=True)
    va = GraphLoader(synthetic_cifar_graphs(32, seed=1), 16)
    te = GraphLoader(synthetic_cifar_graphs(32, seed=2), 16)
    cfg = TrainConfig(forced_epochs=1, early_stopping_patience=2, num_epochs=6,
                      checkpoint=str(tmp_path / "cur_model.pt"), learning_rate=0.05)
    res = train_graph_classification(_CpuGraphModel(), tr, va, te, torch.device("cpu"), cfg)
    assert 1 <= res.epochs <= 6 and 0.0 <= res.test_acc <= 1.0
    assert (tmp_path / "cur_model.pt").exists()


def test_summarize_matches_reference_formula():
    s = summarize([0.5, 0.7, 0.6])
    import numpy as np
    assert s["mean"] == pytest.approx(0.6)
    assert s["ci95"] == pytest.approx(1.96 * np.sqrt(np.var([0.5, 0.7, 0.6])) / np.sqrt(3))


def test_compact_bench_line_fits_driver_budget():
    """The N = 1 line built from round 3's full 29.8 KB result (the one the
    driver could not parse) is under the budget and keeps the required keys,
    the roofline and the CPU baseline."""
    import json
    import os
    from atmlgraphattentionnetworks_amd.benchline import LINE_BUDGET, REQUIRED, compact_single
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    full = json.load(open(os.path.join(root, "profiles", "r03", "bench_default.json")))
    assert len(json.dumps(full)) > 20000
    line = compact_single(full, "gpurun_out/bench_detail.json")
    s = json.dumps(line)
    assert len(s) <= LINE_BUDGET
    for k in REQUIRED:
        assert k in line, k
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in line["roofline"]
    assert line["cpu_baseline"]["cores"] == 16 and line["cpu_baseline"]["kind"] == "port"
    assert line["multi_gpu_emulated"]["reddit"]["allgather_P8"]["bound"] > 1


def test_compact_line_drops_optional_keys_first():
    from atmlgraphattentionnetworks_amd.benchline import REQUIRED, fit
    line = {k: 1 for k in REQUIRED}
    line["big"] = "x" * 10000
    line["small"] = 2
    out = fit(line, ("big", "small"), budget=500)
    assert "big" not in out and out["small"] == 2 and all(k in out for k in REQUIRED)
    out = fit({**line, "other": "y" * 10000}, ("big",), budget=500)
    assert "truncated" in out and all(k in out for k in REQUIRED)


def test_compact_dist_line_keeps_allgather_headline_and_graph():
    """The N > 1 line built from round 5's --dist detail (one-rank RCCL group,
    graph-replayed all-gather step): under the budget, required keys kept, the
    headline on the all-gather strategy with its launch mode, the graph trial
    summarised and 'replicate' beside it."""
    import json
    import os
    from atmlgraphattentionnetworks_amd.benchline import LINE_BUDGET, REQUIRED, compact_dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    full = json.load(open(os.path.join(root, "profiles", "r05", "bench_dist1_graph_detail.json")))
    line = compact_dist(full, "gpurun_out/bench_detail.json")
    assert len(json.dumps(line)) <= LINE_BUDGET
    for k in REQUIRED:
        assert k in line, k
    assert line["config"]["strategy"].startswith("allgather")
    assert line["headline"]["strategy"] == line["config"]["strategy"]
    assert line["headline"]["launch"] == line["config"]["launch"]
    assert line["graph"]["ok"] is True and line["graph"]["eager_value"] < line["value"]
    assert line["replicate"]["strategy"] == "replicate"
    arx = line["workloads"]["arxiv"]
    assert arx["strategy"].startswith("allgather") and arx["graph"]["ok"] is True
