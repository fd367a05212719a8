"""The reference's callers on the GPU layer: GATNet (GATNet.py:12-87) eval
parity against the oracle composition, the run-script loops end to end on
synthetic graphs (run_inductive.py, run_gnn_benchmark.py, the experiment
scripts), and checkpoint round trips."""
import pytest
import torch
import torch.nn.functional as F

from oracle import gat_layer_forward_from_state

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _sub_state(state, prefix):
    return {k[len(prefix):]: v for k, v in state.items() if k.startswith(prefix)}


@pytest.mark.parametrize("name", ["Cora", "Pubmed", "AmazonPhotos"])
def test_gatnet_eval_matches_oracle_composition(name):
    from atmlgraphattentionnetworks_amd.datasets import synthetic_node_dataset
    from atmlgraphattentionnetworks_amd.gatnet import GATNET_CONFIGS, GATNet
    torch.manual_seed(0)
    d = synthetic_node_dataset(name, seed=0, scale=0.25)
    model = GATNet("GAT", name, d.x.size(1))
    with torch.no_grad():
        for p in model.parameters():
            p.add_(0.05 * torch.randn_like(p))  # non-zero biases
    state = {k: v.clone() for k, v in model.state_dict().items()}
    model = model.to(DEV).eval()
    with torch.no_grad():
        out = model(d.to(DEV)).cpu()
    c1, c2 = GATNET_CONFIGS[name]
    h = gat_layer_forward_from_state(_sub_state(state, "conv1."), d.x, d.edge_index,
                                     c1["heads"], c1["concat"])
    h = F.elu(h)
    ref = F.log_softmax(gat_layer_forward_from_state(_sub_state(state, "conv2."), h,
                                                     d.edge_index, c2["heads"], c2["concat"]),
                        dim=1)
    assert torch.allclose(out, ref, atol=2e-5, rtol=0), float((out - ref).abs().max())


def test_node_classification_loop_learns_and_checkpoints(tmp_path):
    from atmlgraphattentionnetworks_amd.datasets import synthetic_node_dataset
    from atmlgraphattentionnetworks_amd.gatnet import GATNet
    from atmlgraphattentionnetworks_amd.run import TrainConfig, train_node_classification
    torch.manual_seed(0)
    d = synthetic_node_dataset("Cora", seed=0).to(DEV)
    model = GATNet("GAT", "Cora", d.x.size(1)).to(DEV)
    ck = str(tmp_path / "cur_model.pt")
    res = train_node_classification(model, d, TrainConfig(forced_epochs=20,
                                                          early_stopping_patience=30,
                                                          num_epochs=300, checkpoint=ck))
    assert res.train_losses[-1] < res.train_losses[0]
    assert res.test_acc > 0.5, res.test_acc  # chance: 1/7
    # checkpoint round trip into a fresh model gives the reported test accuracy
    fresh = GATNet("GAT", "Cora", d.x.size(1)).to(DEV)
    fresh.load_state_dict(torch.load(ck, weights_only=True))
    fresh.eval()
    with torch.no_grad():
        pred = fresh(d).argmax(1)
    acc = float((pred[d.test_mask] == d.y[d.test_mask]).float().mean())
    assert acc == pytest.approx(res.test_acc)


def test_graph_classification_loop_runs():
    from atmlgraphattentionnetworks_amd.datasets import GraphLoader, synthetic_cifar_graphs
    from atmlgraphattentionnetworks_amd.gatnet import GATNet
    from atmlgraphattentionnetworks_amd.run import TrainConfig, train_graph_classification
    torch.manual_seed(0)
    tr = GraphLoader(synthetic_cifar_graphs(1024, seed=0), 512, shuffle=True)
    va = GraphLoader(synthetic_cifar_graphs(256, seed=1), 512)
    te = GraphLoader(synthetic_cifar_graphs(256, seed=2), 512)
    model = GATNet("GAT", "CIFAR10", 3).to(DEV)
    res = train_graph_classification(model, tr, va, te, DEV,
                                     TrainConfig(forced_epochs=1, early_stopping_patience=5,
                                                 num_epochs=8))
    assert res.epochs >= 1 and 0.0 <= res.test_acc <= 1.0
    assert res.train_losses[-1] < res.train_losses[0]


def test_ppi_shape_one_epoch():
    """BASELINE config 1's workload (PPI shape, conv1 4 heads) for one epoch."""
    from atmlgraphattentionnetworks_amd.datasets import synthetic_node_dataset
    from atmlgraphattentionnetworks_amd.gatnet import GATNet
    from atmlgraphattentionnetworks_amd.run import TrainConfig, train_node_classification
    torch.manual_seed(0)
    d = synthetic_node_dataset("PPI", seed=0).to(DEV)
    model = GATNet("GAT", "PPI", 50).to(DEV)
    res = train_node_classification(model, d, TrainConfig(use_early_stopping=False,
                                                          num_epochs=1))
    assert res.epochs == 1 and len(res.train_losses) == 1


@pytest.mark.parametrize("task", ["heads", "params", "act"])
def test_experiment_models_train(task):
    from atmlgraphattentionnetworks_amd.datasets import synthetic_node_dataset
    from atmlgraphattentionnetworks_amd.gatnet import GATActivationModel, GATModel
    from atmlgraphattentionnetworks_amd.run import TrainConfig, train_node_classification
    torch.manual_seed(0)
    d = synthetic_node_dataset("Cora", seed=0, scale=0.5).to(DEV)
    if task == "heads":
        models = [GATModel(d.x.size(1), f, h, 7) for h, f in [(2, 16), (4, 8), (8, 4), (16, 2)]]
    elif task == "params":
        models = [GATModel(d.x.size(1), 8, h, 7) for h in (2, 4, 8, 16, 32)]
    else:
        models = [GATActivationModel(d.x.size(1), 8, 8, 7, m())
                  for m in (torch.nn.LogSigmoid, torch.nn.Tanh, torch.nn.Softmax)]
    for m in models:
        res = train_node_classification(m.to(DEV), d, TrainConfig(use_early_stopping=False,
                                                                  num_epochs=15))
        assert res.train_losses[-1] < res.train_losses[0]


def test_node_classification_loop_with_captured_step():
    """run.py's graphed training step (forward, loss, backward, Adam replayed as
    one HIP graph; device-seeded attention dropout): learns like the eager loop
    and runs the same number of epochs without early stopping."""
    import time
    from atmlgraphattentionnetworks_amd.datasets import synthetic_node_dataset
    from atmlgraphattentionnetworks_amd.gatnet import GATNet
    from atmlgraphattentionnetworks_amd.run import TrainConfig, train_node_classification
    d = synthetic_node_dataset("Cora", seed=0).to(DEV)
    res = {}
    for graph in (False, True):
        torch.manual_seed(0)
        model = GATNet("GAT", "Cora", d.x.size(1)).to(DEV)
        t0 = time.perf_counter()
        r = train_node_classification(model, d, TrainConfig(use_early_stopping=False,
                                                            num_epochs=150, use_graph=graph))
        res[graph] = (r, time.perf_counter() - t0)
    for graph, (r, _) in res.items():
        assert r.epochs == 150 and len(r.train_losses) == 150
        assert r.train_losses[-1] < 0.7 * r.train_losses[0], (graph, r.train_losses[::30])
        assert r.test_acc > 0.5, (graph, r.test_acc)
    print(f"eager {res[False][1]:.2f}s, graphed {res[True][1]:.2f}s for 150 epochs")
