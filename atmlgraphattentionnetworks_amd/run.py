"""The reference's training loops on the MI355X layer.

* :func:`train_node_classification` — ``run_inductive.py:33-140`` (and the
  per-configuration loop of ``run_heads_experiment.py``,
  ``run_params_experiment.py``, ``run_act_func_experiment.py``): full-batch
  Adam, NLL on the training mask, early stopping on validation accuracy /
  loss after ``forced_epochs`` with a state_dict checkpoint, test accuracy of
  the best checkpoint, averaged over runs with a 95 % interval.
* :func:`train_graph_classification` — ``run_gnn_benchmark.py:32-142``:
  mini-batches of collated graphs, per-graph readout, the same early stopping.

The control flow (when the checkpoint is written, when the patience counter
resets) follows the reference line for line; checkpoints are loaded with
``torch.load(..., weights_only=True)``.  Datasets are the synthetic stand-ins
of :mod:`datasets` (no network here).

CLI::

    python -m atmlgraphattentionnetworks_amd.run node --dataset Cora --runs 1
    python -m atmlgraphattentionnetworks_amd.run graph --train-graphs 2048 --runs 1
    python -m atmlgraphattentionnetworks_amd.run heads --dataset Cora --runs 1
"""
from __future__ import annotations

import argparse
import json
import os
import tempfile
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

import numpy as np
import torch
import torch.nn.functional as F

__all__ = ["TrainConfig", "RunResult", "train_node_classification",
           "train_graph_classification", "summarize"]


@dataclass
class TrainConfig:
    """The scripts' hyper-parameter block (``run_inductive.py:17-30``)."""
    learning_rate: float = 0.005
    weight_decay: float = 0.0005
    use_early_stopping: bool = True
    forced_epochs: int = 20
    early_stopping_patience: int = 100
    num_epochs: int = 10000
    logging_frequency: int = 10
    verbose: bool = False
    checkpoint: Optional[str] = None  # default: a file in a fresh temp dir
    # full-batch node classification only: capture the training step (forward,
    # loss, backward, Adam) in one HIP graph and replay it per epoch
    use_graph: bool = False


@dataclass
class RunResult:
    test_acc: float
    epochs: int
    train_losses: List[float] = field(default_factory=list)
    train_accs: List[float] = field(default_factory=list)
    val_losses: List[float] = field(default_factory=list)
    val_accs: List[float] = field(default_factory=list)
    seconds: float = 0.0


def _log(cfg: TrainConfig, *msg):
    if cfg.verbose:
        print(*msg, flush=True)


def _checkpoint_path(cfg: TrainConfig) -> str:
    if cfg.checkpoint:
        os.makedirs(os.path.dirname(os.path.abspath(cfg.checkpoint)), exist_ok=True)
        return cfg.checkpoint
    return os.path.join(tempfile.mkdtemp(prefix="gat_ckpt_"), "cur_model.pt")


def _load_checkpoint(model, path):
    model.load_state_dict(torch.load(path, weights_only=True))


class _GraphedStep:
    """The epoch's training step (``run_inductive.py:74-84``: forward, NLL on
    the training nodes, backward, Adam) captured in one HIP graph.  Same math as
    the eager step; the training nodes are an index tensor (a boolean mask
    select has a data-dependent size), Adam is ``capturable``, and dropout
    masks (torch's for the features, the layer's device-seeded attention
    dropout) are fresh on every replay.  The warm-up steps it runs before
    capturing are real epochs."""

    def __init__(self, model, data, optimizer, warmup: int = 3):
        self.model, self.data, self.opt = model, data, optimizer
        self.idx = data.train_mask.nonzero().squeeze(1)
        self.y = data.y.index_select(0, self.idx)
        self.warmup_out = []
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                # detached: a kept-alive autograd graph would carry its
                # AccumulateGrad nodes (and their stream) into the capture
                self.warmup_out.append(tuple(t.detach() for t in self._step()))
        torch.cuda.current_stream().wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        optimizer.zero_grad(set_to_none=True)
        with torch.cuda.graph(self.graph):
            self.out, self.loss = self._step()

    def _step(self):
        self.opt.zero_grad(set_to_none=True)
        out = self.model(self.data)
        loss = F.nll_loss(out.index_select(0, self.idx), self.y)
        loss.backward()
        self.opt.step()
        return out, loss

    def __call__(self):
        self.graph.replay()
        return self.out, self.loss


def train_node_classification(model: torch.nn.Module, data, cfg: TrainConfig) -> RunResult:
    """One run of ``run_inductive.py:66-133`` on ``data`` (already on the device)."""
    t0 = time.perf_counter()
    res = RunResult(0.0, 0)
    ckpt = _checkpoint_path(cfg)
    saved = False
    optimizer = torch.optim.Adam(model.parameters(), lr=cfg.learning_rate,
                                 weight_decay=cfg.weight_decay, capturable=cfg.use_graph)
    _log(cfg, "Starting training...")
    epoch, stop_counter = 0, 0
    cur_max, cur_min_loss = 0.0, float("inf")
    stop_training = False
    graphed, pending = None, []
    if cfg.use_graph:
        model.train()
        graphed = _GraphedStep(model, data, optimizer)
        pending = list(graphed.warmup_out)
    while not stop_training:
        model.train()
        if graphed is not None:
            out, loss = pending.pop(0) if pending else graphed()
        else:
            optimizer.zero_grad()
            out = model(data)
            loss = F.nll_loss(out[data.train_mask], data.y[data.train_mask])
        pred = out.argmax(dim=1)
        correct = (pred[data.train_mask] == data.y[data.train_mask]).sum()
        res.train_accs.append((correct / data.train_mask.sum()).item())
        res.train_losses.append(loss.item())
        if graphed is None:
            loss.backward()
            optimizer.step()
        if cfg.use_early_stopping:
            if epoch >= cfg.forced_epochs - 1:
                model.eval()
                with torch.no_grad():
                    out = model(data)
                pred = out.argmax(dim=1)
                vloss = F.nll_loss(out[data.val_mask], data.y[data.val_mask]).item()
                correct = (pred[data.val_mask] == data.y[data.val_mask]).sum()
                acc = (correct / data.val_mask.sum()).item()
                res.val_losses.append(vloss)
                res.val_accs.append(acc)
                if acc >= cur_max or vloss <= cur_min_loss:
                    _log(cfg, f"Found new validation maximum at epoch {epoch + 1}: "
                              f"acc {cur_max} -> {acc}, loss {cur_min_loss} -> {vloss}")
                    if acc > cur_max and vloss < cur_min_loss:
                        torch.save(model.state_dict(), ckpt)
                        saved = True
                    cur_max = max(acc, cur_max)
                    cur_min_loss = min(cur_min_loss, vloss)
                    stop_counter = 0
                else:
                    stop_counter += 1
                    if stop_counter >= cfg.early_stopping_patience:
                        _log(cfg, "Stopping training...")
                        stop_training = True
        else:
            if epoch != 0 and (epoch + 1) % cfg.logging_frequency == 0:
                model.eval()
                with torch.no_grad():
                    out = model(data)
                pred = out.argmax(dim=1)
                correct = (pred[data.val_mask] == data.y[data.val_mask]).sum()
                acc = float(int(correct) / int(data.val_mask.sum()))
                res.val_accs.append(acc)
                res.val_losses.append(F.nll_loss(out[data.val_mask],
                                                 data.y[data.val_mask]).item())
                _log(cfg, f"Epoch: {epoch + 1}, Validation Accuracy: {acc}")
            if epoch >= cfg.num_epochs - 1:
                stop_training = True
        epoch += 1
        if cfg.use_early_stopping and epoch >= cfg.num_epochs:
            stop_training = True  # a hard cap; the reference's is 10000 epochs
    model.eval()
    if cfg.use_early_stopping and saved:
        _load_checkpoint(model, ckpt)
    with torch.no_grad():
        pred = model(data).argmax(dim=1)
    correct = (pred[data.test_mask] == data.y[data.test_mask]).sum()
    res.test_acc = float(int(correct) / int(data.test_mask.sum()))
    res.epochs = epoch
    res.seconds = time.perf_counter() - t0
    _log(cfg, f"Test Accuracy: {res.test_acc:.4f}")
    return res


def _eval_batches(model, loader, device):
    losses, accs = 0.0, 0.0
    with torch.no_grad():
        for batch in loader:
            batch = batch.to(device)
            out = model(batch)
            losses += F.nll_loss(out, batch.y).item()
            accs += (torch.sum(out.argmax(dim=1) == batch.y) / batch.y.shape[0]).item()
    return losses / len(loader), accs / len(loader)


def train_graph_classification(model: torch.nn.Module, train_loader, val_loader, test_loader,
                               device, cfg: TrainConfig) -> RunResult:
    """One run of ``run_gnn_benchmark.py:45-136``."""
    t0 = time.perf_counter()
    res = RunResult(0.0, 0)
    ckpt = _checkpoint_path(cfg)
    saved = False
    optimizer = torch.optim.Adam(model.parameters(), lr=cfg.learning_rate,
                                 weight_decay=cfg.weight_decay)
    epoch, stop_counter = 0, 0
    cur_max, cur_min_loss = 0.0, float("inf")
    stop_training = False
    while not stop_training:
        model.train()
        for batch in train_loader:
            batch = batch.to(device)
            optimizer.zero_grad()
            loss = F.nll_loss(model(batch), batch.y)
            loss.backward()
            optimizer.step()
            res.train_losses.append(loss.item())
        model.eval()
        if cfg.use_early_stopping:
            if epoch >= cfg.forced_epochs - 1:
                avg_loss, avg_acc = _eval_batches(model, val_loader, device)
                res.val_losses.append(avg_loss)
                res.val_accs.append(avg_acc)
                if avg_acc > cur_max or avg_loss < cur_min_loss:
                    if avg_acc >= cur_max and avg_loss <= cur_min_loss:
                        torch.save(model.state_dict(), ckpt)
                        saved = True
                    cur_max = max(avg_acc, cur_max)
                    cur_min_loss = min(cur_min_loss, avg_loss)
                    stop_counter = 0
                else:
                    stop_counter += 1
                    if stop_counter >= cfg.early_stopping_patience:
                        stop_training = True
        else:
            if epoch != 0 and (epoch + 1) % cfg.logging_frequency == 0:
                avg_loss, avg_acc = _eval_batches(model, val_loader, device)
                res.val_losses.append(avg_loss)
                res.val_accs.append(avg_acc)
            if epoch >= cfg.num_epochs - 1:
                stop_training = True
        epoch += 1
        if cfg.use_early_stopping and epoch >= cfg.num_epochs:
            stop_training = True
    model.eval()
    if cfg.use_early_stopping and saved:
        _load_checkpoint(model, ckpt)
    _, res.test_acc = _eval_batches(model, test_loader, device)
    res.epochs = epoch
    res.seconds = time.perf_counter() - t0
    return res


def summarize(accs: List[float]) -> Dict[str, float]:
    """Mean and 1.96 * std / sqrt(runs) (``run_inductive.py:136-140``)."""
    a = np.asarray(accs, dtype=np.float64)
    ci = 1.96 * (np.sqrt(np.var(a)) / np.sqrt(len(a))) if len(a) else float("nan")
    return {"mean": float(a.mean()) if len(a) else float("nan"), "ci95": float(ci),
            "runs": len(a)}


def _node_runs(make_model: Callable[[int, int], torch.nn.Module], dataset: str, runs: int,
               cfg: TrainConfig, device, seed: int, scale: float) -> Dict:
    from .datasets import DATASET_SHAPES, synthetic_node_dataset
    accs, details = [], []
    for r in range(runs):
        torch.manual_seed(seed + r)
        data = synthetic_node_dataset(dataset, seed=seed, scale=scale).to(device)
        sh = DATASET_SHAPES[dataset]
        model = make_model(sh.features, sh.classes).to(device)
        res = train_node_classification(model, data, cfg)
        accs.append(res.test_acc)
        details.append({"test_acc": res.test_acc, "epochs": res.epochs,
                        "seconds": round(res.seconds, 3)})
    return {"dataset": dataset, "data": "synthetic", **summarize(accs), "per_run": details}


def main(argv=None) -> Dict:
    from .gatnet import GATActivationModel, GATModel, GATNet
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("task", choices=["node", "graph", "heads", "params", "act"])
    ap.add_argument("--dataset", default="Citeseer")
    ap.add_argument("--runs", type=int, default=1)
    ap.add_argument("--max-epochs", type=int, default=10000)
    ap.add_argument("--forced-epochs", type=int, default=None)
    ap.add_argument("--patience", type=int, default=None)
    ap.add_argument("--no-early-stopping", action="store_true")
    ap.add_argument("--scale", type=float, default=1.0, help="shrink the synthetic graph")
    ap.add_argument("--train-graphs", type=int, default=2048)
    ap.add_argument("--eval-graphs", type=int, default=512)
    ap.add_argument("--batch-size", type=int, default=512)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--checkpoint", default=None)
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--graph", action="store_true",
                    help="node tasks: replay the training step as one captured HIP graph")
    a = ap.parse_args(argv)
    device = torch.device("cuda")
    graph_task = a.task == "graph"
    cfg = TrainConfig(use_early_stopping=not a.no_early_stopping, num_epochs=a.max_epochs,
                      forced_epochs=a.forced_epochs or (1 if graph_task else 20),
                      early_stopping_patience=a.patience or (5 if graph_task else 100),
                      verbose=a.verbose, checkpoint=a.checkpoint,
                      use_graph=a.graph and not graph_task)
    if a.task == "node":
        out = _node_runs(lambda fin, c: GATNet("GAT", a.dataset, fin), a.dataset, a.runs, cfg,
                         device, a.seed, a.scale)
    elif a.task in ("heads", "params"):
        pairs = ([(2, 16), (4, 8), (8, 4), (16, 2)] if a.task == "heads"  # run_heads:50
                 else [(2, 8), (4, 8), (8, 8), (16, 8), (32, 8)])  # run_params:50
        out = {"task": a.task, "results": {}}
        for heads, feats in pairs:
            out["results"][f"{heads}x{feats}"] = _node_runs(
                lambda fin, c, h=heads, f=feats: GATModel(fin, f, h, c), a.dataset, a.runs,
                cfg, device, a.seed, a.scale)
    elif a.task == "act":
        acts = {"log_sigmoid": torch.nn.LogSigmoid, "tanh": torch.nn.Tanh,
                "softmax": torch.nn.Softmax}  # run_act_func_experiment.py:111
        out = {"task": "act", "results": {}}
        for name, ctor in acts.items():
            out["results"][name] = _node_runs(
                lambda fin, c, m=ctor: GATActivationModel(fin, 8, 8, c, m()), a.dataset,
                a.runs, cfg, device, a.seed, a.scale)
    else:
        from .datasets import GraphLoader, synthetic_cifar_graphs
        train = GraphLoader(synthetic_cifar_graphs(a.train_graphs, seed=a.seed), a.batch_size,
                            shuffle=True, seed=a.seed)
        val = GraphLoader(synthetic_cifar_graphs(a.eval_graphs, seed=a.seed + 1), a.batch_size)
        test = GraphLoader(synthetic_cifar_graphs(a.eval_graphs, seed=a.seed + 2), a.batch_size)
        accs, details = [], []
        for r in range(a.runs):
            torch.manual_seed(a.seed + r)
            model = GATNet("GAT", "CIFAR10", 3).to(device)
            res = train_graph_classification(model, train, val, test, device, cfg)
            accs.append(res.test_acc)
            details.append({"test_acc": res.test_acc, "epochs": res.epochs,
                            "seconds": round(res.seconds, 3)})
        out = {"dataset": "CIFAR10", "data": "synthetic", **summarize(accs),
               "per_run": details}
    print(json.dumps(out))
    return out


if __name__ == "__main__":
    main()
