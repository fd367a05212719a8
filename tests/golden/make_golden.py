"""Generate the golden fixtures in ``tests/golden/*.npz`` from the reference's
own ``GAT.py`` (run in THIS container only; ``/root/reference`` does not exist
on the GPU box).

The reference imports ``torch_geometric`` (PyG), which is neither vendored nor
installed; ``pyg_restated/`` restates the three PyG 2.0.x entry points GAT.py
calls (``add_self_loops``, ``MessagePassing`` with ``aggr='add'``,
``utils.softmax``).  Everything else — the constructor's RNG order
(``GAT.py:8-35``), the head loop, stack/transpose, ``message`` and the bias
(``GAT.py:37-67``) — is the reference's own code.

Each fixture holds inputs (x, edge_index, the layer's state_dict) and the
reference output in eval mode.  Usage::

    python tests/golden/make_golden.py          # rewrites tests/golden/*.npz
"""
from __future__ import annotations

import importlib.util
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/GAT.py"

# (name, N, E, Fin, H, F, concat, graph kind, seed)
CASES = [
    # hand-checkable known-answer graphs
    ("kat_asym3", 3, None, 4, 2, 3, True, "asym3", 11),
    ("kat_isolated", 4, None, 5, 2, 2, True, "isolated", 12),
    ("kat_selfloop_multi", 3, None, 3, 3, 2, True, "selfloop_multi", 13),
    ("kat_mean_heads", 4, None, 4, 3, 2, False, "selfloop_multi4", 14),
    ("kat_single_head", 5, None, 3, 1, 4, False, "chain5", 15),
    ("kat_empty", 6, None, 4, 2, 4, True, "empty", 16),
    # the (heads, feats) grids of run_heads_experiment.py:52 and
    # run_params_experiment.py:50, plus GATNet.py's layer shapes
    ("grid_h1_f7_mean", 257, 2500, 12, 1, 7, False, "uniform", 21),
    ("grid_h2_f16_cat", 257, 2500, 12, 2, 16, True, "uniform", 22),
    ("grid_h4_f8_cat", 257, 2500, 12, 4, 8, True, "uniform", 23),
    ("grid_h8_f4_cat", 257, 2500, 12, 8, 4, True, "uniform", 24),
    ("grid_h16_f2_cat", 257, 2500, 12, 16, 2, True, "uniform", 25),
    ("grid_h32_f8_cat", 257, 2500, 12, 32, 8, True, "uniform", 26),
    ("grid_h8_f8_cat", 257, 2500, 12, 8, 8, True, "uniform", 27),
    ("grid_h8_f8_mean", 257, 2500, 12, 8, 8, False, "uniform", 28),
    ("grid_h8_f3_mean", 257, 2500, 64, 8, 3, False, "uniform", 29),
    ("grid_h8_f10_mean", 257, 2500, 64, 8, 10, False, "uniform", 30),
    ("grid_h3_f5_cat", 257, 2500, 9, 3, 5, True, "uniform", 31),
    ("grid_h1_f6_mean_skew", 300, 3000, 16, 1, 6, False, "skew", 32),
    ("ppi_small_h8_f8", 2000, 30000, 50, 8, 8, True, "uniform", 33),
    ("cifar_like_h4_f8", 600, None, 3, 4, 8, True, "knn", 34),
]


def _load_reference():
    sys.dont_write_bytecode = True
    sys.path.insert(0, os.path.join(HERE, "pyg_restated"))
    spec = importlib.util.spec_from_file_location("reference_GAT", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def make_graph(kind: str, n: int, e, rng: np.random.Generator) -> np.ndarray:
    if kind == "asym3":
        return np.array([[0, 2, 1], [1, 1, 0]], dtype=np.int64)
    if kind == "isolated":
        return np.array([[0, 1, 2, 0], [1, 2, 0, 2]], dtype=np.int64)
    if kind == "selfloop_multi":
        # pre-existing self-loop 1->1 and a doubled edge 0->2
        return np.array([[1, 0, 0, 2, 1], [1, 2, 2, 0, 0]], dtype=np.int64)
    if kind == "selfloop_multi4":
        return np.array([[1, 0, 0, 2, 3, 3], [1, 2, 2, 0, 3, 0]], dtype=np.int64)
    if kind == "chain5":
        return np.array([[0, 1, 2, 3], [1, 2, 3, 4]], dtype=np.int64)
    if kind == "empty":
        return np.zeros((2, 0), dtype=np.int64)
    if kind == "uniform":
        dst = rng.integers(0, n, size=e)
        src = (dst + 1 + rng.integers(0, n - 1, size=e)) % n
        return np.stack([src, dst]).astype(np.int64)
    if kind == "skew":
        # power-law in-degree: a few hubs take most edges
        w = 1.0 / np.arange(1, n + 1) ** 1.2
        dst = rng.choice(n, size=e, p=w / w.sum())
        src = rng.integers(0, n, size=e)
        return np.stack([src, dst]).astype(np.int64)
    if kind == "knn":
        # block-diagonal 8-NN graphs like run_gnn_benchmark.py's batches
        srcs, dsts, base = [], [], 0
        while base < n:
            ng = int(min(n - base, rng.integers(40, 80)))
            pos = rng.random((ng, 2))
            d = ((pos[:, None, :] - pos[None, :, :]) ** 2).sum(-1)
            np.fill_diagonal(d, np.inf)
            k = min(8, ng - 1)
            nbr = np.argsort(d, axis=1)[:, :k]
            for i in range(ng):
                for j in nbr[i]:
                    srcs.append(base + j)
                    dsts.append(base + i)
            base += ng
        return np.array([srcs, dsts], dtype=np.int64)
    raise ValueError(kind)


def main():
    ref = _load_reference()
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from oracle import gat_layer_forward_from_state  # cross-check only

    index = []
    for (name, n, e, fin, H, F, concat, kind, seed) in CASES:
        rng = np.random.default_rng(seed)
        ei = make_graph(kind, n, e, rng)
        torch.manual_seed(seed)
        layer = ref.GraphAttentionLayer(fin, F, num_heads=H, concat=concat)
        layer.eval()
        x = torch.from_numpy(rng.standard_normal((n, fin)).astype(np.float32))
        with torch.no_grad():
            out = layer(x, torch.from_numpy(ei))
        state = {k: v.detach().numpy().copy() for k, v in layer.state_dict().items()}
        mine = gat_layer_forward_from_state(layer.state_dict(), x, torch.from_numpy(ei), H, concat)
        diff = float((mine - out).abs().max()) if out.numel() else 0.0
        arrays = {"x": x.numpy(), "edge_index": ei, "out": out.numpy()}
        for k, v in state.items():
            arrays["param/" + k] = v
        meta = dict(name=name, N=n, E=int(ei.shape[1]), Fin=fin, H=H, F=F, concat=concat,
                    kind=kind, seed=seed, state_keys=list(state.keys()))
        arrays["meta"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrays)
        index.append({k: v for k, v in meta.items() if k != "state_keys"} | {"oracle_max_abs_diff": diff})
        print(f"{name:24s} N={n:5d} E={ei.shape[1]:6d} H={H:2d} F={F:2d} concat={concat!s:5s} "
              f"oracle-vs-reference max|diff|={diff:.3e}")
    with open(os.path.join(HERE, "INDEX.json"), "w") as fh:
        json.dump(index, fh, indent=1)


if __name__ == "__main__":
    main()
