import glob
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running (full-size) case")


def golden_names():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN_DIR, "*.npz")))


def load_golden(name):
    """Fixture -> dict(meta, x, edge_index, out, state) (numpy / torch CPU)."""
    import torch

    z = np.load(os.path.join(GOLDEN_DIR, name + ".npz"), allow_pickle=False)
    meta = json.loads(bytes(z["meta"]).decode())
    state = {k[len("param/"):]: torch.from_numpy(z[k].copy()) for k in z.files if k.startswith("param/")}
    ordered = {k: state[k] for k in meta["state_keys"]}
    return dict(meta=meta, x=torch.from_numpy(z["x"].copy()),
                edge_index=torch.from_numpy(z["edge_index"].copy()),
                out=torch.from_numpy(z["out"].copy()), state=ordered)


def _reload_tuning():
    from atmlgraphattentionnetworks_amd import tuning
    tuning.reload()


@pytest.fixture(autouse=True)
def _tuning_follows_env(monkeypatch):
    """The library reads its GAT_* A/B knobs once (atmlgraphattentionnetworks_amd.tuning);
    a test that switches variants with monkeypatch.setenv/delenv gets a fresh
    snapshot after each change, and the original one back at teardown."""
    orig_set, orig_del = monkeypatch.setenv, monkeypatch.delenv

    def setenv(name, value, prepend=None):
        orig_set(name, value, prepend)
        if name.startswith("GAT_"):
            _reload_tuning()

    def delenv(name, raising=True):
        orig_del(name, raising)
        if name.startswith("GAT_"):
            _reload_tuning()

    monkeypatch.setenv, monkeypatch.delenv = setenv, delenv
    yield
    monkeypatch.undo()
    _reload_tuning()
