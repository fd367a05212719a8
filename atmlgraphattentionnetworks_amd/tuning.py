"""Kernel-choice knobs (the variant tests and A/B measurement in tools/).

The GAT_* environment variables are read ONCE, when this module is imported
(and by the HIP library at its first launch), never per forward.  Tools and
tests that switch variants inside one process call ``reload()`` after
changing the environment; it re-reads the Python-side knobs and asks the
library for a new snapshot (``gat_tuning_reload``).  No knob changes results
beyond fp32 summation order; the defaults are the measured-fastest choices.
"""
from __future__ import annotations

import os
from typing import Dict, Optional

# knobs read on the Python side of the boundary: the node table's column
# planes, hub splitting and its segment length, the scheduled CSR copy
PY_KNOBS = ("GAT_WH_SLICES", "GAT_HUB_SPLIT", "GAT_HUB_SEG", "GAT_EDGE_SCHED")

_values: Dict[str, Optional[str]] = {}
# bumped by every reload(): cached launch plans (layer.ForwardPlan) key on it,
# so a knob change reaches the next forward
generation = 0


def reload() -> None:
    """Re-read the environment (Python knobs and the library's snapshot)."""
    global _values, generation
    _values = {k: os.environ.get(k) for k in PY_KNOBS}
    generation += 1
    from . import _lib
    if _lib.is_loaded():
        _lib.load().gat_tuning_reload()


def get(name: str) -> Optional[str]:
    return _values.get(name)


_values = {k: os.environ.get(k) for k in PY_KNOBS}
