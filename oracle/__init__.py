"""Test infrastructure: CPU oracle for the GAT layer forward.

Importable only from ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg.  Never used by the product path.
"""
from .gat_oracle import *  # noqa: F401,F403
