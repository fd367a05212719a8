"""Restated PyG 2.0.x entry points used by the reference GAT.py (test fixture
generation only).  PyG is a third-party dependency that is not vendored in
the reference and not installed here; these three pieces restate its
published algorithm so that the reference's OWN GAT.py:37-67 code can run and
produce golden vectors.  Not shipped, not used by the product."""
from . import nn, utils  # noqa: F401
