"""MI355X-native drop-in for the GAT attention layer of
danieldritter/ATMLGraphAttentionNetworks (``GAT.py:GraphAttentionLayer``).

    from atmlgraphattentionnetworks_amd import GraphAttentionLayer

PyTorch-ROCm host code over the C-ABI HIP library ``libgat_amd.so``
(``include/gat_amd.h``).  See DESIGN.md / INTEGRATION.md.
"""
from .layer import (GraphAttentionLayer, GraphAttentionLayerActivationTest,  # noqa: F401
                    gat_forward, pack_params)
from .graph import CSRGraph, build_csr, get_csr  # noqa: F401

__all__ = ["GraphAttentionLayer", "GraphAttentionLayerActivationTest", "gat_forward",
           "pack_params", "CSRGraph", "build_csr", "get_csr"]
