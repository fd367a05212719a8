"""The C-ABI library loads and exports every symbol include/gat_amd.h declares;
argument validation and layout queries that need no GPU.  CPU only."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "gat_amd.h")


def header_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^int\s+(gat_\w+)\s*\(", text, flags=re.M)))


def test_library_built_and_exports_header_symbols():
    from atmlgraphattentionnetworks_amd import _lib
    assert os.path.exists(_lib.LIB_PATH), "run python -m atmlgraphattentionnetworks_amd.build"
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                        text=True, check=True).stdout
    exported = set(re.findall(r"\bT (gat_\w+)", nm))
    declared = header_functions()
    assert declared, "no functions parsed from the header"
    for name in declared:
        assert name in exported, f"{name} declared in gat_amd.h but not exported"
    # the ctypes binding covers exactly the header
    assert sorted(_lib.SIGNATURES) == declared


def test_load_and_version():
    from atmlgraphattentionnetworks_amd import _lib
    lib = _lib.load()
    assert lib.gat_abi_version() == _lib.GAT_ABI_VERSION


@pytest.mark.parametrize("H,F,ld,s_off", [(8, 8, 72, 64), (4, 8, 36, 32), (1, 7, 12, 8),
                                          (3, 5, 20, 16), (32, 8, 288, 256), (16, 2, 48, 32)])
def test_table_layout(H, F, ld, s_off):
    from atmlgraphattentionnetworks_amd import _lib
    assert _lib.table_layout(H, F) == (ld, s_off)


def test_argument_validation_without_gpu():
    from atmlgraphattentionnetworks_amd import _lib
    lib = _lib.load()
    # bad sizes are rejected before anything touches a device
    assert lib.gat_project(None, -1, 4, None, None, None, None, None, None, 2, 2, None, 4, None,
                           2, None, None) == _lib.GAT_EINVAL
    assert lib.gat_project(None, 10, 4, None, None, None, None, None, None, 65, 2, None, 132,
                           None, 65, None, None) == _lib.GAT_EUNSUPPORTED
    assert lib.gat_project(None, 10, 4, None, None, None, None, None, None, 2, 3, None, 6,
                           None, 2, None, None) == _lib.GAT_EINVAL  # ld_wh not 16-B aligned
    def E(rb, re_, ld_wh, s_src, ld_s):
        return lib.gat_edge_aggregate(None, None, None, rb, re_, None, ld_wh, s_src, ld_s, None,
                                      None, None, 2, 2, 1, 0.2, None, None, None, 0, None)
    assert E(0, 10, 2, 1, 2) == _lib.GAT_EINVAL  # ld_wh < H*F
    assert E(0, 10, 4, 1, 1) == _lib.GAT_EINVAL  # ld_s < H
    assert E(0, 10, 4, None, 2) == _lib.GAT_EINVAL  # neither s_src nor (a_src, c_src)
    assert E(5, 5, 4, 1, 2) == _lib.GAT_OK  # zero rows: nothing to launch
    with pytest.raises(_lib.GatLibraryError):
        _lib.check(_lib.GAT_EUNSUPPORTED, "x")


def test_csr_workspace_size():
    from atmlgraphattentionnetworks_amd import _lib
    small = _lib.csr_workspace_size(1000, 100)
    big = _lib.csr_workspace_size(10_000_000, 200_000)
    assert 4 * 1000 * 4 <= small < big
    with pytest.raises(_lib.GatLibraryError):
        _lib.csr_workspace_size(2**31, 10)
