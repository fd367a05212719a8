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


@pytest.mark.parametrize("fin,H,F,nbytes", [(602, 8, 8, 3 * 64 * 640 * 2), (200, 4, 8, 3 * 32 * 256 * 2),
                                            (129, 8, 8, 3 * 64 * 192 * 2), (128, 8, 8, 0),
                                            (50, 8, 8, 0), (602, 4, 4, 0), (602, 8, 12, 0)])
def test_project_workspace_size(fin, H, F, nbytes):
    """gat_project_workspace_size (ABI 8): the pre-split W planes [3][16 NT][round_up(Fin, 64)]
    bf16 for Fin > 128 with 2 or 4 column tiles of 16 (H*F in (16, 32] or (48, 64]), else 0."""
    from atmlgraphattentionnetworks_amd import _lib
    assert _lib.project_workspace_bytes(fin, H, F) == nbytes


def test_project_ex_and_merge_ex_validate_without_gpu():
    """gat_project_ex / gat_edge_merge_ex reject bad arguments before any launch."""
    from atmlgraphattentionnetworks_amd import _lib
    lib = _lib.load()

    def P(n, slices, ld, chunk_rows, chunk_stride, heads=8, f=8):
        return lib.gat_project_ex(None, n, 16, None, None, None, None, None, None, heads, f, slices,
                                  None, ld, None, heads, None, chunk_rows, chunk_stride, None, 0,
                                  None)
    assert P(10, 0, 64, 0, 0) == _lib.GAT_EINVAL          # no slices
    assert P(10, 3, 64, 0, 0) == _lib.GAT_EINVAL          # 64 columns do not split in 3
    assert P(10, 1, 64, 64, 4096) == _lib.GAT_EINVAL      # row chunks need planes
    assert P(10, 2, 32, 64, 4096) == _lib.GAT_EINVAL      # a chunk larger than its block
    assert P(10, 2, 64, 64, 100) == _lib.GAT_EINVAL       # chunk stride below one block
    assert P(10, 1, 64, -1, 0) == _lib.GAT_EINVAL
    assert lib.gat_edge_merge_ex(None, None, None, 0, None, None, 8, 8, 1, None, None, None, None,
                                 None) == _lib.GAT_OK     # no hubs: nothing to launch
    assert lib.gat_edge_merge_ex(None, None, None, 2, None, None, 8, 8, 1, None, None, None, None,
                                 None) == _lib.GAT_EINVAL
    assert lib.gat_edge_merge_ex(None, None, None, 1, None, None, 65, 4, 1, None, None, None, None,
                                 None) == _lib.GAT_EUNSUPPORTED


def test_csr_workspace_size():
    from atmlgraphattentionnetworks_amd import _lib
    small = _lib.csr_workspace_size(1000, 100)
    big = _lib.csr_workspace_size(10_000_000, 200_000)
    assert 4 * 1000 * 4 <= small < big
    with pytest.raises(_lib.GatLibraryError):
        _lib.csr_workspace_size(2**31, 10)


def test_training_entry_points_validate_without_gpu():
    """The training and backward entry points reject bad arguments before any
    launch (so these calls need no device)."""
    from atmlgraphattentionnetworks_amd import _lib
    lib = _lib.load()
    EINVAL, EUNS, OK = _lib.GAT_EINVAL, _lib.GAT_EUNSUPPORTED, _lib.GAT_OK

    def ex(act=0, p=0.5, rows=(0, 10), ld_wh=8):
        return lib.gat_edge_aggregate_ex(None, None, None, rows[0], rows[1], None, ld_wh, 1, 2,
                                         None, None, None, 2, 4, 1, act, 0.2, p, 1, None, None,
                                         None, None, None, 0, None)
    assert ex(act=7) == EINVAL  # unknown score activation
    assert ex(p=1.5) == EINVAL and ex(p=-0.1) == EINVAL  # dropout outside [0, 1]
    assert ex(ld_wh=4) == EINVAL  # ld_wh < heads * f
    assert ex(rows=(3, 3)) == OK  # nothing to do

    def rows_bwd(act=0, p=0.0, heads=2, f=4):
        return lib.gat_edge_backward_rows(None, None, None, 0, 10, None, None, 8, None, 2, None,
                                          None, None, None, None, None, heads, f, 1, act, 0.2, p,
                                          0, None, None, None, 0, None)
    assert rows_bwd(act=9) == EINVAL
    assert rows_bwd(p=2.0) == EINVAL
    assert rows_bwd(heads=65, f=1) == EUNS

    ld = ctypes.c_int()
    assert lib.gat_bwd_table_layout(8, 8, 1, ctypes.byref(ld)) == OK and ld.value == 64 + 32
    assert lib.gat_bwd_table_layout(8, 8, 0, ctypes.byref(ld)) == OK and ld.value == 8 + 32
    assert lib.gat_bwd_table_layout(0, 8, 0, ctypes.byref(ld)) == EINVAL
    # recompute backward: a bad table stride is EINVAL, an unsupported shape EUNSUPPORTED
    def tgt(f=8, ld_t=96, slope=0.2):
        return lib.gat_bwd_targets(None, None, None, 0, 10, None, 64, None, None, None, None,
                                   None, None, 8, f, 1, slope, 0.0, 0, None, None, None, ld_t, 0,
                                   None)
    assert tgt(ld_t=90) == EINVAL
    assert tgt(f=7, ld_t=96) == EUNS  # f % 4 != 0 -> stored-coefficient path
    assert tgt(slope=-0.5) == EUNS
    # kink-sum training forward and its edge-free pass 1: missing outputs or a
    # bad dropout probability are EINVAL before any launch
    def train(p=0.0, q=None):
        return lib.gat_edge_aggregate_train(None, None, None, 0, 10, None, 64, 8, 8, None, 8, 8,
                                            1, 0.2, p, 0, None, None, None, 8, 8, q, 8, 0, None)
    assert train(q=None) == EINVAL  # q_heads required (for a non-empty row range)
    assert train(p=1.5, q=8) == EINVAL
    def table(f=8, ld_t=96, n=10, ptr=8):
        return lib.gat_bwd_table(ptr, 8, 8, 8, 8, 8, n, 8, f, 1, 8, 8, ld_t, None)
    assert table(ptr=None) == EINVAL
    assert table(ld_t=92) == EINVAL
    assert table(f=6, ld_t=96) == EUNS  # f % 4 != 0
    assert table(n=0) == OK  # nothing to do
    parts = ctypes.c_int()
    assert lib.gat_bwd_sources_parts(1000, 8, 8, ctypes.byref(parts)) == OK
    assert parts.value % 4 == 0 and parts.value >= 4
    # workspace queries
    assert _lib.csc_workspace_size(10_000, 1000) > 4 * 4 * 10_000
    assert _lib.weight_grad_workspace_size(44906, 50, 64) > 0
    sz = ctypes.c_size_t()
    assert lib.gat_sum_partials_workspace_size(100, 272, ctypes.byref(sz)) == OK and sz.value == 0
    assert lib.gat_sum_partials_workspace_size(8192, 272, ctypes.byref(sz)) == OK
    assert sz.value == 32 * 272 * 4
    assert lib.gat_sum_partials(None, 8192, 272, None, None, 0, None) == _lib.GAT_EWORKSPACE
    assert lib.gat_dropout_seed_next(None, None, None) == EINVAL


C_DEMO = r"""
#include <stdio.h>
#include "gat_amd.h"
int main(void) {
    int ld = 0, s_off = 0, ld_t = 0;
    size_t bytes = 0;
    if (gat_abi_version() != GAT_ABI_VERSION) return 1;
    if (gat_table_layout(8, 8, &ld, &s_off) != GAT_OK || ld != 72 || s_off != 64) return 2;
    if (gat_bwd_table_layout(8, 8, 1, &ld_t) != GAT_OK || ld_t != 96) return 3;
    if (gat_csr_workspace_size(1226368, 44906, &bytes) != GAT_OK || bytes == 0) return 4;
    if (gat_project(0, -1, 4, 0, 0, 0, 0, 0, 0, 2, 2, 0, 4, 0, 2, 0, 0) != GAT_EINVAL) return 5;
    printf("c-abi ok %d %d %zu\n", ld, ld_t, bytes);
    return 0;
}
"""


def test_header_compiles_and_links_from_plain_c(tmp_path):
    """The boundary is consumable from C: a program compiled with gcc against
    include/gat_amd.h alone links libgat_amd.so and calls the host-side entry
    points (layouts, workspace sizes, argument validation)."""
    from atmlgraphattentionnetworks_amd import _lib
    src = tmp_path / "demo.c"
    src.write_text(C_DEMO)
    exe = tmp_path / "demo"
    libdir = os.path.dirname(_lib.LIB_PATH)
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    str(src), "-L", libdir, "-l:libgat_amd.so", "-Wl,-rpath," + libdir,
                    "-o", str(exe)], check=True, capture_output=True, text=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    assert r.stdout.startswith("c-abi ok 72 96")


def test_every_library_knob_is_registered():
    """Every GAT_* knob the HIP sources read must be in the snapshot registry
    (gat_abi.hip kKnobNames): knob() returns null for an unregistered name, so
    an A/B through such a knob silently runs the default path in both arms."""
    import glob
    import re
    csrc = os.path.join(ROOT, "atmlgraphattentionnetworks_amd", "csrc")
    used = set()
    for path in glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.h")):
        text = open(path).read()
        used |= set(re.findall(r'(?:knob|kernel_choice)\("(GAT_[A-Z0-9_]+)"', text))
    abi = open(os.path.join(csrc, "gat_abi.hip")).read()
    reg = abi[abi.index("kKnobNames[]"):abi.index("};", abi.index("kKnobNames[]"))]
    registered = set(re.findall(r'"(GAT_[A-Z0-9_]+)"', reg))
    assert used, "no knob uses found"
    assert used <= registered, f"unregistered knobs: {sorted(used - registered)}"
