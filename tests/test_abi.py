"""The C-ABI library loads without a GPU and exports exactly what include/*.h declares."""
import ctypes
import os
import re

from conftest import ROOT


def _declared():
    names = set()
    for f in os.listdir(os.path.join(ROOT, "include")):
        if f.endswith(".h"):
            src = open(os.path.join(ROOT, "include", f)).read()
            src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
            names |= set(re.findall(r"\b(mmpde_[a-z0-9_]+)\s*\(", src))
    return names


def test_header_declares_entry_points():
    names = _declared()
    for must in ("mmpde_knn_graph", "mmpde_knn_query", "mmpde_gnn_forward", "mmpde_gnn_edge_mean",
                 "mmpde_dmm_mesh_graph", "mmpde_dmm_mesh_array", "mmpde_itp_interp"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from mmpde_amd import _lib

    h = ctypes.CDLL(_lib.LIB_PATH)
    for name in _declared():
        assert hasattr(h, name), name
    assert set(_lib.EXPORTS) == _declared()


def test_version_and_status_strings_without_gpu():
    from mmpde_amd import _lib

    lib = _lib.lib()
    assert lib.mmpde_version() == _lib.ABI_VERSION
    assert lib.mmpde_status_string(0) == b"ok"
    assert lib.mmpde_status_string(-1) == b"invalid argument"
    # sizing helpers are pure host arithmetic
    # 8 [n, 128] buffers, per-row maxima (row_max_floats = 2000) plus one
    # 32-B range record per 16-row tile (63 tiles), 16 layers' images
    assert lib.mmpde_gnn_workspace_bytes(1000) == 8 * 1000 * 128 * 4 + (2000 + 8 * 63) * 4 + 16 * 395776
    assert lib.mmpde_gnn_pack_bytes(6) == 6 * 395776
    assert lib.mmpde_itp_pack_bytes() > 0


def test_null_arguments_are_rejected_before_launch():
    from mmpde_amd import _lib

    lib = _lib.lib()
    assert lib.mmpde_knn_graph(None, 1, 100, 35, None, None, None) == -1
    assert lib.mmpde_gnn_edge_mean(None, None, None, 10, 35, None, None, None, None) == -1
    assert lib.mmpde_linear_skinny(None, 1, 1, 1, None, 1, None, 1, 0, None, 1, None) == -1
    assert lib.mmpde_gnn_edge_mean_deg(None, None, None, None, 10, 35, None, None, None, None) == -1
    assert lib.mmpde_gnn_edge_backward(None, None, None, None, 10, 35, None, None, None, None,
                                       None, None, None, None, None) == -1
    assert lib.mmpde_gnn_edge_source_sum(None, None, None, 10, None, None) == -1
    # fp16x3 edge backward: null pointers and an unknown GEMM mode refused before any launch
    assert lib.mmpde_gnn_edge_backward_ex(None, None, None, None, 10, 35, None, None, None, None, None,
                                          None, None, None, 1, None) == -1
    assert lib.mmpde_gnn_edge_backward_ex(None, None, None, None, 10, 35, None, None, None, None, None,
                                          None, None, None, 7, None) == -1
    assert lib.mmpde_gnn_edge_backward_sorted(None, None, None, None, 10, 35, None, None, None, None, None,
                                              None, None, None, None, None, 1, None) == -1
    assert lib.mmpde_gnn_edge_source_sum_sorted(None, None, 10, None, None) == -1
    assert lib.mmpde_rows_grad_weight(None, 1, 10, 4, None, 1, 4, None, None, None, 0, None) == -1
    assert lib.mmpde_batch_norm_rows_train(None, None, 10, 128, None, None, 1e-5, 0.1, None, None, None, None,
                                           None, 0, None) == -1
    assert lib.mmpde_batch_norm_rows_backward(None, None, None, 10, 128, None, None, None, None, None, None, 0,
                                              None) == -1
    assert lib.mmpde_reverse_adjacency(None, 10, 35, None, 10, None, None, None, None, 0, None, None) == -1


def test_edge_backward_partials_sizing_without_gpu():
    from mmpde_amd import _lib

    g = ctypes.c_int(0)
    n = _lib.lib().mmpde_gnn_edge_backward_partials(ctypes.byref(g))
    # per-workgroup dW2 / db2 partials, then the fp16x3 mode's two W2 images
    # (128 x 128 fp16 hi / lo + 128 column scales each), W2^T, the maxima and
    # their per-workgroup partials
    extra = 2 * (128 * 128 * 4 + 128 * 4) // 4 + 128 * 128 + 64 + 3 * 1024
    assert g.value > 0 and n == g.value * (128 * 128 + 128) + extra
