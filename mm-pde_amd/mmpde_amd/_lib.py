"""ctypes binding of libmmpde_hip.so (the C-ABI declared in include/mmpde_hip.h).

The product path has no CPU fallback: every op checks that its tensors live on
a ROCm device and raises ``HipExtensionMissing`` if the gfx950 library is not
built / loadable.  Device memory and the stream come from PyTorch (the current
torch stream is passed to every launch); the library itself never allocates.
"""
from __future__ import annotations

import ctypes
import os

import torch

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libmmpde_hip.so")
ABI_VERSION = 12100

ACT_NONE, ACT_TANH, ACT_RELU, ACT_ELU = 0, 1, 2, 3
PAD_ZEROS, PAD_CIRCULAR = 0, 1
# message_net_2 edge GEMM arithmetic (include/mmpde_hip.h MMPDE_EDGE_GEMM_*)
EDGE_GEMM = {"f32": 0, "f16x3": 1}

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I = ctypes.c_int
_F = ctypes.c_float


class HipExtensionMissing(RuntimeError):
    """libmmpde_hip.so is absent or cannot be loaded (run __graft_entry__.build())."""


class MmpdeError(RuntimeError):
    pass


# --------------------------------------------------------------------------- structs
class GnnScales(ctypes.Structure):
    _fields_ = [("inv_lx", _F), ("inv_ly", _F), ("inv_tmax", _F), ("tw", _I), ("pos_xy", _I),
                ("t", _F), ("t_ptr", _P)]


class GnnEmbedParams(ctypes.Structure):
    _fields_ = [(n, _P) for n in ("w0", "b0", "bn1_w", "bn1_b", "bn1_rm", "bn1_rv", "w3", "b3",
                                  "bn4_w", "bn4_b", "bn4_rm", "bn4_rv")] + [("eps", _F)]


class GnnLayerParams(ctypes.Structure):
    _fields_ = [(n, _P) for n in ("msg1_w", "msg1_b", "msg2_w", "msg2_b", "upd1_w", "upd1_b",
                                  "upd2_w", "upd2_b", "bn_w", "bn_b", "bn_rm", "bn_rv")] + \
        [("eps", _F), ("msg1_ld", _I64), ("upd1_ld", _I64)]


class GnnHeadParams(ctypes.Structure):
    _fields_ = [(n, _P) for n in ("c0_w", "c0_b", "c2_w", "c2_b", "c4_w", "c4_b")] + \
        [("out_scale", _F), ("out_scales", _P), ("tw", _I)]


_P3 = _P * 3


class GnnExec(ctypes.Structure):
    """mmpde_gnn_exec: optional per-layer hipEvents + the edge-GEMM arithmetic."""
    _fields_ = [("edge_begin", ctypes.POINTER(_P)), ("edge_end", ctypes.POINTER(_P)),
                ("edge_gemm", _I), ("packed", _P), ("node_end", ctypes.POINTER(_P)),
                ("degree", _P), ("seg_n", _I64)]


class DmmGraphBranch(ctypes.Structure):
    _fields_ = [(n, _P) for n in ("emb0_w", "emb0_b", "emb1_w", "emb1_b", "emb1_rm", "emb1_rv",
                                  "emb3_w", "emb3_b", "emb4_w", "emb4_b", "emb4_rm", "emb4_rv")] + \
        [(n, _P3) for n in ("g_msg1_w", "g_msg1_b", "g_msg2_w", "g_msg2_b", "g_upd1_w", "g_upd1_b",
                            "g_upd2_w", "g_upd2_b", "g_bn_w", "g_bn_b", "g_bn_rm", "g_bn_rv")] + \
        [("n_gnn_layers", _I)] + \
        [(n, _P) for n in ("dec0_w", "dec0_b", "dec1_w", "dec1_b", "om0_w", "om0_b", "om2_w",
                           "om2_b", "om4_w", "om4_b")] + [("eps", _F)]


class DmmArrayBranch(ctypes.Structure):
    _fields_ = [(n, _P) for n in ("c0_w", "c0_b", "c1_w", "c1_b", "c2_w", "c2_b", "c3_w", "c3_b",
                                  "fc2_w", "fc2_b", "fc3_w", "fc3_b")] + [("s", _I)]


class DmmHead(ctypes.Structure):
    _fields_ = [("t0_w", _P), ("t0_b", _P), ("t1_w", _P), ("t1_b", _P), ("th", _I),
                ("latent", _I), ("o0_w", _P), ("o0_b", _P), ("o1_w", _P), ("hidden", _I)]


class ItpMlp(ctypes.Structure):
    _fields_ = [(n, _P) for n in ("w0", "b0", "w1", "b1", "w2", "b2")]


class RgemmArgs(ctypes.Structure):
    """mmpde_rgemm_args (include/mmpde_hip.h)."""
    _fields_ = [("m", _I64), ("kh", _I), ("layout", _I), ("w", _P * 2), ("ldw", _I64),
                ("a", _P * 2), ("amask", _P * 2), ("lda", _I64 * 2), ("parts", _I),
                ("out", _P * 2), ("ldo", _I64 * 2), ("wc", _I64 * 2), ("wk", _I64 * 2),
                ("ncols", _I * 2), ("bias", _P * 2), ("omask", _P * 2), ("ldom", _I64 * 2),
                ("accumulate", _I * 2), ("relu", _I), ("xs", _P), ("ldxs", _I64), ("ns", _I * 2),
                ("xw", _P * 2), ("ldxw", _I64), ("xscale", _F * 2)]


class RgemmTnArgs(ctypes.Structure):
    """mmpde_rgemm_tn_args (include/mmpde_hip.h)."""
    _fields_ = [("m", _I64), ("chunk_rows", _I), ("gcols", _I), ("g", _P), ("gmask", _P), ("ldg", _I64),
                ("nseg", _I), ("x", _P * 3), ("ldx", _I64 * 3), ("kx", _I * 3), ("dwcol", _I64 * 3),
                ("xs", _P), ("ldxs", _I64), ("ns", _I), ("dwcol_s", _I64), ("sign_s", _F),
                ("accumulate_s", _I), ("dw", _P), ("lddw", _I64), ("db", _P)]


RGEMM_NT, RGEMM_NN = 0, 1


# --------------------------------------------------------------------------- loader
_SIGS = {
    "mmpde_version": (_I, []),
    "mmpde_status_string": (ctypes.c_char_p, [_I]),
    "mmpde_knn_graph": (_I, [_P, _I64, _I64, _I, _P, _P, _P]),
    "mmpde_knn_candidates": (_I, [_P, _P, _I64, _P, _P]),
    "mmpde_knn_moved_cells_bytes": (_I64, [_I64]),
    "mmpde_knn_moved_cells": (_I, [_P, _P, _I64, _I64, _P, _P]),
    "mmpde_knn_table_misses": (_I, [_P, _I64, _P, _P]),
    "mmpde_knn_graph_cand_scratch_bytes": (_I64, [_I64, _I64]),
    "mmpde_knn_skip_threshold": (_I, [_P, _P, _I64, _P, _I, _I, _P, _P]),
    "mmpde_knn_graph_cand": (_I, [_P, _P, _P, _F, _I64, _I64, _I, _P, _P, _P, _P, _P]),
    "mmpde_knn_query_cand": (_I, [_P, _P, _P, _P, _P, _F, _I64, _I64, _I, _P, _P, _P, _P, _P]),
    "mmpde_knn_query": (_I, [_P, _P, _I64, _I64, _I64, _I, _P, _P, _P]),
    "mmpde_edge_index_from_nbr": (_I, [_P, _I64, _I, _P, _P]),
    "mmpde_linear_skinny": (_I, [_P, _I64, _I64, _I64, _P, _I64, _P, _I64, _I, _P, _I64, _P]),
    "mmpde_linear_skinny_workspace_bytes": (_I64, [_I64, _I64, _I64]),
    "mmpde_linear_skinny_ws": (_I, [_P, _I64, _I64, _I64, _P, _I64, _P, _I64, _I, _P, _I64, _P, _I64,
                                    _P]),
    "mmpde_gnn_edge_backward_ex": (_I, [_P, _P, _P, _P, _I64, _I, _P, _P, _P, _P, _P, _P, _P, _P, _I, _P]),
    "mmpde_traj_mse": (_I, [_P, _P, _I64, _I64, _P, _P]),
    "mmpde_conv2d": (_I, [_P, _I64, _I, _I, _I, _P, _P, _I, _I, _I, _I, _P, _I, _P, _P]),
    "mmpde_resample_bilinear": (_I, [_P, _I64, _I, _I, _I, _I, _P, _P]),
    "mmpde_conv2d_ex": (_I, [_P, _I64, _I, _I, _I, _P, _P, _I, _I, _I, _I, _I, _P, _I, _I, _P, _P]),
    "mmpde_conv2d_grad_weight": (_I, [_P, _I64, _I, _I, _I, _P, _I, _I, _I, _I, _P, _P, _P]),
    "mmpde_rows_grad_weight_workspace_bytes": (_I64, [_I64, _I, _I]),
    "mmpde_reverse_adjacency_scratch_bytes": (_I64, [_I64, _I, _I64]),
    "mmpde_reverse_adjacency": (_I, [_P, _I64, _I, _P, _I64, _P, _P, _P, _P, _I64, _P, _P]),
    "mmpde_gnn_edge_backward_sorted": (_I, [_P, _P, _P, _P, _I64, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                           _I, _P]),
    "mmpde_gnn_edge_source_sum_sorted": (_I, [_P, _P, _I64, _P, _P]),
    "mmpde_rows_grad_weight": (_I, [_P, _I64, _I64, _I, _P, _I64, _I, _P, _P, _P, _I64, _P]),
    "mmpde_batch_norm_rows_workspace_bytes": (_I64, [_I64, _I]),
    "mmpde_batch_norm_rows_train": (_I, [_P, _P, _I64, _I, _P, _P, _F, _F, _P, _P, _P, _P, _P, _I64, _P]),
    "mmpde_batch_norm_rows_backward": (_I, [_P, _P, _P, _I64, _I, _P, _P, _P, _P, _P, _P, _I64, _P]),
    "mmpde_rgemm": (_I, [_P, _P]),
    "mmpde_rgemm_tn_workspace_bytes": (_I64, [_I64, _I, _I]),
    "mmpde_rgemm_tn": (_I, [_P, _P, _I64, _P]),
    "mmpde_rows_small": (_I, [_P, _I64, _I64, _I, _P, _I64, _I, _P, _I, _P, _I64, _P]),
    "mmpde_outer_rows": (_I, [_P, _I64, _P, _I64, _I, _I64, _I64, _P, _I64, _P, _P]),
    "mmpde_transpose": (_I, [_P, _I64, _I64, _I64, _P, _I64, _P]),
    "mmpde_tanh_bwd": (_I, [_P, _P, _I64, _P, _P]),
    "mmpde_head_train_workspace_bytes": (_I64, [_I64]),
    "mmpde_head_train_forward": (_I, [_P, _I64, _I64, _P, _P, _P, _P, _P, _P, _P, _P]),
    "mmpde_head_train_backward": (_I, [_P, _I64, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _I64, _P, _P, _I64,
                                       _P]),
    "mmpde_gnn_workspace_bytes": (_I64, [_I64]),
    "mmpde_gnn_embed": (_I, [_P, _P, _I64, GnnScales, _P, _P, _P, _P]),
    "mmpde_gnn_layer": (_I, [_P, _P, _P, _I64, _I, _P, GnnScales, _P, _P, _P, _P]),
    "mmpde_gnn_edge_mean": (_I, [_P, _P, _P, _I64, _I, _P, _P, _P, _P]),
    "mmpde_gnn_edge_mean_deg": (_I, [_P, _P, _P, _P, _I64, _I, _P, _P, _P, _P]),
    "mmpde_gnn_edge_mean_workspace_bytes": (_I64, [_I64, _I]),
    "mmpde_gnn_edge_mean_ex": (_I, [_P, _P, _P, _P, _I64, _I, _P, _P, _P, _P, _I, _P, _I64, _P]),
    "mmpde_gnn_edge_backward_partials": (_I64, [ctypes.POINTER(_I)]),
    "mmpde_gnn_edge_backward": (_I, [_P, _P, _P, _P, _I64, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "mmpde_gnn_edge_source_sum": (_I, [_P, _P, _P, _I64, _P, _P]),
    "mmpde_segment_sum": (_I, [_P, _I64, _P, _P, _I64, _P, _P]),
    "mmpde_gnn_head": (_I, [_P, _I64, _P, _P, _P]),
    "mmpde_gnn_forward": (_I, [_P, _P, _I64, _I, _P, GnnScales, _P, _P, _I, _P, _P, _P, _P]),
    "mmpde_gnn_pack_bytes": (_I64, [_I]),
    "mmpde_gnn_pack_f16x3": (_I, [_P, _I, _P, _P]),
    "mmpde_gnn_forward_ex": (_I, [_P, _P, _I64, _I, _P, GnnScales, _P, _P, _I, _P, _P, _P, _P,
                                  _P]),
    "mmpde_dmm_workspace_bytes": (_I64, [_I64, _I64, _I, _I]),
    "mmpde_dmm_mesh_graph": (_I, [_P, _P, _I64, _I64, _P, _I, _P, _P, _P, _P, _P]),
    "mmpde_dmm_mesh_array": (_I, [_P, _P, _I64, _I64, _P, _P, _P, _P, _P]),
    "mmpde_dmm_head_cache_bytes": (_I64, [_I64, _I]),
    "mmpde_radius_graph": (_I, [_P, _I64, _I64, _F, _I, _P, _P, _P]),
    "mmpde_dmm_head_prepare": (_I, [_P, _I64, _P, _P, _P, _P]),
    "mmpde_dmm_mesh_graph_cached": (_I, [_P, _P, _I64, _I64, _P, _I, _P, _P, _P, _P, _P, _P]),
    "mmpde_dmm_mesh_array_cached": (_I, [_P, _P, _I64, _I64, _P, _P, _P, _P, _P, _P]),
    "mmpde_dmm_branch_graph": (_I, [_P, _P, _I64, _I64, _P, _I, _P, _P, _P, _P, _P]),
    "mmpde_dmm_branch_array": (_I, [_P, _I64, _P, _P, _P, _P, _P]),
    "mmpde_dmm_phi_workspace_bytes": (_I64, [_I64, _I64, _I, _I, _I]),
    "mmpde_dmm_phi": (_I, [_P, _I64, _P, _I64, _P, _P, _P, _P, _P, _P]),
    "mmpde_itp_pack_bytes": (_I64, []),
    "mmpde_itp_pack": (_I, [_P, _P, _P]),
    "mmpde_itp_interp": (_I, [_P, _P, _P, _P, _I64, _I64, _I64, _P, _P, _P, _P]),
    "mmpde_itp_interp_ex": (_I, [_P, _P, _P, _P, _I64, _I64, _I64, _P, _P, _P, _P, _P]),
    "mmpde_softmax_interp": (_I, [_P, _I64, _I64, _P, _I64, _P, _I64, _F, _P, _P]),
    "mmpde_softmax_interp_grad": (_I, [_P, _I64, _I64, _P, _I64, _P, _I64, _F, _P, _P, _P]),
}

EXPORTS = tuple(_SIGS)
_LIB = None


def lib():
    """Load (once) and return the ctypes handle; raise loudly if unavailable."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise HipExtensionMissing(
                f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; "
                f"g.build()'` (hipcc --offload-arch=gfx950)")
        try:
            h = ctypes.CDLL(LIB_PATH)
        except OSError as e:  # pragma: no cover - depends on the box
            raise HipExtensionMissing(f"cannot load {LIB_PATH}: {e}") from e
        for name, (res, args) in _SIGS.items():
            f = getattr(h, name)
            f.restype = res
            f.argtypes = args
        v = h.mmpde_version()
        if v // 100 != ABI_VERSION // 100:
            raise HipExtensionMissing(f"ABI mismatch: library {v}, bindings {ABI_VERSION}")
        _LIB = h
    return _LIB


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().mmpde_status_string(rc).decode()
        raise MmpdeError(f"{what} failed: {msg} (status {rc})")


def stream(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_device(*tensors):
    """The HIP path runs only on ROCm device tensors; no CPU fallback exists."""
    for t in tensors:
        if t is not None and (not isinstance(t, torch.Tensor) or not t.is_cuda):
            raise RuntimeError("mmpde_amd kernels need ROCm device tensors (no CPU fallback); "
                               "move the model and inputs to a cuda device")
    lib()


def ptr(t):
    if t is None:
        return None
    return t.data_ptr()


def f32c(t: torch.Tensor) -> torch.Tensor:
    t = t.detach()
    if t.dtype != torch.float32:
        t = t.float()
    if not t.is_contiguous() or t.data_ptr() % 16:
        t = t.contiguous().clone() if t.data_ptr() % 16 else t.contiguous()
    return t
