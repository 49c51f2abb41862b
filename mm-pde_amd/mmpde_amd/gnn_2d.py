"""MP_PDE_Solver_2D on the HIP kernels (drop-in for reference gnn_2d.py:19-141).

Module tree, parameter names, ``state_dict`` keys, constructor arguments and
``__repr__() == 'GNN'`` (the type switch of train_helper_2d.py:107,174) match the
reference, so reference checkpoints load unchanged.  ``forward(data)`` runs the
whole solver in one C-ABI call (mmpde_gnn_forward): embedding, 6 fused
message-passing layers, Conv1d head -- eval-mode semantics (BatchNorm with
running statistics), fp32 throughout.  There is no CPU / eager fallback.

In ``train()`` mode (train_helper_2d.py:107-128) the forward is differentiable:
the edge stage -- message_net_2 over every in-edge and the mean
(gnn_2d.py:59-63, aggr='mean') -- runs as the ``EdgeMean`` autograd.Function on
HIP kernels (mmpde_gnn_edge_mean_ex forward, mmpde_gnn_edge_backward_sorted
+ mmpde_gnn_edge_source_sum_sorted backward: no per-edge activation is
stored); the
per-node work runs as autograd Functions over HIP kernels and library GEMMs:
message_net_1 factored into its target and source halves and the update MLPs
as ops.LinearRows (row-chunked weight gradients), every BatchNorm1d -- with the
layer's residual add fused in -- as ops.BatchNormRows
(mmpde_batch_norm_rows_train / _backward), the Conv1d head as unfold +
LinearRows (skinny weight gradients on mmpde_rows_grad_weight).
"""
from __future__ import annotations

import ctypes
from types import SimpleNamespace

import torch
from torch import nn

from . import _lib as L

# Diagnostic record (tests only; None in normal use): while it is a list, every
# train-mode forward appends the activation pattern the HIP kernels evaluated
# -- ("emb", z > 0) for the embedding's ReLU of each solver, then per fused GNN
# layer ("layer", a, b, v > 0, upd > 0, relu_mask): message_net_1's halves (the
# z1 = a_i + b_j > 0 pattern), message_net_2's z2 > 0 bits (relu_mask words,
# mmpde_gnn_edge_mean_ex) and update_net_1 / _2's patterns.  The training tests
# feed it to the float64 oracle (oracle/refcpu.py RELU_PATTERN), so gradients
# are compared on one activation pattern.
RELU_RECORD = None

from .ops import (HeadTrain, LinearRows, batch_norm_rows, head_train_fits, linear_train, nbr_table_from_edge_index,
                  reverse_adjacency)


class BatchNorm(nn.Module):
    """Key-compatible stand-in for torch_geometric.nn.BatchNorm (PyG 2.0.3 wraps
    nn.BatchNorm1d as ``.module``; reference gnn_2d.py:51).  The eval forward is
    fused into the HIP layer kernels; this forward serves the training path."""

    def __init__(self, in_channels, eps=1e-5, momentum=0.1, affine=True,
                 track_running_stats=True):
        super().__init__()
        self.module = nn.BatchNorm1d(in_channels, eps, momentum, affine, track_running_stats)

    def forward(self, x):
        return self.module(x)

    def forward_res(self, x, res):
        """module(x + res), the add fused into the HIP BatchNorm in train mode."""
        return batch_norm_rows(self.module, x, res)


class EdgeGraph:
    """A message-passing graph as the HIP edge kernels take it: target-major
    neighbour table nbr int32 [n, k], optional in-degrees int32 [n] (ragged
    tables), and -- built on first use by a backward -- the reverse adjacency.
    checked: the table's sources are known to lie in [0, n) (built by
    nbr_table_from_edge_index, which range-checks them); any other table is
    range-checked once, when its reverse adjacency is built (a source outside
    [0, n) would otherwise lose its gradient silently)."""

    def __init__(self, nbr: torch.Tensor, deg: torch.Tensor | None = None, checked: bool = False):
        self.nbr = nbr.to(torch.int32).contiguous()
        self.deg = deg.to(torch.int32).contiguous() if deg is not None else None
        self.checked = checked
        self._rev = None

    @classmethod
    def of(cls, data, n: int):
        nbr = getattr(data, "nbr", None)
        deg = getattr(data, "deg", None) if nbr is not None else None
        # engine tables (kNN / radius kernels) are marked nbr_checked by the graph creator
        checked = nbr is None or bool(getattr(data, "nbr_checked", False))
        if nbr is None:
            nbr, deg = nbr_table_from_edge_index(data.edge_index, n)
        return cls(nbr, deg, checked)

    def reverse(self):
        if self._rev is None:
            # with the slot positions of the source-major backward
            self._rev = reverse_adjacency(self.nbr, self.deg, check=not self.checked, slot_pos=True)
            self.checked = True
        return self._rev


def _edge_mean_fwd(a, b, w2, b2, graph: EdgeGraph, edge_gemm: str, keep_mask: bool = True):
    """mean_i over the in-edges of relu(W2 relu(a_i + b_j) + b2) (EdgeMean's
    forward): (mean [n, 128], the f16x3 ReLU pattern of message_net_2 or None).
    keep_mask False (no backward will run): no ReLU pattern, and the f16x3
    mode runs the inference forward's wave kernel instead of the ring kernel."""
    n, k = graph.nbr.shape
    mean = torch.empty((n, 128), dtype=torch.float32, device=a.device)
    mode = L.EDGE_GEMM[edge_gemm]
    lib = L.lib()
    wsb = lib.mmpde_gnn_edge_mean_workspace_bytes(n, mode)
    ws = torch.empty((max(wsb, 16) // 4,), dtype=torch.float32, device=a.device) if wsb else None
    # the forward keeps message_net_2's ReLU pattern (16 B per edge) for the
    # backward, which then skips recomputing z2 (and differentiates exactly the
    # function the forward evaluated: its own z2 summation order differs)
    mask = torch.empty((n * k, 4), dtype=torch.int32, device=a.device) if k <= 64 and keep_mask else None
    L.check(lib.mmpde_gnn_edge_mean_ex(L.ptr(a), L.ptr(b), L.ptr(graph.nbr), L.ptr(graph.deg), n, k,
                                       L.ptr(w2), L.ptr(b2), L.ptr(mean), L.ptr(mask), mode, L.ptr(ws), wsb,
                                       L.stream(a.device)),
            "mmpde_gnn_edge_mean_ex")
    return mean, mask


def _edge_mean_bwd(a, b, w2, b2, graph: EdgeGraph, mask, edge_gemm: str, g):
    """(dL/da, dL/db, dL/dW2, dL/db2) of _edge_mean_fwd for dL/dmean = g: the
    per-edge dL/dz1 rows written source-major (slot_pos), then summed per
    source as contiguous runs."""
    n, k = graph.nbr.shape
    dev = a.device
    lib = L.lib()
    ga = torch.empty_like(a)
    gb = torch.empty_like(b)
    gedge = torch.empty((n * k, 128), dtype=torch.float32, device=dev)
    part = torch.empty((lib.mmpde_gnn_edge_backward_partials(None),), dtype=torch.float32, device=dev)
    gw2 = torch.empty((128, 128), dtype=torch.float32, device=dev)
    gb2 = torch.empty((128,), dtype=torch.float32, device=dev)
    st = L.stream(dev)
    rev_off, _, slot_pos = graph.reverse()
    L.check(lib.mmpde_gnn_edge_backward_sorted(L.ptr(a), L.ptr(b), L.ptr(graph.nbr), L.ptr(graph.deg),
                                               n, k, L.ptr(w2), L.ptr(b2), L.ptr(g), L.ptr(slot_pos),
                                               L.ptr(mask), L.ptr(ga), L.ptr(gedge), L.ptr(part),
                                               L.ptr(gw2), L.ptr(gb2), L.EDGE_GEMM[edge_gemm], st),
            "mmpde_gnn_edge_backward_sorted")
    L.check(lib.mmpde_gnn_edge_source_sum_sorted(L.ptr(gedge), L.ptr(rev_off), n, L.ptr(gb), st),
            "mmpde_gnn_edge_source_sum_sorted")
    return ga, gb, gw2, gb2


class EdgeMean(torch.autograd.Function):
    """mean_i = 1/max(deg_i, 1) sum_{e < deg_i} relu(W2 relu(a_i + b_{nbr[i,e]}) + b2):
    message_net_2 over the in-edges and PyG's aggr='mean' (gnn_2d.py:36,59-63),
    with a = the target half and b = the source half of message_net_1's
    pre-activation.  Gradients for a, b, W2 and b2, deterministic; forward and
    backward GEMMs in exact fp32 (edge_gemm 'f32') or the fp16x3 split
    (edge_gemm 'f16x3': mmpde_gnn_edge_mean_ex keeps message_net_2's ReLU
    pattern, 16 B per edge, which mmpde_gnn_edge_backward_sorted reuses instead
    of recomputing z2)."""

    @staticmethod
    def forward(ctx, a, b, w2, b2, graph: EdgeGraph, edge_gemm: str = "f32"):
        n, k = graph.nbr.shape
        if a.shape != (n, 128) or b.shape != (n, 128) or w2.shape != (128, 128):
            raise ValueError("EdgeMean takes a, b [n, 128] and W2 [128, 128]")
        L.require_device(a, b, w2, b2, graph.nbr, graph.deg)
        a, b, w2, b2 = L.f32c(a), L.f32c(b), L.f32c(w2), L.f32c(b2)
        mean, mask = _edge_mean_fwd(a, b, w2, b2, graph, edge_gemm, keep_mask=any(ctx.needs_input_grad[:4]))
        ctx.save_for_backward(a, b, w2, b2)
        ctx.graph = graph
        ctx.mask = mask
        ctx.edge_gemm = edge_gemm
        return mean

    @staticmethod
    def backward(ctx, g):
        a, b, w2, b2 = ctx.saved_tensors
        ga, gb, gw2, gb2 = _edge_mean_bwd(a, b, w2, b2, ctx.graph, ctx.mask, ctx.edge_gemm, L.f32c(g))
        return ga, gb, gw2, gb2, None, None


class GnnLayerTrain(torch.autograd.Function):
    """One train-mode GNN_Layer_FS_2D (gnn_2d.py:53-69; time_window 1, one
    variable, width 128) on HIP kernels, forward and backward:

        a   = h W1[:, :128]^T + (u, x, y, t) W1[:, 256:260]^T + b1     (target half)
        b   = h W1[:, 128:256]^T - (u, x, y) W1[:, 256:259]^T          (source half)
        m   = EdgeMean(a, b)                        (message_net_2 + PyG mean)
        v   = relu([h | m] U1[:, :256]^T + t U1[:, 256] + c1)           (update_net_1)
        upd = relu(v U2^T + c2)                                          (update_net_2)
        h'  = BatchNorm1d_train(h + upd)

    every GEMM on mmpde_rgemm (exact fp32 MFMA; the concatenations read in
    place, bias / ReLU / the ReLU-backward masks / the residual fused), the
    weight gradients on mmpde_rgemm_tn, BatchNorm on the row kernels.  The
    backward accumulates dL/dh (residual + update_net_1 + both message_net_1
    halves) in one buffer.  extras = (u, x/Lx, y/Ly, t/tmax) [n, 4]."""

    @staticmethod
    def forward(ctx, h, extras, w1, b1, w2, b2, u1, c1, u2, c2, bnw, bnb, graph, edge_gemm, bn):
        from . import rows
        L.require_device(h, extras, w1, u1, u2)
        h, extras = L.f32c(h), L.f32c(extras)
        W1, B1, W2, B2 = (L.f32c(t) for t in (w1, b1, w2, b2))
        U1 = torch.nn.functional.pad(u1.detach().float(), (0, 3)).contiguous()   # [128, 260]: 16-B rows
        C1, U2, C2 = L.f32c(c1), L.f32c(u2), L.f32c(c2)
        n = h.shape[0]
        dev = h.device
        st = L.stream(dev)
        P = rows._p
        f32 = dict(dtype=torch.float32, device=dev)
        ab = torch.empty((2, n, 128), **f32)
        a, b = ab[0], ab[1]
        rows.rgemm(n, 64, L.RGEMM_NT, (P(W1), P(W1, 64)), 260, (P(h), P(h, 64)), (128, 128),
                   [dict(out=P(a), ldo=128, wc=0, wk=0, ncols=128, bias=P(B1), ns=4, xw=P(W1, 256)),
                    dict(out=P(b), ldo=128, wc=0, wk=128, ncols=128, ns=3, xw=P(W1, 256), xscale=-1.0)],
                   xs=P(extras), ldxs=4, ldxw=260, stream=st)
        mean, mask = _edge_mean_fwd(a, b, W2, B2, graph, edge_gemm)
        v = torch.empty((n, 128), **f32)
        rows.rgemm(n, 128, L.RGEMM_NT, (P(U1), P(U1, 128)), 260, (P(h), P(mean)), (128, 128),
                   [dict(out=P(v), ldo=128, ncols=128, bias=P(C1), ns=1, xw=P(U1, 256))],
                   relu=True, xs=P(extras, 3), ldxs=4, ldxw=260, stream=st)
        upd = torch.empty((n, 128), **f32)
        rows.rgemm(n, 64, L.RGEMM_NT, (P(U2), P(U2, 64)), 128, (P(v), P(v, 64)), (128, 128),
                   [dict(out=P(upd), ldo=128, ncols=128, bias=P(C2))], relu=True, stream=st)
        # BatchNorm1d(h + upd) in train mode (running statistics as nn.BatchNorm1d)
        factor = 0.0
        if bn.track_running_stats and bn.num_batches_tracked is not None:
            bn.num_batches_tracked.add_(1)
            factor = 1.0 / float(bn.num_batches_tracked) if bn.momentum is None else bn.momentum
        rm = bn.running_mean if bn.track_running_stats else None
        rv = bn.running_var if bn.track_running_stats else None
        lib = L.lib()
        nb = lib.mmpde_batch_norm_rows_workspace_bytes(n, 128) + 3 * 128 * 4
        ws = torch.empty((nb // 4,), **f32)
        stats = torch.empty((4 * 128,), **f32)
        hn = torch.empty((n, 128), **f32)
        BW = L.f32c(bnw) if bnw is not None else None
        L.check(lib.mmpde_batch_norm_rows_train(
            L.ptr(h), L.ptr(upd), n, 128, L.ptr(BW), L.ptr(L.f32c(bnb) if bnb is not None else None),
            float(bn.eps), float(factor), L.ptr(rm), L.ptr(rv), L.ptr(hn), L.ptr(stats), L.ptr(ws), nb, st),
            "mmpde_batch_norm_rows_train")
        if RELU_RECORD is not None:
            RELU_RECORD.append(("layer", a, b, v > 0, upd > 0, mask))
        ctx.save_for_backward(h, extras, a, b, mean, v, upd, stats, W1, B1, W2, B2, U1, U2, BW)
        ctx.graph, ctx.mask, ctx.edge_gemm, ctx.bn_ws = graph, mask, edge_gemm, nb
        ctx.has_bn = (bnw is not None, bnb is not None)
        return hn

    @staticmethod
    def backward(ctx, dhn):
        from . import rows
        h, extras, a, b, mean, v, upd, stats, W1, B1, W2, B2, U1, U2, BW = ctx.saved_tensors
        n = h.shape[0]
        dev = h.device
        st = L.stream(dev)
        P = rows._p
        f32 = dict(dtype=torch.float32, device=dev)
        lib = L.lib()
        dhn = L.f32c(dhn)
        # BatchNorm backward: dx = dL/d(h + upd), the residual's and update's alike
        dx = torch.empty((n, 128), **f32)
        dgam = torch.empty((128,), **f32) if ctx.has_bn[0] else None
        dbet = torch.empty((128,), **f32) if ctx.has_bn[1] else None
        ws = torch.empty((ctx.bn_ws // 4,), **f32)
        L.check(lib.mmpde_batch_norm_rows_backward(L.ptr(h), L.ptr(upd), L.ptr(dhn), n, 128, L.ptr(BW),
                                                   L.ptr(stats), L.ptr(dx), L.ptr(dgam), L.ptr(dbet),
                                                   L.ptr(ws), ctx.bn_ws, st),
                "mmpde_batch_norm_rows_backward")
        # update_net_2: dv = ((dx * [upd > 0]) U2) * [v > 0] (update_net_1's pre-activation gradient)
        dv = torch.empty((n, 128), **f32)
        rows.rgemm(n, 64, L.RGEMM_NN, (P(U2), P(U2, 64 * 128)), 128, (P(dx), P(dx, 64)), (128, 128),
                   [dict(out=P(dv), ldo=128, ncols=128, omask=P(v), ldom=128)],
                   amask=(P(upd), P(upd, 64)), stream=st)
        dU2 = torch.empty((128, 128), **f32)
        dc2 = torch.empty((128,), **f32)
        rows.rgemm_tn(n, P(dx), 128, 128, [(P(v), 128, 128, 0)], dU2, 128, db=dc2, gmask=P(upd), stream=st)
        # update_net_1: dh += dv U1[:, :128] (onto the residual's dx), dmean = dv U1[:, 128:256]
        dmean = torch.empty((n, 128), **f32)
        rows.rgemm(n, 64, L.RGEMM_NN, (P(U1), P(U1, 64 * 260)), 260, (P(dv), P(dv, 64)), (128, 128),
                   [dict(out=P(dx), ldo=128, wc=0, ncols=128, acc=True),
                    dict(out=P(dmean), ldo=128, wc=128, ncols=128)], stream=st)
        dU1 = torch.empty((128, 257), **f32)
        dc1 = torch.empty((128,), **f32)
        rows.rgemm_tn(n, P(dv), 128, 128, [(P(h), 128, 128, 0), (P(mean), 128, 128, 128)], dU1, 257,
                      db=dc1, xs=P(extras, 3), ldxs=4, ns=1, dwcol_s=256, stream=st)
        # message_net_2 + mean
        da, db, dW2, db2 = _edge_mean_bwd(a, b, W2, B2, ctx.graph, ctx.mask, ctx.edge_gemm, dmean)
        # message_net_1 halves: dh += da W1[:, :128] + db W1[:, 128:256]
        rows.rgemm(n, 128, L.RGEMM_NN, (P(W1), P(W1, 128)), 260, (P(da), P(db)), (128, 128),
                   [dict(out=P(dx), ldo=128, wc=0, ncols=128, acc=True)], stream=st)
        dW1 = torch.empty((128, 260), **f32)
        db1 = torch.empty((128,), **f32)
        rows.rgemm_tn(n, P(da), 128, 128, [(P(h), 128, 128, 0)], dW1, 260, db=db1,
                      xs=P(extras), ldxs=4, ns=4, dwcol_s=256, stream=st)
        rows.rgemm_tn(n, P(db), 128, 128, [(P(h), 128, 128, 128)], dW1, 260,
                      xs=P(extras), ldxs=4, ns=3, dwcol_s=256, sign_s=-1.0, accumulate_s=True, stream=st)
        dext = None
        if ctx.needs_input_grad[1]:
            # (u, x, y, t) enter a with W1[:, 256:260], b with -W1[:, 256:259] and v
            # with t U1[:, 256] (u needs it when ItpNet interpolated it, Burgers)
            dext = torch.empty((n, 4), **f32)
            # the halves share one row stride: -W1[:, 256:259] as a padded copy
            nwp = torch.zeros((128, 260), **f32)
            nwp[:, 256:259] = -W1[:, 256:259]
            rows.rgemm(n, 128, L.RGEMM_NN, (P(W1, 256), P(nwp, 256)), 260, (P(da), P(db)), (128, 128),
                       [dict(out=P(dext), ldo=4, ncols=4)], stream=st)
            rows.rgemm(n, 64, L.RGEMM_NN, (P(U1, 256), P(U1, 64 * 260 + 256)), 260, (P(dv), P(dv, 64)),
                       (128, 128), [dict(out=P(dext, 3), ldo=4, ncols=1, acc=True)], stream=st)
        return (dx, dext, dW1, db1, dW2, db2, dU1, dc1, dU2, dc2, dgam, dbet, None, None, None)


class GNN_Layer_FS_2D(nn.Module):  # noqa: N801 - reference name
    """Message-passing layer (reference gnn_2d.py:19-69): message
    relu(W2 relu(W1 cat(h_i, h_j, u_i-u_j, dx, dy, t_i))), mean over the
    in-edges, update h + relu(U2 relu(U1 cat(h, m, t))), BatchNorm."""

    def __init__(self, in_features, out_features, hidden_features, time_window, n_variables):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.hidden_features, self.time_window, self.n_variables = \
            hidden_features, time_window, n_variables
        msg_in = 2 * in_features + time_window + 2 + n_variables
        self.message_net_1 = nn.Sequential(nn.Linear(msg_in, hidden_features), nn.ReLU())
        self.message_net_2 = nn.Sequential(nn.Linear(hidden_features, out_features), nn.ReLU())
        self.update_net_1 = nn.Sequential(
            nn.Linear(in_features + hidden_features + n_variables, hidden_features), nn.ReLU())
        self.update_net_2 = nn.Sequential(nn.Linear(hidden_features, out_features), nn.ReLU())
        self.norm = BatchNorm(hidden_features)
        self._pack_key = None
        self._pack = None

    def supported(self):
        return (self.in_features == self.out_features == self.hidden_features == 128
                and self.time_window == 1 and self.n_variables == 1)

    def _params(self):
        """ctypes parameter block (cached until a parameter changes)."""
        ts = [self.message_net_1[0].weight, self.message_net_1[0].bias,
              self.message_net_2[0].weight, self.message_net_2[0].bias,
              self.update_net_1[0].weight, self.update_net_1[0].bias,
              self.update_net_2[0].weight, self.update_net_2[0].bias,
              self.norm.module.weight, self.norm.module.bias,
              self.norm.module.running_mean, self.norm.module.running_var]
        key = tuple((t.data_ptr(), t._version) for t in ts)
        if key != self._pack_key:
            f = [L.f32c(t) for t in ts]
            u1 = f[4]
            u1p = torch.zeros((u1.shape[0], 260), dtype=torch.float32, device=u1.device)
            u1p[:, :u1.shape[1]] = u1          # row stride 260 keeps rows 16-B aligned
            w1 = f[0]
            if w1.shape[1] % 4:                # 259 + tw columns: pad rows to 16 B too
                w1p = torch.zeros((w1.shape[0], (w1.shape[1] + 3) & ~3), dtype=torch.float32,
                                  device=w1.device)
                w1p[:, :w1.shape[1]] = w1
                w1 = w1p
            keep = [w1] + f[1:4] + [u1p] + f[5:]
            p = L.GnnLayerParams(*[t.data_ptr() for t in keep], float(self.norm.module.eps),
                                 w1.shape[1], 260)
            self._pack, self._pack_key = (p, keep), key
        return self._pack[0]

    def fused_train_ok(self):
        """GnnLayerTrain covers the reference defaults (width 128, time_window 1,
        one variable) with its BatchNorm in training mode (batch statistics,
        running-stat update); a BatchNorm held in eval mode inside a training
        model (e.g. a frozen norm) takes the unfused path, whose BatchNormRows
        applies the running statistics."""
        return (self.in_features == self.out_features == self.hidden_features == 128
                and self.time_window == 1 and self.n_variables == 1 and self.norm.module.training)

    def train_forward_fused(self, h, extras, graph: EdgeGraph, edge_gemm: str = "f32"):
        """gnn_2d.py:53-69 in train mode as one GnnLayerTrain (extras = (u, x/Lx,
        y/Ly, t/tmax) [n, 4])."""
        m1, m2 = self.message_net_1[0], self.message_net_2[0]
        u1, u2 = self.update_net_1[0], self.update_net_2[0]
        bn = self.norm.module
        return GnnLayerTrain.apply(h, extras, m1.weight, m1.bias, m2.weight, m2.bias, u1.weight, u1.bias,
                                   u2.weight, u2.bias, bn.weight, bn.bias, graph, edge_gemm, bn)

    def train_forward(self, h, u, pos_x, pos_y, variables, graph: EdgeGraph, edge_gemm: str = "f32"):
        """Differentiable layer (gnn_2d.py:53-69).  message_net_1 of the edge (i, j)
        is W1 cat(h_i, h_j, u_i - u_j, dx, dy, t_i) + b1 = a_i + b_j with
        a = [h u x y t] Wa^T + b1 and b = [h u x y] Wb^T (Wb holding -W1 on the
        difference columns): two node GEMMs, then the EdgeMean kernels."""
        if self.hidden_features != 128 or self.out_features != 128:
            raise NotImplementedError("HIP edge kernels take hidden = out = 128")
        f, tw = self.in_features, self.time_window
        w1, b1 = self.message_net_1[0].weight, self.message_net_1[0].bias
        wdu = w1[:, 2 * f:2 * f + tw]
        wdxy = w1[:, 2 * f + tw:2 * f + tw + 2]
        wt = w1[:, 2 * f + tw + 2:]
        a = LinearRows.apply(torch.cat((h, u, pos_x, pos_y, variables), -1),
                             torch.cat((w1[:, :f], wdu, wdxy, wt), 1), b1)
        b = LinearRows.apply(torch.cat((h, u, pos_x, pos_y), -1),
                             torch.cat((w1[:, f:2 * f], -wdu, -wdxy), 1), None)
        m2 = self.message_net_2[0]
        mean = EdgeMean.apply(a, b, m2.weight, m2.bias, graph, edge_gemm)
        v = torch.relu(linear_train(torch.cat((h, mean, variables), -1), self.update_net_1[0]))
        upd = torch.relu(linear_train(v, self.update_net_2[0]))
        return self.norm.forward_res(h, upd)

    def forward(self, x, u, pos_x, pos_y, variables, edge_index, batch):
        """Layer-level API of the reference (gnn_2d.py:53-57), any edge_index.
        The fused one-launch layer (mmpde_gnn_layer) takes time_window 1, one
        variable and a grouped fixed-degree graph (knn_graph's layout); any
        other time_window / variable count / ragged or ungrouped edge_index runs
        the two node GEMMs as device torch ops and the edge stage on the HIP
        EdgeMean kernels (the train() path; in-degree 0 gives the PyG mean 0)."""
        L.require_device(x, u, pos_x, pos_y, variables)
        n = x.shape[0]
        nbr, deg = nbr_table_from_edge_index(edge_index, n)
        if self.training or not self.supported() or deg is not None:
            if u.dim() == 1:
                u = u[:, None]
            return self.train_forward(x, u, pos_x, pos_y, variables, EdgeGraph(nbr, deg, checked=True))
        pos = torch.cat((variables, pos_x, pos_y), dim=-1).float().contiguous()
        ws = torch.empty((4 * n * 128,), dtype=torch.float32, device=x.device)
        out = torch.empty((n, 128), dtype=torch.float32, device=x.device)
        p = self._params()
        L.check(L.lib().mmpde_gnn_layer(L.ptr(L.f32c(x)), L.ptr(L.f32c(u).reshape(-1)), L.ptr(pos),
                                        n, nbr.shape[1], L.ptr(nbr), L.GnnScales(1.0, 1.0, 1.0),
                                        ctypes.byref(p), L.ptr(ws), L.ptr(out),
                                        L.stream(x.device)), "mmpde_gnn_layer")
        return out


class MP_PDE_Solver_2D(nn.Module):  # noqa: N801 - reference name
    """Reference gnn_2d.py:72-141.  forward(data) -> [n, time_window]."""

    def __init__(self, pde, time_window=1, hidden_features=128, hidden_layer=6,
                 eq_variables={}):  # noqa: B006 - reference signature
        super().__init__()
        self.pde = pde
        self.out_features = time_window
        self.hidden_features = hidden_features
        self.hidden_layer = hidden_layer
        self.time_window = time_window
        self.eq_variables = eq_variables
        self.gnn_layers = nn.ModuleList(
            GNN_Layer_FS_2D(in_features=hidden_features, hidden_features=hidden_features,
                            out_features=hidden_features, time_window=time_window,
                            n_variables=len(eq_variables) + 1)
            for _ in range(hidden_layer))
        self.embedding_mlp = nn.Sequential(
            nn.Linear(time_window + 3 + len(eq_variables), hidden_features),
            nn.BatchNorm1d(hidden_features), nn.ReLU(),
            nn.Linear(hidden_features, hidden_features), nn.BatchNorm1d(hidden_features))
        self.output_mlp = nn.Sequential(
            nn.Conv1d(1, 4, 16, stride=3), nn.ReLU(),
            nn.Conv1d(4, 8, 12, stride=3), nn.ReLU(),
            nn.Conv1d(8, 1, 8, stride=2))
        self._pack_key = None
        self._pack = None
        self._f16x3 = None
        # GEMM arithmetic of the fused layers: "f32" (exact fp32 MFMA) or "f16x3"
        # (fp32 emulated by scaled fp16 hi/lo splits; include/mmpde_hip.h)
        self.edge_gemm = "f32"

    def __repr__(self):
        return "GNN"

    # ----------------------------------------------------------------- packing
    def out_scales(self) -> torch.Tensor:
        """cumsum(ones(1, tw) * pde.dt * 0.1) evaluated as gnn_2d.py:137-138 (fp32,
        on the host): [tw]."""
        dt = torch.ones(1, self.time_window) * self.pde.dt * 0.1
        return torch.cumsum(dt, dim=1)[0]

    def out_scale(self) -> float:
        """The tw = 1 head scale (pde.dt * 0.1)."""
        return float(self.out_scales()[0])

    def scales(self) -> L.GnnScales:
        one = torch.ones((), dtype=torch.float32)
        return L.GnnScales(float(one / self.pde.Lx), float(one / self.pde.Ly),
                           float(one / self.pde.tmax), self.time_window)

    def device_params(self):
        """(scales, embed, layer array, head) ctypes blocks, cached by parameter
        identity/version."""
        e, o = self.embedding_mlp, self.output_mlp
        ts = [e[0].weight, e[0].bias, e[1].weight, e[1].bias, e[1].running_mean,
              e[1].running_var, e[3].weight, e[3].bias, e[4].weight, e[4].bias,
              e[4].running_mean, e[4].running_var,
              o[0].weight, o[0].bias, o[2].weight, o[2].bias, o[4].weight, o[4].bias]
        layer_params = [g._params() for g in self.gnn_layers]
        key = (tuple((t.data_ptr(), t._version) for t in ts),
               tuple(ctypes.addressof(p) for p in layer_params), self.pde.dt, self.pde.tmax)
        if key != self._pack_key:
            f = [L.f32c(t) for t in ts]
            emb = L.GnnEmbedParams(*[t.data_ptr() for t in f[:12]], float(e[1].eps))
            scl = self.out_scales().to(f[12].device)
            f.append(scl)                      # kept alive with the parameter block
            head = L.GnnHeadParams(*[t.data_ptr() for t in f[12:18]], self.out_scale(),
                                   scl.data_ptr(), self.time_window)
            arr = (L.GnnLayerParams * len(layer_params))(*layer_params)
            self._pack = ((self.scales(), emb, arr, head), f, [g._pack for g in self.gnn_layers])
            self._pack_key = key
            self._f16x3 = None
        return self._pack[0]

    def packed_f16x3(self, device):
        """Split fp16 weight images of every layer (mmpde_gnn_pack_f16x3), rebuilt
        when a parameter changes (device_params refresh)."""
        _, _, arr, _ = self.device_params()
        if self._f16x3 is None:
            nb = L.lib().mmpde_gnn_pack_bytes(len(arr))
            buf = torch.empty((nb // 4,), dtype=torch.float32, device=device)
            L.check(L.lib().mmpde_gnn_pack_f16x3(arr, len(arr), L.ptr(buf), L.stream(device)),
                    "mmpde_gnn_pack_f16x3")
            self._f16x3 = buf
        return self._f16x3

    def check_supported(self):
        if self.hidden_features != 128 or not 1 <= self.time_window <= 16 or \
                len(self.eq_variables):
            raise NotImplementedError("HIP solver supports hidden 128, time_window 1..16, no "
                                      "extra equation variables (reference defaults)")

    # ----------------------------------------------------------------- forward
    def forward(self, data, out: torch.Tensor | None = None, workspace=None, trace=None):
        """gnn_2d.py:119-141 on one C-ABI call.  `data` needs .x [n,1], .pos [n,3]
        and either .nbr (int32 [n,k], plus .deg [n] for a ragged table such as the
        radius graph's) or a PyG .edge_index (any in-degrees).  `trace`: optional
        _lib.GnnExec carrying hipEvents recorded around each layer's fused kernel
        (its edge_gemm field is set from self.edge_gemm)."""
        if self.training:
            return self.train_forward(data)
        call, out, _keep = self._call(data, out, workspace, trace)
        L.check(L.lib().mmpde_gnn_forward_ex(
            call.u, call.pos, call.n, call.k, call.nbr, call.sc, call.emb, call.layers,
            call.n_layers, call.head, call.workspace, call.out, call.exec, L.stream(data.x.device)),
            "mmpde_gnn_forward")
        return out

    def _call(self, data, out, workspace, trace):
        """(mmpde_gnn_forward_ex arguments, out, keep-alive) of one eval forward (see forward)."""
        self.check_supported()
        u, pos = data.x, data.pos
        L.require_device(u, pos)
        n = u.shape[0]
        nbr = getattr(data, "nbr", None)
        deg = getattr(data, "deg", None) if nbr is not None else None
        if nbr is None:
            nbr, deg = nbr_table_from_edge_index(data.edge_index, n)
        if deg is not None:
            L.require_device(deg)
            deg = deg.to(torch.int32).contiguous()
        u = L.f32c(u).reshape(-1)
        pos = L.f32c(pos)
        sc, emb, arr, head = self.device_params()
        t_slot = None
        if pos.shape[-1] == 2:   # (x, y) rows, one t for every node (the rollout's form)
            t, t_slot = getattr(data, "t", None), getattr(data, "t_slot", None)
            if t is None and t_slot is None:
                raise ValueError("pos with 2 columns needs data.t or data.t_slot")
            if t_slot is not None:
                L.require_device(t_slot)
                t_slot = L.f32c(t_slot)
            sc = L.GnnScales(sc.inv_lx, sc.inv_ly, sc.inv_tmax, sc.tw, 1, float(t or 0.0),
                             L.ptr(t_slot) if t_slot is not None else None)
        elif pos.shape[-1] != 3:
            raise ValueError("pos must be [n, 3] (t, x, y) or [n, 2] (x, y)")
        if workspace is None:
            workspace = torch.empty((L.lib().mmpde_gnn_workspace_bytes(n) // 4,),
                                    dtype=torch.float32, device=u.device)
        if out is None:
            out = torch.empty((n, self.time_window), dtype=torch.float32, device=u.device)
        if trace is None:
            trace = L.GnnExec(None, None, 0, None)
        trace.edge_gemm = L.EDGE_GEMM[self.edge_gemm]
        trace.degree = L.ptr(deg)
        # nodes per trajectory: the f16x3 split scale is then taken per trajectory
        # (a trajectory's output does not depend on the others in the batch)
        seg = getattr(data, "seg_n", None)
        trace.seg_n = int(seg) if seg else 0
        trace.packed = (L.ptr(self.packed_f16x3(u.device)) if self.edge_gemm == "f16x3"
                        else None)
        call = SimpleNamespace(u=L.ptr(u), pos=L.ptr(pos), n=n, k=nbr.shape[1], nbr=L.ptr(nbr), sc=sc,
                               emb=ctypes.addressof(emb), layers=ctypes.addressof(arr), n_layers=len(arr),
                               head=ctypes.addressof(head), workspace=L.ptr(workspace), out=L.ptr(out),
                               exec=ctypes.addressof(trace))
        return call, out, (u, pos, nbr, deg, t_slot, workspace, out, trace, emb, arr, head)


    # ----------------------------------------------------------------- training
    def train_forward(self, data):
        """gnn_2d.py:119-141 in train() mode, differentiable (see module doc)."""
        if self.hidden_features != 128:
            raise NotImplementedError("HIP edge kernels take hidden_features = 128")
        u, pos = data.x, data.pos
        L.require_device(u, pos)
        n = u.shape[0]
        graph = EdgeGraph.of(data, n)
        pos_x = pos[:, 1][:, None] / self.pde.Lx
        pos_y = pos[:, 2][:, None] / self.pde.Ly
        variables = pos[:, 0][:, None] / self.pde.tmax
        e = self.embedding_mlp
        node_input = torch.cat((u, pos_x, pos_y, variables), -1)
        z = torch.relu(batch_norm_rows(e[1], linear_train(node_input, e[0])))
        if RELU_RECORD is not None:
            RELU_RECORD.append(("emb", (z > 0).detach()))
        h = batch_norm_rows(e[4], linear_train(z, e[3]))
        for layer in self.gnn_layers:
            if layer.fused_train_ok() and self.time_window == 1 and h.shape[0] >= 2:
                # (u, x, y, t) is the embedding input itself (tw = 1)
                h = layer.train_forward_fused(h, node_input, graph, self.edge_gemm)
            else:
                h = layer.train_forward(h, u, pos_x, pos_y, variables, graph, self.edge_gemm)
        diff = self._head_train(h)
        return self.out_scales_on(h.device)[None] * diff

    def out_scales_on(self, device) -> torch.Tensor:
        """out_scales() on `device`, cached per (device, dt, tw): a pageable
        host->device copy per forward would wait for the stream to drain."""
        key = (str(device), float(self.pde.dt), self.time_window)
        cache = self.__dict__.setdefault("_out_scales_cache", {})
        hit = cache.get(key)
        if hit is None:
            hit = self.out_scales().to(device)
            cache.clear()
            cache[key] = hit
        return hit

    def _head_train(self, h: torch.Tensor) -> torch.Tensor:
        """output_mlp(h[:, None]).squeeze(1) (gnn_2d.py:108-114,136), as the
        same three strided Conv1d written as unfold + GEMM (per node: 128 -> 38
        x 4 -> 9 x 8 -> 1): LinearRows over the window rows (weight and bias
        gradients on mmpde_rows_grad_weight) and unfold's gather-form
        backward instead of MIOpen's convolution search and kernels (which
        cost ~1 ms per training iteration and a multi-second search on first
        use)."""
        o = self.output_mlp
        if head_train_fits(o, h):
            # the whole head, forward and backward, in two HIP launches
            c0, c2, c4 = o[0], o[2], o[4]
            return HeadTrain.apply(h, c0.weight, c0.bias, c2.weight, c2.bias, c4.weight, c4.bias)
        n = h.shape[0]
        x = h
        y = None
        for i, idx in enumerate((0, 2, 4)):
            c = o[idx]
            cout, cin, ks = c.weight.shape
            st = c.stride[0]
            if i == 0:
                win = x.unfold(1, ks, st)                               # [n, L, ks]   (cin = 1)
            else:
                win = y.transpose(1, 2).unfold(2, ks, st)               # [n, cin, L, ks]
                win = win.permute(0, 2, 1, 3).reshape(n, win.shape[2], cin * ks)
            L_ = win.shape[1]
            y = LinearRows.apply(win.reshape(n * L_, cin * ks), c.weight.reshape(cout, cin * ks),
                                 c.bias).reshape(n, L_, cout)           # [n, L, cout]
            if idx != 4:
                y = torch.relu(y)
        return y.transpose(1, 2).squeeze(1)                             # [n, L_last]
