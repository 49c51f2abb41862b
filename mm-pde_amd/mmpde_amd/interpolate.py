"""ItpNet on the HIP kernels (drop-in for reference interpolate.py:5-99).

Parameters and state_dict keys match the reference: ``layers`` (mode '1'),
``layers2`` (mode '2'), the never-used ``layers3`` (kept for key parity) and the
``down`` residual-cut network (Linear MLP for the cylinder mesh, Conv2d stack
for Burgers).  Modes '1'/'2' run inside the fused kNN-30 + MLP + weighted-sum
kernel driven by GraphCreator_FS_2D.interpolate; ``forward(..., 'res_cut')``
runs the ``down`` network on the skinny-GEMM / conv kernels.

In ``train()`` mode (mmpde.py:86, the ItpNet parameters are in the AdamW groups
of mmpde.py:269-271) the forward follows interpolate.py:77-99 with device torch
ops under autograd: the gradients reach ``layers``, ``layers2`` and ``down``
through create_graph's mode-'1' interpolation and interpolate_pred's mode '2' +
res_cut (train_helper_2d.py:108,116).  ``forward(neighbors, query, '1'|'2')``
is that module-level MLP in either mode.
"""
from __future__ import annotations

import ctypes

import torch
from torch import nn

from . import _lib as L
from . import ops


def _mlp(widths):
    return nn.ModuleList(nn.Linear(a, b) for a, b in zip(widths[:-1], widths[1:]))


class ResCutMlp(torch.autograd.Function):
    """The cylinder ``down`` MLP (interpolate.py:58-60: Linear, Tanh x 3, Linear)
    in train mode at M = B rows: forward on mmpde_linear_skinny (tanh fused),
    backward per layer dW = dZ^T X, db = sum dZ (mmpde_outer_rows), dX = dZ W as
    the skinny forward of W^T (mmpde_transpose), times tanh' of the layer input
    (mmpde_tanh_bwd).  Exact fp32 products in fixed orders: deterministic."""

    @staticmethod
    def forward(ctx, x, *params):
        ws, bs = params[0::2], params[1::2]
        acts = (L.ACT_TANH, L.ACT_TANH, L.ACT_TANH, L.ACT_NONE)
        ins = [L.f32c(x)]
        for w, b, act in zip(ws, bs, acts):
            ins.append(ops.linear_skinny(ins[-1], w, b, act))
        y = ins.pop()
        ctx.save_for_backward(*ins, *[L.f32c(w) for w in ws])
        return y

    @staticmethod
    def backward(ctx, dy):
        saved = ctx.saved_tensors
        ins, ws = saved[:4], saved[4:]
        lib = L.lib()
        dev = dy.device
        st = L.stream(dev)
        grads = [None] * 8
        g = L.f32c(dy)
        m = g.shape[0]
        for layer in (3, 2, 1, 0):
            w, xin = ws[layer], ins[layer]
            n, k = w.shape
            need_w, need_b = ctx.needs_input_grad[1 + 2 * layer], ctx.needs_input_grad[2 + 2 * layer]
            if need_w or need_b:
                dw = torch.empty((n, k), dtype=torch.float32, device=dev)
                db = torch.empty((n,), dtype=torch.float32, device=dev) if need_b else None
                L.check(lib.mmpde_outer_rows(L.ptr(g), n, L.ptr(xin), k, m, n, k, L.ptr(dw), k, L.ptr(db), st),
                        "mmpde_outer_rows")
                grads[2 * layer] = dw if need_w else None
                grads[2 * layer + 1] = db
            if layer == 0 and not ctx.needs_input_grad[0]:
                g = None
                break
            wt = torch.empty((k, n), dtype=torch.float32, device=dev)
            L.check(lib.mmpde_transpose(L.ptr(w), n, k, k, L.ptr(wt), n, st), "mmpde_transpose")
            dx = ops.linear_skinny(g, wt)
            if layer > 0:   # the layer's input is the previous layer's tanh output
                L.check(lib.mmpde_tanh_bwd(L.ptr(dx), L.ptr(xin), dx.numel(), L.ptr(dx), st), "mmpde_tanh_bwd")
            g = dx
        return (g, *grads)


class ItpNet(nn.Module):
    def __init__(self, ori_nx, ori_ny, layers1, layers2, layers3, normalize=False):
        super().__init__()
        if normalize:
            raise NotImplementedError("ItpNet(normalize=True) is not used by MM-PDE")
        self.n = 30
        self.layers1_node = [self.n * 2 + 2] + list(layers1) + [self.n]
        self.n_layers1 = len(self.layers1_node) - 1
        assert self.n_layers1 >= 1
        self.layers = _mlp(self.layers1_node)
        self.layers2_node = [self.n * 2 + 2] + list(layers2) + [self.n]
        self.n_layers2 = len(self.layers2_node) - 1
        self.layers2 = _mlp(self.layers2_node)
        npts = ori_nx * ori_ny if ori_ny is not None else ori_nx
        self.layers3_node = [npts] + list(layers3) + [npts]
        self.n_layers3 = len(self.layers3_node) - 1
        self.layers3 = _mlp(self.layers3_node)   # built but never used (interpolate.py:48-60)
        self.conv = ori_ny is not None
        if self.conv:
            c = layers3
            self.down = nn.Sequential(
                nn.Conv2d(c[0], c[1], 5, padding=2), nn.Tanh(),
                nn.Conv2d(c[1], c[2], 5, padding=2), nn.Tanh(),
                nn.Conv2d(c[2], c[3], 5, padding=2), nn.Tanh(),
                nn.Conv2d(c[3], c[4], 5, padding=2), nn.Tanh())
        else:
            self.down = nn.Sequential(
                nn.Linear(ori_nx, 2048), nn.Tanh(), nn.Linear(2048, 512), nn.Tanh(),
                nn.Linear(512, 2048), nn.Tanh(), nn.Linear(2048, ori_nx))
        self._packs = {}

    # ----------------------------------------------------------------- packing
    def packed(self, mode: str) -> torch.Tensor:
        """Weights of mode '1' / '2' re-laid as the MFMA operand image of
        mmpde_itp_interp (cached until a parameter changes)."""
        mods = self.layers if mode == "1" else self.layers2
        if [m.out_features for m in mods] != [128, 64, 30] or mods[0].in_features != 62:
            raise NotImplementedError("fused ItpNet kernel needs layers [62, 128, 64, 30] "
                                      "(the reference defaults --itpnet_node1/2 = 128,64)")
        ts = [t for m in mods for t in (m.weight, m.bias)]
        key = tuple((t.data_ptr(), t._version) for t in ts)
        hit = self._packs.get(mode)
        if hit is not None and hit[0] == key:
            return hit[1]
        L.require_device(*ts)
        f = [L.f32c(t) for t in ts]
        mlp = L.ItpMlp(*[t.data_ptr() for t in f])
        buf = torch.empty((L.lib().mmpde_itp_pack_bytes() // 4,), dtype=torch.float32,
                          device=f[0].device)
        L.check(L.lib().mmpde_itp_pack(ctypes.byref(mlp), L.ptr(buf), L.stream(buf.device)),
                "mmpde_itp_pack")
        self._packs[mode] = (key, buf, f)
        return buf

    def weights(self, neighbors: torch.Tensor, query_points: torch.Tensor, mode: str):
        """interpolate.py:79-93: the 30 weights of every query from its neighbours'
        coordinates [..., 30, 2] and its own [..., 1, 2] (tanh MLP, linear last)."""
        L.require_device(neighbors, query_points)
        mods = self.layers if mode == "1" else self.layers2
        x = torch.cat((neighbors, query_points), dim=-2).reshape(
            neighbors.shape[0], neighbors.shape[1], -1)
        lead = x.shape[:-1]
        x = x.reshape(-1, x.shape[-1])
        for i, lin in enumerate(mods):
            # rows of every trajectory's queries: the row-chunked weight
            # gradient of ops.LinearRows (the library's K = rows GEMM is slow)
            if not (x.requires_grad or lin.weight.requires_grad):
                x = lin(x)
            elif x.shape[-1] % 8:
                # the 62-wide input zero-padded to a multiple of 8 (x and W alike:
                # the extra products are exact zeros), so that the row GEMM's
                # MFMA form takes it (interpolate.py:84's 2 * 30 + 2 features)
                padk = -x.shape[-1] % 8
                x = ops.LinearRows.apply(torch.nn.functional.pad(x, (0, padk)).contiguous(),
                                         torch.nn.functional.pad(lin.weight, (0, padk)), lin.bias)
            else:
                x = ops.linear_train(x, lin)
            if i != len(mods) - 1:
                x = torch.tanh(x)
        return x.reshape(*lead, x.shape[-1])

    def res_cut(self, data: torch.Tensor) -> torch.Tensor:
        """``down`` network (interpolate.py:95-97): data [B, N] (cylinder) or
        [B, 1, s, s] (Burgers)."""
        L.require_device(data)
        d = self.down
        if self.training:
            # differentiable, on the HIP kernels (no library GEMM / MIOpen)
            if self.conv:
                x = data
                for i in (0, 2, 4, 6):
                    x = torch.tanh(ops.Conv2dSame.apply(x, d[i].weight, d[i].bias, False))
                return x
            params = [t for i in (0, 2, 4, 6) for t in (d[i].weight, d[i].bias)]
            return ResCutMlp.apply(data.reshape(data.shape[0], -1), *params)
        if self.conv:
            x = data
            for i in (0, 2, 4, 6):
                x = ops.conv2d(x, d[i].weight, d[i].bias, 1, 2, L.ACT_TANH)
            return x
        x = data.reshape(data.shape[0], -1)
        layers = [(d[i].weight, d[i].bias, act)
                  for i, act in ((0, L.ACT_TANH), (2, L.ACT_TANH), (4, L.ACT_TANH), (6, L.ACT_NONE))]
        for w, b, act in layers:
            x = ops.linear_skinny(x, w, b, act)
        return x

    def forward(self, neighbors, query_points, mode, data=None):
        """interpolate.py:77-99.  Modes '1'/'2' return the [..., 30] weights;
        the rollout path never calls this (GraphCreator_FS_2D.interpolate fuses
        the kNN-30 search, these weights and the weighted sum in one kernel)."""
        if mode == "res_cut":
            return self.res_cut(data)
        if mode in ("1", "2"):
            return self.weights(neighbors, query_points, mode)
        return data   # interpolate.py:77-99 returns `data` unchanged for other modes
