"""Train-mode Linears on the HIP row GEMMs (mmpde_rgemm / mmpde_rgemm_tn,
csrc/rgemm.hip): the forward and input gradient of every node-level Linear of
the GNN (gnn_2d.py:53-69,99-106) and of ItpNet's MLPs (interpolate.py:79-93),
and their weight / bias gradients over the row axis, instead of the library
GEMMs (and the cat / ReLU / residual elementwise kernels) torch autograd runs
under loss.backward() (train_helper_2d.py:126).

* ``linear_fwd`` / ``linear_bwd_input`` / ``linear_bwd_weight``: y = x W^T + b
  and its gradients for ops.LinearRows (any row count, K and N).
* ``GnnLayerTrain``: one whole train-mode GNN_Layer_FS_2D (message_net_1 as
  target / source halves, message_net_2 + mean on the EdgeMean kernels,
  update_net_1 / _2, the residual and BatchNorm1d) as one autograd Function
  whose backward accumulates dL/dh in place (no elementwise adds).

Exact fp32 products, fixed summation orders: deterministic.
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _lib as L

_F4 = 4  # bytes per float
# rows per weight-gradient partial (fixed: deterministic sums); MMPDE_TN_CHUNK
# (an even row count) overrides it for A/B runs (tools/rgemm_bench.py)
CHUNK_ROWS = int(os.environ.get("MMPDE_TN_CHUNK", "256"))


def _p(t: torch.Tensor | None, col: int = 0) -> int | None:
    """Device pointer of column `col` of a row-major fp32 tensor."""
    return None if t is None else t.data_ptr() + _F4 * col


def rgemm(m: int, kh: int, layout: int, w, ldw: int, a, lda, parts, amask=(None, None),
          relu: bool = False, xs=None, ldxs: int = 0, ldxw: int = 0, stream=None):
    """One mmpde_rgemm launch.  w, a, amask: two (pointer) halves; parts: list
    of dicts with out (ptr), ldo, wc, wk, ncols and optional bias (ptr), omask
    (ptr), ldom, acc, ns, xw (ptr), xscale."""
    g = L.RgemmArgs()
    g.m, g.kh, g.layout, g.ldw = m, kh, layout, ldw
    g.w[0], g.w[1] = w
    g.a[0], g.a[1] = a
    g.amask[0], g.amask[1] = amask
    g.lda[0], g.lda[1] = lda
    g.parts = len(parts)
    for i, q in enumerate(parts):
        g.out[i], g.ldo[i], g.wc[i], g.wk[i], g.ncols[i] = q["out"], q["ldo"], q.get("wc", 0), q.get("wk", 0), \
            q["ncols"]
        g.bias[i] = q.get("bias")
        g.omask[i], g.ldom[i] = q.get("omask"), q.get("ldom", 0)
        g.accumulate[i] = int(q.get("acc", False))
        g.ns[i], g.xw[i], g.xscale[i] = q.get("ns", 0), q.get("xw"), q.get("xscale", 1.0)
    g.relu = int(relu)
    g.xs, g.ldxs, g.ldxw = xs, ldxs, ldxw
    L.check(L.lib().mmpde_rgemm(ctypes.byref(g), stream), "mmpde_rgemm")


def rgemm_tn(m: int, g_ptr: int, ldg: int, gcols: int, segs, dw: torch.Tensor, lddw: int,
             db: torch.Tensor | None = None, gmask=None, xs=None, ldxs: int = 0, ns: int = 0,
             dwcol_s: int = 0, sign_s: float = 1.0, accumulate_s: bool = False, stream=None,
             device=None):
    """dW[c][dwcol + j] = sum_rows G[:, c] x[:, j] per segment (x ptr, ldx, kx,
    dwcol), the small segment xs (ns columns) to dwcol_s (+ sign_s, accumulated
    or stored), db = sum_rows G (mmpde_rgemm_tn)."""
    a = L.RgemmTnArgs()
    a.m, a.chunk_rows, a.gcols, a.g, a.gmask, a.ldg = m, CHUNK_ROWS, gcols, g_ptr, gmask, ldg
    a.nseg = len(segs)
    cols = 0
    for i, (x, ldx, kx, dwcol) in enumerate(segs):
        a.x[i], a.ldx[i], a.kx[i], a.dwcol[i] = x, ldx, kx, dwcol
        cols += (kx + 63) // 64 * 64
    cols += ns + 1
    a.xs, a.ldxs, a.ns, a.dwcol_s, a.sign_s, a.accumulate_s = xs, ldxs, ns, dwcol_s, sign_s, int(accumulate_s)
    a.dw, a.lddw, a.db = dw.data_ptr(), lddw, _p(db)
    nb = L.lib().mmpde_rgemm_tn_workspace_bytes(m, CHUNK_ROWS, cols)
    ws = torch.empty((nb // 4,), dtype=torch.float32, device=device or dw.device)
    L.check(L.lib().mmpde_rgemm_tn(ctypes.byref(a), L.ptr(ws), nb, stream), "mmpde_rgemm_tn")


def _halves(x: torch.Tensor, w: torch.Tensor, k: int):
    """(kh, (a0, a1), (w0, w1), small) for y = x W^T with K = k: two halves of kh
    columns; the remaining (k - 2 kh <= 4) columns go to the small segment."""
    if k <= 4:
        return 0, (None, None), (None, None), k
    kh = k // 2
    if kh % 4 and k >= 16:
        kh -= kh % 4
    rest = k - 2 * kh
    if rest > 4:              # not reachable for k >= 16 (rest < 8 with kh % 4 == 0) except odd k
        kh, rest = k // 2, k % 2
    return kh, (_p(x), _p(x, kh)), (_p(w), _p(w, kh)), rest


def _mfma_width(k: int) -> bool:
    """K the MFMA row GEMM takes at full rate: two 16-byte-aligned halves of
    32, 64 or 128 columns (the weight-stationary form), or wider multiples of 8."""
    return k % 8 == 0 and (k // 2 in (32, 64, 128) or k > 256)


def _skinny(k: int, nout: int) -> bool:
    """Maps mmpde_rows_small takes instead (a 32 x 32 MFMA tile would run mostly
    empty, or K splits into no aligned halves): the Conv1d head's windows, the
    embedding's first Linear, ItpNet's 62- and 30-wide layers."""
    return k <= 128 and nout <= 128 and (min(k, nout) <= 16 or not _mfma_width(k))


def rows_small(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None, layout: int) -> torch.Tensor:
    """mmpde_rows_small: NT y = x W^T + b; NN y = x W (W [N, K] either way)."""
    n = x.shape[0]
    nout, k = w.shape
    width = nout if layout == L.RGEMM_NT else k
    y = torch.empty((n, width), dtype=torch.float32, device=x.device)
    L.check(L.lib().mmpde_rows_small(_p(x), x.stride(0), n, k, _p(w), w.stride(0), layout, _p(b), nout,
                                     _p(y), width, L.stream(x.device)), "mmpde_rows_small")
    return y


def linear_fwd(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None) -> torch.Tensor:
    """y = x W^T + b (x [n, K] fp32 contiguous, W [N, K] contiguous)."""
    n, k = x.shape
    nout = w.shape[0]
    if _skinny(k, nout):
        return rows_small(x, w, b, L.RGEMM_NT)
    y = torch.empty((n, nout), dtype=torch.float32, device=x.device)
    st = L.stream(x.device)
    kh, a, wh, rest = _halves(x, w, k)
    for c0 in range(0, nout, 256):
        parts = [dict(out=_p(y, c), ldo=nout, wc=c, ncols=min(128, nout - c), bias=_p(b, c), ns=rest,
                      xw=_p(w, c * k + 2 * kh) if rest else None)
                 for c in range(c0, min(nout, c0 + 256), 128)]
        rgemm(n, kh, L.RGEMM_NT, wh, k, a, (k, k), parts, xs=_p(x, 2 * kh) if rest else None,
              ldxs=k, ldxw=k, stream=st)
    return y


def linear_bwd_input(dy: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """dX = dY W (dY [n, N] fp32 contiguous, W [N, K]): halves over the N
    outputs, the last N - 2 kh of them in the small segment."""
    n, nout = dy.shape
    k = w.shape[1]
    if k <= 128 and nout <= 128 and (min(k, nout) <= 16 or not _mfma_width(nout)):   # GEMM K = nout
        return rows_small(dy, w, None, L.RGEMM_NN)
    gx = torch.empty((n, k), dtype=torch.float32, device=dy.device)
    st = L.stream(dy.device)
    kh, _, _, rest = _halves(dy, w, nout)
    for j0 in range(0, k, 256):
        parts = [dict(out=_p(gx, j), ldo=k, wc=j, wk=0, ncols=min(128, k - j), ns=rest,
                      xw=_p(w, 2 * kh * k + j) if rest else None)
                 for j in range(j0, min(k, j0 + 256), 128)]
        rgemm(n, kh, L.RGEMM_NN, (_p(w), _p(w, kh * k)), k, (_p(dy), _p(dy, kh)), (nout, nout),
              parts, xs=_p(dy, 2 * kh) if rest else None, ldxs=nout, ldxw=k, stream=st)
    return gx


def linear_bwd_weight(dy: torch.Tensor, x: torch.Tensor, dw: torch.Tensor | None, db: torch.Tensor | None):
    """dW = dY^T X into dw [N, K] (nullable), db = sum_rows dY into db [N]
    (nullable), 128 outputs per mmpde_rgemm_tn call."""
    n, nout = dy.shape
    k = x.shape[1]
    st = L.stream(dy.device)
    dwt = dw if dw is not None else torch.empty((nout, k), dtype=torch.float32, device=dy.device)
    for c in range(0, nout, 128):
        rgemm_tn(n, _p(dy, c), nout, min(128, nout - c), [(_p(x), k, k, 0)], dwt[c:], k,
                 db=db[c:] if db is not None else None, stream=st)
