"""Tensor-level wrappers over the C-ABI (one function per entry point).

Every function launches on the current torch stream of the input's device and
returns new device tensors; nothing here synchronises or falls back to CPU.
"""
from __future__ import annotations

import ctypes

import os

import torch

from . import _lib as L
from . import rows

# kNN kernels stage one trajectory's points in LDS and keep its distances in
# registers (csrc/knn.hip): at most this many points per trajectory
# (include/mmpde_hip.h mmpde_knn_graph / mmpde_knn_query).  The reference's
# benchmarked grids are 2521 (cy) and 48 x 48 = 2304 (burgers); burgers at the
# PDE's own default 96 x 96 (PDEs.py:27) exceeds it.
KNN_MAX_POINTS = 16384


def _knn_points_check(n_per: int, k: int, what: str):
    if n_per > KNN_MAX_POINTS:
        raise ValueError(f"{what}: {n_per} points per trajectory; the HIP kNN kernels take at "
                         f"most {KNN_MAX_POINTS} (run --base_resolution <= 128 x 128)")
    if k > 63:
        raise ValueError(f"{what}: k = {k}; the HIP kNN kernels take k <= 63")


def knn_graph_nbr(pos: torch.Tensor, batches: int, k: int, count_degenerate: bool = False):
    """torch_cluster.knn_graph(pos, k, batch, loop=False) for `batches` equal
    contiguous segments (reference data_creator_2d.py:260, dmm_model.py:228).
    Returns nbr [n, k] int32 (global source indices, (d2, index) order)
    [, degenerate count tensor]."""
    L.require_device(pos)
    pos = L.f32c(pos).reshape(-1, 2)
    n = pos.shape[0]
    if n % batches:
        raise ValueError("pos rows must split into equal batch segments")
    _knn_points_check(n // batches, k, "knn_graph")
    nbr = torch.empty((n, k), dtype=torch.int32, device=pos.device)
    deg = torch.zeros((1,), dtype=torch.int32, device=pos.device) if count_degenerate else None
    L.check(L.lib().mmpde_knn_graph(L.ptr(pos), batches, n // batches, k, L.ptr(nbr),
                                    L.ptr(deg), L.stream(pos.device)), "mmpde_knn_graph")
    return (nbr, deg) if count_degenerate else nbr


KNN_CAND = 128  # candidates per point in mmpde_knn_candidates' table


def knn_candidates(xi: torch.Tensor, ref: torch.Tensor | None = None):
    """Static candidate table of knn_graph_moved / knn_query_moved for fixed
    points xi [N, 2] and reference points ref [N, 2] (default xi; for a query,
    the fixed query points): [N, 128] int32, the 128 nearest of ref_p in xi in
    (d2, index) order, or None where the candidate path does not apply (N
    outside [128, 4096])."""
    L.require_device(xi, ref)
    xi = L.f32c(xi).reshape(-1, 2)
    N = xi.shape[0]
    if N < KNN_CAND or N > 4096:
        return None
    if ref is not None:
        ref = L.f32c(ref).reshape(-1, 2)
        if ref.shape[0] != N:
            raise ValueError("ref must hold one reference point per xi point")
    cand = torch.empty((N, KNN_CAND), dtype=torch.int32, device=xi.device)
    L.check(L.lib().mmpde_knn_candidates(L.ptr(xi), L.ptr(ref), N, L.ptr(cand), L.stream(xi.device)),
            "mmpde_knn_candidates")
    return cand


def knn_skip_threshold(xi: torch.Tensor, cand, kk: int, ref: torch.Tensor | None = None,
                       moved_queries: bool = False) -> float:
    """The skip_above of knn_graph_moved / knn_query_moved for a table cand =
    knn_candidates(xi, ref) and kk = k + 1 (graph) or k (query): the median of
    R128 - R_kk over the reference points, halved for queries that move with
    the mesh (the graph) (mmpde_knn_skip_threshold).  Reads one float back to
    the host: call once per table, not per step."""
    if cand is None:
        return 0.0
    L.require_device(xi, cand, ref)
    xi = L.f32c(xi).reshape(-1, 2)
    ref = None if ref is None else L.f32c(ref).reshape(-1, 2)
    out = torch.empty((1,), dtype=torch.float32, device=xi.device)
    L.check(L.lib().mmpde_knn_skip_threshold(L.ptr(xi), L.ptr(ref), xi.shape[0], L.ptr(cand), kk,
                                             int(moved_queries), L.ptr(out), L.stream(xi.device)),
            "mmpde_knn_skip_threshold")
    return float(out.item())


def knn_moved_cells(pos: torch.Tensor, xi: torch.Tensor, batches: int,
                    out: torch.Tensor | None = None) -> torch.Tensor:
    """Per-trajectory displacement record of moved points pos [batches * N, 2]
    (every trajectory moved from xi [N, 2]): the largest |pos_j - xi_j| per cell
    of a 16 x 16 grid over xi's box (mmpde_knn_moved_cells).  One per moved mesh,
    shared by knn_graph_moved and knn_query_moved."""
    L.require_device(pos, xi)
    pos = L.f32c(pos).reshape(-1, 2)
    xi = L.f32c(xi).reshape(-1, 2)
    N = xi.shape[0]
    if pos.shape[0] != batches * N:
        raise ValueError("pos must hold `batches` meshes of xi's size")
    nf = L.lib().mmpde_knn_moved_cells_bytes(batches) // 4
    if out is None or out.numel() < nf:
        out = torch.empty((nf,), dtype=torch.float32, device=pos.device)
    L.check(L.lib().mmpde_knn_moved_cells(L.ptr(pos), L.ptr(xi), batches, N, L.ptr(out),
                                          L.stream(pos.device)), "mmpde_knn_moved_cells")
    return out


def knn_table_share(cells: torch.Tensor, batches: int, n_per: int) -> torch.Tensor:
    """[batches, 2] float: per trajectory, the share of the graph (column 0) and
    query (column 1) lookups the candidate tables answered since `cells` was
    computed (knn_moved_cells), from the record's miss counters (diagnostics)."""
    L.require_device(cells)
    miss = torch.empty((batches, 2), dtype=torch.int32, device=cells.device)
    L.check(L.lib().mmpde_knn_table_misses(L.ptr(cells), batches, L.ptr(miss),
                                           L.stream(cells.device)), "mmpde_knn_table_misses")
    return 1.0 - miss.float() / n_per


def _capturing() -> bool:
    """A hipGraph capture is in progress on the current stream."""
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


class KnnTablePolicy:
    """Per-role choice between the candidate table (knn_graph_moved /
    knn_query_moved) and the plain full search for a rollout, from a cost model
    and the share f of lookups the table answered at an earlier step.

    Cost model (tools/knn_cand_time.py, cy B=16 on MI355X): the table path costs
    about T_cand + (1 - f) T_full -- the candidate kernel (37-44 us when every
    lookup passes) plus the full search of the lookups it could not answer --
    against T_full (61-80 us) for the full search, so it pays only while f >
    T_cand / T_full ~ 0.6; MIN_SHARE = 0.7 leaves room for the sorts the failed
    lookups also pay.  f is read back without a sync: the per-trajectory miss
    counters are copied to pinned host memory behind an event after a table
    call and consumed at a later step.  A role starts on the table (checked
    every CHECK_EVERY calls); below MIN_SHARE it runs the full search -- no
    candidate or cell kernels -- and after PROBE_EVERY calls makes ONE table
    call (a probe), staying on the full search until the probe's share is
    known.  Either path gives the same indices bit for bit."""

    MIN_SHARE = 0.7
    PROBE_EVERY = 64
    CHECK_EVERY = 4

    def __init__(self, device, batches: int, n_per: int, roles):
        self.device = torch.device(device)
        self.B, self.N = batches, n_per
        self.state = {r: {"mode": "table", "wait": 0, "since": 0, "pending": None, "share": None}
                      for r in roles}
        self.enabled = True

    def _resolve(self, st):
        pend = st["pending"]
        if pend is None or not pend[0].query():
            return
        st["pending"] = None
        share = 1.0 - float(pend[1].sum()) / (self.B * self.N)
        st["share"] = share
        if share >= self.MIN_SHARE:
            if st["mode"] != "table":
                st["mode"], st["since"] = "table", 0
        else:
            st["mode"], st["wait"] = "full", self.PROBE_EVERY

    def use_table(self, role) -> bool:
        if not self.enabled:
            return True
        st = self.state[role]
        self._resolve(st)
        if st["mode"] == "full":
            st["wait"] -= 1
            # no probe inside a hipGraph capture: its read-back cannot be queued
            # there (after_table), so the probe would never resolve
            if st["wait"] < 0 and not _capturing():
                st["mode"], st["since"] = "probe", 0
                return True                          # the probe call
            return False
        if st["mode"] == "probe":                    # probe made, its share not known yet
            return False
        return True

    def mode(self, role) -> str:
        return self.state[role]["mode"]

    def after_table(self, role, cells: torch.Tensor, column: int) -> None:
        """Queue the read-back of the miss counters of the table call just made
        with `cells` (on the current stream, after that call): at a probe and
        every CHECK_EVERY table calls."""
        st = self.state[role]
        st["since"] += 1
        if st["pending"] is not None or (st["mode"] == "table" and (st["since"] - 1) % self.CHECK_EVERY):
            return
        if _capturing():
            if st["mode"] == "probe":                # cannot read back: retry after capture
                st["mode"], st["wait"] = "full", self.PROBE_EVERY
            return
        miss = torch.empty((self.B, 2), dtype=torch.int32, device=self.device)
        L.check(L.lib().mmpde_knn_table_misses(L.ptr(cells), self.B, L.ptr(miss), L.stream(self.device)),
                "mmpde_knn_table_misses")
        host = torch.empty((self.B,), dtype=torch.int32, pin_memory=True)
        host.copy_(miss[:, column], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        st["pending"] = (ev, host)


def _cand_scratch(scratch, batches, N, device):
    need = L.lib().mmpde_knn_graph_cand_scratch_bytes(batches, N)
    if scratch is None or scratch.numel() * scratch.element_size() < need:
        scratch = torch.empty((max(need, 1),), dtype=torch.uint8, device=device)
    return scratch


def knn_graph_moved(pos: torch.Tensor, xi: torch.Tensor, cand, batches: int, k: int,
                    scratch: torch.Tensor | None = None, count_degenerate: bool = False,
                    cells: torch.Tensor | None = None, skip_above: float = 0.0):
    """knn_graph_nbr of moved points pos [batches * N, 2] (every trajectory's
    mesh moved from the same xi [N, 2]), bit for bit, answered from the
    candidate table `cand` (knn_candidates(xi)) where a distance bound proves
    it complete and by the full search elsewhere (reference
    data_creator_2d.py:260 on the DMM's moved mesh).  cells: knn_moved_cells(pos,
    xi, batches) if already computed; skip_above > 0: trajectories moved
    further go straight to the full search (knn_skip_threshold)."""
    if cand is None:
        return knn_graph_nbr(pos, batches, k, count_degenerate)
    L.require_device(pos)
    pos = L.f32c(pos).reshape(-1, 2)
    xi = L.f32c(xi).reshape(-1, 2)
    n = pos.shape[0]
    N = xi.shape[0]
    if n != batches * N or cand.shape != (N, KNN_CAND):
        raise ValueError("pos must hold `batches` meshes of xi's size; cand from knn_candidates(xi)")
    _knn_points_check(N, k, "knn_graph")
    if cells is None:
        cells = knn_moved_cells(pos, xi, batches)
    scratch = _cand_scratch(scratch, batches, N, pos.device)
    nbr = torch.empty((n, k), dtype=torch.int32, device=pos.device)
    deg = torch.zeros((1,), dtype=torch.int32, device=pos.device) if count_degenerate else None
    L.check(L.lib().mmpde_knn_graph_cand(L.ptr(pos), L.ptr(xi), L.ptr(cells), float(skip_above),
                                         batches, N, k,
                                         L.ptr(cand), L.ptr(nbr), L.ptr(deg), L.ptr(scratch),
                                         L.stream(pos.device)), "mmpde_knn_graph_cand")
    return (nbr, deg) if count_degenerate else nbr


def radius_graph_nbr(pos: torch.Tensor, batches: int, r: float, max_num_neighbors: int = 32):
    """torch_cluster.radius_graph(pos, r, batch, loop=False, max_num_neighbors) for
    `batches` equal contiguous segments (reference data_creator_2d.py:257-258),
    CUDA semantics (first max_num_neighbors + 1 in index order within r, self
    dropped).  Returns (nbr int32 [n, max_num_neighbors + 1] global sources,
    padded with -1; degree int32 [n])."""
    L.require_device(pos)
    pos = L.f32c(pos).reshape(-1, 2)
    n = pos.shape[0]
    if n % batches:
        raise ValueError("pos rows must split into equal batch segments")
    w = max_num_neighbors + 1
    nbr = torch.empty((n, w), dtype=torch.int32, device=pos.device)
    deg = torch.empty((n,), dtype=torch.int32, device=pos.device)
    L.check(L.lib().mmpde_radius_graph(L.ptr(pos), batches, n // batches, float(r),
                                       max_num_neighbors, L.ptr(nbr), L.ptr(deg),
                                       L.stream(pos.device)), "mmpde_radius_graph")
    return nbr, deg


def edge_index_from_nbr(nbr: torch.Tensor, degree: torch.Tensor | None = None) -> torch.Tensor:
    """PyG edge_index int64 [2, E] (row 0 source, row 1 target) of a target-major
    table; with `degree`, row i contributes its first degree[i] entries."""
    if degree is not None:
        n, k = nbr.shape
        keep = torch.arange(k, device=nbr.device)[None, :] < degree[:, None].long()
        tgt = torch.arange(n, device=nbr.device)[:, None].expand(n, k)
        return torch.stack((nbr.long()[keep], tgt[keep]))
    """PyG edge_index int64 [2, n*k] (row 0 source, row 1 target)."""
    L.require_device(nbr)
    n, k = nbr.shape
    ei = torch.empty((2, n * k), dtype=torch.int64, device=nbr.device)
    L.check(L.lib().mmpde_edge_index_from_nbr(L.ptr(nbr.contiguous()), n, k, L.ptr(ei),
                                              L.stream(nbr.device)), "mmpde_edge_index_from_nbr")
    return ei


def nbr_from_edge_index(edge_index: torch.Tensor, n: int) -> torch.Tensor:
    """Recover the fixed-degree target-major table from a PyG edge_index whose
    targets are grouped (the layout knn_graph produces).  Raises on ragged
    degree (use nbr_table_from_edge_index)."""
    e = edge_index.shape[1]
    if e % n:
        raise ValueError("edge_index has ragged in-degree; fixed-degree kernels need k*n edges")
    k = e // n
    tgt = torch.arange(n, device=edge_index.device).repeat_interleave(k)
    if not bool(torch.equal(edge_index[1], tgt)):
        raise ValueError("edge_index targets are not grouped as knn_graph emits them")
    return edge_index[0].reshape(n, k).to(torch.int32).contiguous()


def nbr_table_from_edge_index(edge_index: torch.Tensor, n: int):
    """Any PyG edge_index -> (nbr int32 [n, k], degree int32 [n] or None).  A
    grouped fixed-degree graph gives degree None; otherwise the in-edges of every
    target (stable order) fill its row, padded with -1, k = max in-degree."""
    e = edge_index.shape[1]
    if e % n == 0:
        k = e // n
        tgt = torch.arange(n, device=edge_index.device).repeat_interleave(k)
        if bool(torch.equal(edge_index[1], tgt)):
            src = edge_index[0]
            if e and (int(src.min()) < 0 or int(src.max()) >= n):
                raise ValueError("edge_index holds nodes outside [0, n)")
            return src.reshape(n, k).to(torch.int32).contiguous(), None
    src, tgt = edge_index[0].long(), edge_index[1].long()
    if e and (int(src.min()) < 0 or int(src.max()) >= n or int(tgt.min()) < 0 or int(tgt.max()) >= n):
        raise ValueError("edge_index holds nodes outside [0, n)")
    order = torch.argsort(tgt, stable=True)
    src, tgt = src[order], tgt[order]
    deg = torch.bincount(tgt, minlength=n)
    k = max(int(deg.max().item()) if e else 0, 1)
    start = torch.cumsum(deg, 0) - deg
    slot = torch.arange(e, device=edge_index.device) - start[tgt]
    nbr = torch.full((n, k), -1, dtype=torch.int32, device=edge_index.device)
    nbr[tgt, slot] = src.to(torch.int32)
    return nbr, deg.to(torch.int32)


def _ties(ties):
    if ties is not None and (ties.dtype != torch.int32 or ties.numel() < 1 or not ties.is_cuda):
        raise ValueError("ties must be an int32 device counter")
    return ties


def knn_query(src: torch.Tensor, qry: torch.Tensor, batches: int, k: int,
              ties: torch.Tensor | None = None) -> torch.Tensor:
    """Per-trajectory sklearn NearestNeighbors(k).fit(src_b).kneighbors(qry_b):
    LOCAL indices int32 [batches * n_qry, k], fp64-distance order
    (reference data_creator_2d.py:66-78).  ties: optional int32 [1] device
    counter, += the queries with an exact fp64 distance tie among their first
    k (or at rank k): where sklearn's order is its KD-tree's, parity unpinned."""
    L.require_device(src, qry)
    src = L.f32c(src).reshape(-1, 2)
    qry = L.f32c(qry).reshape(-1, 2)
    ns, nq = src.shape[0] // batches, qry.shape[0] // batches
    _knn_points_check(ns, k, "knn_query")
    idx = torch.empty((batches * nq, k), dtype=torch.int32, device=src.device)
    L.check(L.lib().mmpde_knn_query(L.ptr(src), L.ptr(qry), batches, ns, nq, k, L.ptr(idx),
                                    L.ptr(_ties(ties)), L.stream(src.device)), "mmpde_knn_query")
    return idx


def knn_query_moved(src: torch.Tensor, qry: torch.Tensor, xi: torch.Tensor, cand, batches: int,
                    k: int, scratch: torch.Tensor | None = None, ref: torch.Tensor | None = None,
                    cells: torch.Tensor | None = None, skip_above: float = 0.0,
                    ties: torch.Tensor | None = None) -> torch.Tensor:
    """knn_query of qry onto moved points src (every trajectory's mesh moved
    from the same xi [N, 2]; n_src = n_qry = N), bit for bit, answered from the
    candidate table `cand` = knn_candidates(xi, ref) (ref: the fixed points the
    queries sit at or near, default xi) where a distance bound proves it
    complete and by the full search elsewhere (reference data_creator_2d.py:66-78
    onto the DMM's moved mesh).  cells: knn_moved_cells(src, xi, batches) if
    already computed; skip_above as for knn_graph_moved; ties as for knn_query."""
    if cand is None:
        return knn_query(src, qry, batches, k, ties)
    L.require_device(src, qry, ref)
    src = L.f32c(src).reshape(-1, 2)
    qry = L.f32c(qry).reshape(-1, 2)
    xi = L.f32c(xi).reshape(-1, 2)
    N = xi.shape[0]
    if src.shape[0] != batches * N or qry.shape[0] != batches * N or cand.shape != (N, KNN_CAND):
        raise ValueError("src and qry must hold `batches` point sets of xi's size; "
                         "cand from knn_candidates(xi, ref)")
    if ref is not None:
        ref = L.f32c(ref).reshape(-1, 2)
        if ref.shape[0] != N:
            raise ValueError("ref must hold one reference point per xi point")
    _knn_points_check(N, k, "knn_query")
    if cells is None:
        cells = knn_moved_cells(src, xi, batches)
    scratch = _cand_scratch(scratch, batches, N, src.device)
    idx = torch.empty((batches * N, k), dtype=torch.int32, device=src.device)
    L.check(L.lib().mmpde_knn_query_cand(L.ptr(src), L.ptr(qry), L.ptr(xi), L.ptr(ref),
                                         L.ptr(cells), float(skip_above), batches, N, k,
                                         L.ptr(cand), L.ptr(idx), L.ptr(_ties(ties)),
                                         L.ptr(scratch), L.stream(src.device)),
            "mmpde_knn_query_cand")
    return idx


_SKINNY_WS = {}


def _skinny_workspace(device, nbytes: int) -> torch.Tensor:
    """Split-K scratch of mmpde_linear_skinny_ws: zeroed once, then reused (each
    call leaves its ticket counters at zero).  One per device and stream: calls
    on one stream are ordered, so they may share it."""
    key = (str(device), torch.cuda.current_stream(device).cuda_stream)
    ws = _SKINNY_WS.get(key)
    if ws is None or ws.numel() * 4 < nbytes:
        ws = torch.zeros((max(nbytes, 4) // 4 + 1024,), dtype=torch.float32, device=device)
        _SKINNY_WS[key] = ws
    return ws


def linear_skinny(x: torch.Tensor, w: torch.Tensor, b=None, act: int = L.ACT_NONE,
                  out: torch.Tensor | None = None) -> torch.Tensor:
    """act(x @ w.T + b) for a few rows (M = trajectories)."""
    L.require_device(x, w)
    x = L.f32c(x)
    w = L.f32c(w)
    m, k = x.shape
    n = w.shape[0]
    y = out if out is not None else torch.empty((m, n), dtype=torch.float32, device=x.device)
    lib = L.lib()
    wsb = lib.mmpde_linear_skinny_workspace_bytes(m, n, k)
    ws = _skinny_workspace(x.device, wsb)
    L.check(lib.mmpde_linear_skinny_ws(L.ptr(x), k, m, k, L.ptr(w), k,
                                       L.ptr(L.f32c(b)) if b is not None else None, n, act,
                                       L.ptr(y), n, L.ptr(ws), wsb, L.stream(x.device)),
            "mmpde_linear_skinny")
    return y


def linear_rows(x: torch.Tensor, w: torch.Tensor, b=None, act: int = L.ACT_NONE) -> torch.Tensor:
    """act(x @ w.T + b) for any number of rows (x [..., k]): linear_skinny on
    blocks of at most 4096 rows (the skinny kernel's row limit)."""
    lead = x.shape[:-1]
    x2 = L.f32c(x).reshape(-1, x.shape[-1])
    y = torch.empty((x2.shape[0], w.shape[0]), dtype=torch.float32, device=x2.device)
    for r0 in range(0, x2.shape[0], 4096):
        linear_skinny(x2[r0:r0 + 4096], w, b, act, out=y[r0:r0 + 4096])
    return y.reshape(*lead, w.shape[0])


def resample_bilinear(u: torch.Tensor, oh: int, ow: int) -> torch.Tensor:
    """F.interpolate(u[:, None], size=(oh, ow), mode='bilinear',
    align_corners=True)[:, 0] of u [..., h, w] (data_creator_2d.py:102-103)."""
    L.require_device(u)
    h, w = u.shape[-2:]
    x = L.f32c(u).reshape(-1, h, w)
    y = torch.empty((x.shape[0], oh, ow), dtype=torch.float32, device=x.device)
    L.check(L.lib().mmpde_resample_bilinear(L.ptr(x), x.shape[0], h, w, oh, ow, L.ptr(y),
                                            L.stream(x.device)), "mmpde_resample_bilinear")
    return y.reshape(*u.shape[:-2], oh, ow)


def conv2d(x: torch.Tensor, w: torch.Tensor, b, stride: int, pad: int, act: int,
           residual=None, circular: bool = False, res_after_act: bool = False) -> torch.Tensor:
    """act(conv2d(x, w, b, stride, pad) [+ residual]), NCHW fp32; circular:
    padding_mode='circular'; res_after_act: residual + act(conv2d(...))."""
    L.require_device(x, w)
    x = L.f32c(x)
    bt, cin, h, wd = x.shape
    cout, _, ks, _ = w.shape
    oh = (h + 2 * pad - ks) // stride + 1
    ow = (wd + 2 * pad - ks) // stride + 1
    y = torch.empty((bt, cout, oh, ow), dtype=torch.float32, device=x.device)
    res = L.f32c(residual) if residual is not None else None
    L.check(L.lib().mmpde_conv2d_ex(L.ptr(x), bt, cin, h, wd, L.ptr(L.f32c(w)),
                                    L.ptr(L.f32c(b)) if b is not None else None, cout, ks, stride,
                                    pad, L.PAD_CIRCULAR if circular else L.PAD_ZEROS, L.ptr(res),
                                    int(res_after_act), act, L.ptr(y), L.stream(x.device)),
            "mmpde_conv2d_ex")
    return y


def conv2d_grad_weight(x: torch.Tensor, dy: torch.Tensor, ks: int, pad: int, circular: bool,
                       bias: bool = True):
    """(dw [cout, cin, ks, ks], db [cout] or None) of a stride-1 conv2d with
    output size = input size (mmpde_conv2d_grad_weight; deterministic)."""
    L.require_device(x, dy)
    x, dy = L.f32c(x), L.f32c(dy)
    bt, cin, h, wd = x.shape
    cout = dy.shape[1]
    if dy.shape != (bt, cout, h, wd):
        raise ValueError("dy must be [batches, cout, h, w] of x's batches and plane")
    dw = torch.empty((cout, cin, ks, ks), dtype=torch.float32, device=x.device)
    db = torch.empty((cout,), dtype=torch.float32, device=x.device) if bias else None
    L.check(L.lib().mmpde_conv2d_grad_weight(L.ptr(x), bt, cin, h, wd, L.ptr(dy), cout, ks, pad,
                                             L.PAD_CIRCULAR if circular else L.PAD_ZEROS, L.ptr(dw), L.ptr(db),
                                             L.stream(x.device)), "mmpde_conv2d_grad_weight")
    return dw, db


class LinearRows(torch.autograd.Function):
    """y = x W^T + b over many rows: the train-mode Linears of GNN_Layer_FS_2D /
    MP_PDE_Solver_2D (gnn_2d.py:53-69,99-114) and ItpNet (interpolate.py:79-93)
    on the HIP row GEMMs (rows.py, csrc/rgemm.hip: exact fp32 MFMA): forward
    mmpde_rgemm (NT), dX = dY W mmpde_rgemm (NN), dW = dY^T X and db over the
    rows in fixed row chunks (mmpde_rgemm_tn), or for a skinny map (the Conv1d
    head's windows, the embedding's first Linear) mmpde_rows_grad_weight.  No
    library GEMM; deterministic for a given shape."""

    @staticmethod
    def forward(ctx, x, w, b):
        L.require_device(x, w, b)
        x, wc = L.f32c(x), L.f32c(w)
        ctx.save_for_backward(x, wc)
        ctx.has_bias = b is not None
        return rows.linear_fwd(x, wc, L.f32c(b) if b is not None else None)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = L.f32c(dy)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = rows.linear_bwd_input(dy, w)
        n, k = x.shape
        nout = w.shape[0]
        want_b = ctx.has_bias and ctx.needs_input_grad[2]
        if not (want_b or ctx.needs_input_grad[1]):
            return gx, None, None          # frozen weight and bias: dX only
        if n >= 4096 and rows_grad_fits(k, nout):
            # skinny map (head windows, embedding): dW and db in one row pass
            gw, gb = rows_grad_weight(x, dy, k if ctx.needs_input_grad[1] else 0, want_b)
            return gx, gw, gb
        gw = torch.empty_like(w) if ctx.needs_input_grad[1] else None
        gb = torch.empty((nout,), dtype=torch.float32, device=x.device) if want_b else None
        rows.linear_bwd_weight(dy, x, gw, gb)
        return gx, gw, gb


def rows_grad_fits(k: int, nout: int) -> bool:
    """Shapes mmpde_rows_grad_weight takes with the weight gradient."""
    return 0 < k <= 64 and nout <= 128 and k * nout + nout <= 1280


class HeadTrain(torch.autograd.Function):
    """output_mlp(h[:, None]) of MP_PDE_Solver_2D at time_window 1 (gnn_2d.py:
    108-114: Conv1d(1, 4, 16, 3) -> ReLU -> Conv1d(4, 8, 12, 3) -> ReLU ->
    Conv1d(8, 1, 8, 2)) in train mode: y [n, 1] from h [n, 128] on
    mmpde_head_train_forward, dL/dh and the six weight / bias gradients on
    mmpde_head_train_backward (one lane per node, fixed summation orders)."""

    @staticmethod
    def forward(ctx, h, w1, b1, w2, b2, w3, b3):
        L.require_device(h, w1, b1, w2, b2, w3, b3)
        h = L.f32c(h)
        ws = [L.f32c(t) for t in (w1, b1, w2, b2, w3, b3)]
        n = h.shape[0]
        y = torch.empty((n, 1), dtype=torch.float32, device=h.device)
        L.check(L.lib().mmpde_head_train_forward(L.ptr(h), h.stride(0), n, *[L.ptr(t) for t in ws], L.ptr(y),
                                                 L.stream(h.device)), "mmpde_head_train_forward")
        ctx.save_for_backward(h, *ws)
        ctx.shapes = [tuple(t.shape) for t in (w1, b1, w2, b2, w3, b3)]
        return y

    @staticmethod
    def backward(ctx, dy):
        h, *ws = ctx.saved_tensors
        dy = L.f32c(dy)
        n = h.shape[0]
        dev = h.device
        dh = torch.empty_like(h)
        grads = torch.empty((HEAD_TRAIN_GRADS,), dtype=torch.float32, device=dev)
        nb = L.lib().mmpde_head_train_workspace_bytes(n)
        wk = torch.empty((nb // 4,), dtype=torch.float32, device=dev)
        L.check(L.lib().mmpde_head_train_backward(L.ptr(h), h.stride(0), n, *[L.ptr(t) for t in ws], L.ptr(dy),
                                                  L.ptr(dh), dh.stride(0), L.ptr(grads), L.ptr(wk), nb,
                                                  L.stream(dev)), "mmpde_head_train_backward")
        out, o = [], 0
        for shp in ctx.shapes:
            k = 1
            for d in shp:
                k *= d
            out.append(grads[o:o + k].view(shp))
            o += k
        gh = dh if ctx.needs_input_grad[0] else None
        return (gh, *[g if ctx.needs_input_grad[1 + j] else None for j, g in enumerate(out)])


HEAD_TRAIN_GRADS = 525  # include/mmpde_hip.h MMPDE_HEAD_TRAIN_GRADS


def head_train_fits(output_mlp, h: torch.Tensor) -> bool:
    """The Conv1d head HeadTrain implements (gnn_2d.py:108-114 at time_window 1).
    MMPDE_HEAD_FUSED=0 keeps the unfold + LinearRows form (A/B runs)."""
    if os.environ.get("MMPDE_HEAD_FUSED", "1") == "0":
        return False
    try:
        convs = [output_mlp[i] for i in (0, 2, 4)]
    except (IndexError, TypeError):
        return False
    if len(output_mlp) != 5 or not all(isinstance(c, torch.nn.Conv1d) for c in convs):
        return False
    want = [((4, 1, 16), 3), ((8, 4, 12), 3), ((1, 8, 8), 2)]
    for c, (shape, st) in zip(convs, want):
        if (tuple(c.weight.shape) != shape or c.stride[0] != st or c.padding[0] != 0 or c.dilation[0] != 1
                or c.groups != 1 or c.bias is None or c.padding_mode != "zeros"):
            return False
    return (isinstance(output_mlp[1], torch.nn.ReLU) and isinstance(output_mlp[3], torch.nn.ReLU)
            and h.dim() == 2 and h.shape[1] == 128 and h.is_cuda and h.dtype == torch.float32)


def rows_grad_weight(x: torch.Tensor, dy: torch.Tensor, k: int, bias: bool):
    """(dW = dy^T x [nout, k] or None when k = 0, db = sum_rows dy or None) on
    mmpde_rows_grad_weight (fixed summation order)."""
    rows, nout = dy.shape
    dy = L.f32c(dy)
    x = L.f32c(x) if k else None
    dev = dy.device
    gw = torch.empty((nout, k), dtype=torch.float32, device=dev) if k else None
    gb = torch.empty((nout,), dtype=torch.float32, device=dev) if bias else None
    nb = L.lib().mmpde_rows_grad_weight_workspace_bytes(rows, k, nout)
    ws = torch.empty((nb // 4,), dtype=torch.float32, device=dev)
    L.check(L.lib().mmpde_rows_grad_weight(L.ptr(x), x.stride(0) if k else 0, rows, k, L.ptr(dy), dy.stride(0),
                                           nout, L.ptr(gw), L.ptr(gb), L.ptr(ws), nb, L.stream(dev)),
            "mmpde_rows_grad_weight")
    return gw, gb


class BatchNormRows(torch.autograd.Function):
    """nn.BatchNorm1d in train mode over [n, C] rows of x + res (the residual
    add of GNN_Layer_FS_2D, norm(h + update), gnn_2d.py:69, and the
    embedding's BatchNorm1d, gnn_2d.py:101,105) on
    mmpde_batch_norm_rows_train / _backward: batch statistics, running
    statistics update in place, normalisation; gradients for x, res, weight
    and bias.  Deterministic."""

    @staticmethod
    def forward(ctx, x, res, weight, bias, eps, factor, running_mean, running_var):
        n, C = x.shape
        dev = x.device
        y = torch.empty_like(x)
        stats = torch.empty((4 * C,), dtype=torch.float32, device=dev)
        nb = L.lib().mmpde_batch_norm_rows_workspace_bytes(n, C) + 12 * C
        ws = torch.empty((nb // 4,), dtype=torch.float32, device=dev)
        L.check(L.lib().mmpde_batch_norm_rows_train(
            L.ptr(x), L.ptr(res), n, C, L.ptr(weight), L.ptr(bias), float(eps), float(factor),
            L.ptr(running_mean), L.ptr(running_var), L.ptr(y), L.ptr(stats), L.ptr(ws), nb, L.stream(dev)),
            "mmpde_batch_norm_rows_train")
        ctx.save_for_backward(x, res, weight, stats)
        ctx.ws = nb
        ctx.has = (res is not None, weight is not None, bias is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, res, weight, stats = ctx.saved_tensors
        has_res, has_w, has_b = ctx.has
        n, C = x.shape
        dev = x.device
        dy = L.f32c(dy)
        dx = torch.empty_like(x)
        dw = torch.empty((C,), dtype=torch.float32, device=dev) if has_w else None
        db = torch.empty((C,), dtype=torch.float32, device=dev) if has_b else None
        ws = torch.empty((ctx.ws // 4,), dtype=torch.float32, device=dev)
        L.check(L.lib().mmpde_batch_norm_rows_backward(
            L.ptr(x), L.ptr(res), L.ptr(dy), n, C, L.ptr(weight), L.ptr(stats), L.ptr(dx), L.ptr(dw), L.ptr(db),
            L.ptr(ws), ctx.ws, L.stream(dev)), "mmpde_batch_norm_rows_backward")
        return dx, (dx if has_res else None), dw, db, None, None, None, None


def batch_norm_rows(bn: torch.nn.BatchNorm1d, x: torch.Tensor, res: torch.Tensor | None = None) -> torch.Tensor:
    """bn(x + res) for [n, C] rows: the HIP kernels in train mode (running
    statistics and num_batches_tracked advanced as nn.BatchNorm1d does), the
    module itself in eval mode."""
    if not bn.training or x.dim() != 2 or x.shape[1] % 4 or x.shape[1] > 1024 or x.shape[0] < 2:
        return bn(x if res is None else x + res)
    factor = 0.0
    if bn.track_running_stats and bn.num_batches_tracked is not None:
        bn.num_batches_tracked.add_(1)
        factor = 1.0 / float(bn.num_batches_tracked) if bn.momentum is None else bn.momentum
    rm = bn.running_mean if bn.track_running_stats else None
    rv = bn.running_var if bn.track_running_stats else None
    x = x.float().contiguous()                  # no detach: autograd inputs
    res = res.float().contiguous() if res is not None else None
    return BatchNormRows.apply(x, res, bn.weight, bn.bias, bn.eps, factor, rm, rv)


def linear_train(x: torch.Tensor, lin: torch.nn.Linear) -> torch.Tensor:
    """lin(x) for [n, k] rows in train mode through LinearRows."""
    return LinearRows.apply(x.contiguous(), lin.weight, lin.bias)


class Conv2dSame(torch.autograd.Function):
    """Differentiable stride-1 conv2d with output size = input size (odd ks,
    pad = ks // 2), zero or circular padding, on the HIP kernels: forward
    mmpde_conv2d_ex; backward dx = the same convolution of dy with the flipped,
    transposed kernel (circular indices wrap the same way), dw / db
    mmpde_conv2d_grad_weight.  Deterministic."""

    @staticmethod
    def forward(ctx, x, w, b, circular: bool):
        ks = w.shape[-1]
        if w.shape[-2] != ks or ks % 2 != 1:
            raise ValueError("Conv2dSame takes square odd kernels")
        ctx.save_for_backward(x, w)
        ctx.circular = circular
        ctx.has_bias = b is not None
        return conv2d(x, w, b, 1, ks // 2, L.ACT_NONE, circular=circular)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        ks = w.shape[-1]
        dy = L.f32c(dy)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            wt = w.flip(2, 3).transpose(0, 1).contiguous()
            gx = conv2d(dy, wt, None, 1, ks // 2, L.ACT_NONE, circular=ctx.circular)
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            gw, gb = conv2d_grad_weight(x, dy, ks, ks // 2, ctx.circular, bias=ctx.has_bias)
        return gx, gw, gb, None


def itp_interp(src, vals, qry, idx, batches: int, packed: torch.Tensor, addend=None, addend2=None):
    """ItpNet weights + weighted neighbour sum (interpolate.py:77-93,
    data_creator_2d.py:80-83), + addend, then + addend2 (both optional).
    Returns [batches * n_qry] fp32."""
    L.require_device(src, vals, qry, idx, packed)
    src = L.f32c(src).reshape(-1, 2)
    qry = L.f32c(qry).reshape(-1, 2)
    vals = L.f32c(vals).reshape(-1)
    ns, nq = src.shape[0] // batches, qry.shape[0] // batches
    out = torch.empty((batches * nq,), dtype=torch.float32, device=src.device)
    add = L.f32c(addend).reshape(-1) if addend is not None else None
    add2 = L.f32c(addend2).reshape(-1) if addend2 is not None else None
    L.check(L.lib().mmpde_itp_interp_ex(L.ptr(src), L.ptr(vals), L.ptr(qry), L.ptr(idx.contiguous()),
                                        batches, ns, nq, L.ptr(packed), L.ptr(add), L.ptr(add2),
                                        L.ptr(out), L.stream(src.device)), "mmpde_itp_interp_ex")
    return out


def reverse_adjacency(nbr: torch.Tensor, degree: torch.Tensor | None = None,
                      n_src: int | None = None, check: bool = True, slot_pos: bool = False):
    """Source-major view of a target-major table, for the source-side gradient of
    the edge stage (mmpde_gnn_edge_source_sum): rev_edge int64 = the live slot
    ids i*k+e grouped by source j (stable: target order within a source),
    rev_off int64 [n_src+1] = the group offsets (n_src defaults to the number of
    targets).  Device tables: mmpde_reverse_adjacency (no host round trip
    unless `check`, which reads back the count of sources outside [0, n_src)
    and raises on any; the engine's own kNN tables pass check=False;
    slot_pos=True adds the int32 [nt*k] position of every slot in that order,
    for mmpde_gnn_edge_backward_sorted).  Host tables (tests): the same lists
    from a stable argsort."""
    nt, k = nbr.shape
    n = nt if n_src is None else n_src
    if nbr.is_cuda:
        dev = nbr.device
        nbr = nbr.to(torch.int32).contiguous()
        deg = degree.to(torch.int32).contiguous() if degree is not None else None
        rev_off = torch.empty((n + 1,), dtype=torch.int64, device=dev)
        rev_edge = torch.empty((max(nt * k, 1),), dtype=torch.int64, device=dev)
        sb = L.lib().mmpde_reverse_adjacency_scratch_bytes(nt, k, n)
        scratch = torch.empty(((sb + 255) // 256 * 64,), dtype=torch.float32, device=dev).view(torch.uint8)
        bad = torch.empty((1,), dtype=torch.int32, device=dev)
        pos = torch.empty((max(nt * k, 1),), dtype=torch.int32, device=dev) if slot_pos else None
        L.check(L.lib().mmpde_reverse_adjacency(L.ptr(nbr), nt, k, L.ptr(deg), n, L.ptr(rev_off),
                                                L.ptr(rev_edge), L.ptr(pos), L.ptr(scratch), scratch.numel(),
                                                L.ptr(bad), L.stream(dev)), "mmpde_reverse_adjacency")
        if check and int(bad.item()):
            raise ValueError("neighbour table holds sources outside [0, n)")
        return (rev_off, rev_edge, pos) if slot_pos else (rev_off, rev_edge)
    if slot_pos:
        raise ValueError("slot_pos: device tables only")
    src = nbr.reshape(-1).long()
    slot = torch.arange(nt * k, device=nbr.device)
    if degree is not None:
        live = (torch.arange(k, device=nbr.device)[None, :] < degree[:, None].long()).reshape(-1)
        src, slot = src[live], slot[live]
    if src.numel() and (int(src.min()) < 0 or int(src.max()) >= n):
        raise ValueError("neighbour table holds sources outside [0, n)")
    order = torch.argsort(src, stable=True)
    rev_edge = slot[order].contiguous()
    rev_off = torch.zeros((n + 1,), dtype=torch.int64, device=nbr.device)
    rev_off[1:] = torch.cumsum(torch.bincount(src, minlength=n), 0)
    return rev_off, rev_edge


class GatherRows(torch.autograd.Function):
    """rows[idx] for a flat index list, whose backward is the fixed-order
    segmented sum mmpde_segment_sum over the reverse index lists (torch's
    scatter-add backward of a gather accumulates with atomics, in no fixed
    order).  rows [n, w] fp32, idx int [m] -> [m, w]."""

    @staticmethod
    def forward(ctx, rows, idx, check=False):
        L.require_device(rows, idx)
        ctx.n = rows.shape[0]
        ctx.idx = idx
        ctx.check = check      # idx from the engine's kNN kernels: in range
        return rows[idx.long()]

    @staticmethod
    def backward(ctx, g):
        g = L.f32c(g)
        n, w = ctx.n, g.shape[1]
        rev_off, rev_edge = reverse_adjacency(ctx.idx.reshape(-1, 1), n_src=n, check=ctx.check)
        out = torch.empty((n, w), dtype=torch.float32, device=g.device)
        L.check(L.lib().mmpde_segment_sum(L.ptr(g), w, L.ptr(rev_off), L.ptr(rev_edge), n,
                                          L.ptr(out), L.stream(g.device)), "mmpde_segment_sum")
        return out, None, None
