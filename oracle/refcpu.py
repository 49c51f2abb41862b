"""oracle/refcpu.py -- TEST INFRASTRUCTURE ONLY.  CPU restatement of the MM-PDE
forward step, used as the parity checker and as bench.py's CPU baseline
(``cpu_baseline.kind == "port"``).  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s cpu_baseline leg may import this module.  Nothing in the
product package (``mm-pde_amd/mmpde_amd``) imports it.

Written from the source text of the reference (Peiyannn/MM-PDE, read-only at
/root/reference; running it in this container was refused -- SURVEY.md §8(c)),
op for op and unfused, in the reference's own order:

* dense arithmetic (Linear / BatchNorm(eval) / Conv1d / Conv2d / tanh / relu /
  autograd.grad) is done with the very torch ops the reference calls, so it is
  pinned by torch itself;
* PyG 2.0.3 ``MessagePassing.propagate`` (aggr='mean', flow source->target) and
  torch_scatter 2.0.9 ``scatter(reduce='mean')`` are restated explicitly
  (gather x_i = x[edge_index[1]], x_j = x[edge_index[0]], sum at the target,
  divide by the in-degree clamped to >= 1);
* torch_cluster 1.5.9 ``knn_graph`` and sklearn 1.3.0 ``NearestNeighbors`` are
  restated in C (oracle/knn_oracle.c), loaded through ctypes.

Parity status: torch ops -- pinned (same library);
sklearn kNN-30 -- pinned against sklearn 1.7.2 fixtures on tie-free inputs;
torch_cluster kNN graph and the PyG mean aggregation -- "parity unpinned"
(restated from the published algorithm; hand KATs in tests/).

All functions take plain ``state_dict``-style dicts whose keys are exactly the
reference module's ``state_dict()`` keys.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np
import torch
import torch.nn.functional as F

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "_build", "libknn_oracle.so")
        if not os.path.exists(path):
            subprocess.run(["make", "-s", "-C", _HERE], check=True)
        lib = ctypes.CDLL(path)
        lib.knn_graph_oracle.restype = ctypes.c_int64
        lib.knn_graph_oracle.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                         ctypes.c_int, ctypes.c_void_p]
        lib.knn_query_oracle.restype = ctypes.c_int64
        lib.knn_query_oracle.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                         ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                         ctypes.c_void_p]
        lib.radius_graph_oracle.restype = None
        lib.radius_graph_oracle.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                            ctypes.c_float, ctypes.c_int, ctypes.c_void_p,
                                            ctypes.c_void_p]
        _LIB = lib
    return _LIB


# ----------------------------------------------------------------------------
# PDE descriptors -- reference PDEs.py:20-41 (burgers), 44-67 (cy)
# ----------------------------------------------------------------------------
class PDEConst:
    def __init__(self, kind, grid_size, ori_grid=None):
        self.kind = kind
        if kind == "burgers":                      # PDEs.py:20-41
            self.tmin, self.tmax, self.Lx, self.Ly = 0, 30, 1, 1
            self.dt = self.tmax / (31 - 1)          # dt from the DEFAULT grid (31,96,96)
        elif kind == "cy":                          # PDEs.py:44-67
            self.tmin, self.tmax, self.Lx, self.Ly = 0, 2.9, 1, 1
            self.dt = self.tmax / (30 - 1)          # dt from the DEFAULT grid (30,2521)
        else:
            raise ValueError(kind)
        # mmpde.py:179-181 overwrites the three grid sizes with --base_resolution
        self.grid_size = tuple(grid_size)
        self.movingmesh_grid_size = tuple(grid_size)
        self.ori_grid_size = tuple(grid_size)
        self.ori_grid = ori_grid


# ----------------------------------------------------------------------------
# kNN searches (C restatement, oracle/knn_oracle.c)
# ----------------------------------------------------------------------------
def knn_graph(x: torch.Tensor, k: int, batches: int):
    """torch_cluster.knn_graph(x, k, batch, loop=False), flow source->target, for
    equal-size contiguous batch segments.  Returns (edge_index [2, n*k] int64,
    nbr [n, k] int64, degenerate_count).  edge_index[0] = source (neighbour),
    edge_index[1] = target (query) -- reference data_creator_2d.py:260."""
    x = x.detach().to(torch.float32).contiguous().cpu()
    n = x.shape[0]
    n_per = n // batches
    assert n_per * batches == n
    nbr = torch.empty((n, k), dtype=torch.int64)
    deg = _lib().knn_graph_oracle(x.data_ptr(), batches, n_per, k, nbr.data_ptr())
    tgt = torch.arange(n, dtype=torch.int64).repeat_interleave(k)
    edge_index = torch.stack([nbr.reshape(-1), tgt])
    return edge_index, nbr, int(deg)


def radius_graph(x: torch.Tensor, r: float, batches: int, max_num_neighbors: int = 32):
    """torch_cluster.radius_graph(x, r, batch, loop=False, max_num_neighbors), CUDA
    semantics, equal contiguous batch segments (reference data_creator_2d.py:257-258).
    Returns (edge_index [2, E] int64 target-major, nbr [n, max_nn+1] int64 padded
    with -1, deg [n] int64)."""
    x = x.detach().to(torch.float32).contiguous().cpu()
    n = x.shape[0]
    n_per = n // batches
    assert n_per * batches == n
    w = max_num_neighbors + 1
    nbr = torch.empty((n, w), dtype=torch.int64)
    deg = torch.empty((n,), dtype=torch.int64)
    _lib().radius_graph_oracle(x.data_ptr(), batches, n_per, r, max_num_neighbors,
                               nbr.data_ptr(), deg.data_ptr())
    keep = torch.arange(w)[None, :] < deg[:, None]
    tgt = torch.arange(n)[:, None].expand(n, w)
    edge_index = torch.stack([nbr[keep], tgt[keep]])
    return edge_index, nbr, deg


def knn_query(src: torch.Tensor, qry: torch.Tensor, batches: int, k: int):
    """Per-trajectory sklearn NearestNeighbors(k).fit(src_b).kneighbors(qry_b)
    indices (local, sorted by (float64 distance, index)) -- reference
    data_creator_2d.py:66-78.  Returns int64 [batches, n_qry, k]."""
    src = src.detach().to(torch.float32).contiguous().cpu()
    qry = qry.detach().to(torch.float32).contiguous().cpu()
    n_src = src.shape[0] // batches
    n_qry = qry.shape[0] // batches
    idx = torch.empty((batches, n_qry, k), dtype=torch.int64)
    _lib().knn_query_oracle(src.data_ptr(), qry.data_ptr(), batches, n_src, n_qry, k,
                            idx.data_ptr())
    return idx


# ----------------------------------------------------------------------------
# small functional helpers, same torch ops as the reference modules
# ----------------------------------------------------------------------------
# Activation pattern hook (tests only): None = torch.relu everywhere (the
# reference's op).  A callable (sd, prefix, site) -> bool mask or None imposes
# a given ReLU pattern at a site: relu(x) becomes x * mask, so the forward
# keeps the same values wherever the pattern agrees with x's sign, and the
# backward is gated by the mask.  Sites: "emb" (embedding_mlp.2), and per GNN
# layer "z1" (message_net_1, [E, 128] in edge order i k + e), "z2"
# (message_net_2), "v" (update_net_1), "upd" (update_net_2).  The training
# tests condition the float64 oracle on the HIP forward's own pattern
# (mmpde_amd.gnn_2d.RELU_RECORD): an activation within rounding of a kink then
# cannot take different sides in the two evaluations.
RELU_PATTERN = None


def _relu(sd, p, site, x):
    m = RELU_PATTERN(sd, p, site) if RELU_PATTERN is not None else None
    return torch.relu(x) if m is None else x * m.to(x.dtype)


def _lin(sd, p, x):
    return F.linear(x, sd[p + ".weight"], sd[p + ".bias"])


def _bn(sd, p, x, eps=1e-5, train=False, momentum=0.1):
    # nn.BatchNorm1d in eval() (model.eval(), mmpde.py:132-136 / 201); with
    # train=True the training-mode module (model.train(), mmpde.py:71-73): batch
    # statistics, running buffers of `sd` updated in place (momentum 0.1)
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"],
                        sd[p + ".weight"], sd[p + ".bias"], train, momentum if train else 0.0, eps)


def propagate_mean(edge_index, n, message_fn):
    """PyG 2.0.3 MessagePassing.propagate with aggr='mean', flow source->target:
    i = edge_index[1] (target), j = edge_index[0] (source); torch_scatter mean
    divides the scattered sum by the in-degree clamped to >= 1."""
    j, i = edge_index[0], edge_index[1]
    msg = message_fn(i, j)                                   # [E, F]
    out = torch.zeros((n, msg.shape[1]), dtype=msg.dtype)
    out.index_add_(0, i, msg)
    cnt = torch.zeros((n,), dtype=msg.dtype)
    cnt.index_add_(0, i, torch.ones_like(i, dtype=msg.dtype))
    return out / cnt.clamp(min=1)[:, None]


# ----------------------------------------------------------------------------
# MP_PDE_Solver_2D -- reference gnn_2d.py:19-141
# ----------------------------------------------------------------------------
def gnn_layer(sd, p, x, u, pos_x, pos_y, variables, edge_index, train=False):
    """GNN_Layer_FS_2D.forward / message / update, gnn_2d.py:53-69."""
    n = x.shape[0]

    def message(i, j):  # gnn_2d.py:59-63
        m = torch.cat((x[i], x[j], u[i] - u[j], pos_x[i] - pos_x[j],
                       pos_y[i] - pos_y[j], variables[i]), dim=-1)
        m = _relu(sd, p, "z1", _lin(sd, p + ".message_net_1.0", m))
        return _relu(sd, p, "z2", _lin(sd, p + ".message_net_2.0", m))

    agg = propagate_mean(edge_index, n, message)
    # update, gnn_2d.py:65-69
    upd = _relu(sd, p, "v", _lin(sd, p + ".update_net_1.0", torch.cat((x, agg, variables), dim=-1)))
    upd = _relu(sd, p, "upd", _lin(sd, p + ".update_net_2.0", upd))
    x = x + upd
    # PyG BatchNorm wraps nn.BatchNorm1d as `.module` (gnn_2d.py:51,56)
    return _bn(sd, p + ".norm.module", x, train=train)


def mp_pde_solver(sd, pde: PDEConst, u, pos, edge_index, time_window=1, hidden_layer=6,
                  return_hidden=False, train=False):
    """MP_PDE_Solver_2D.forward, gnn_2d.py:119-141.  u=[n,tw], pos=[n,3]=(t,x,y).
    train=True: the model.train() forward (BatchNorm on batch statistics)."""
    pos_x = pos[:, 1][:, None] / pde.Lx
    pos_y = pos[:, 2][:, None] / pde.Ly
    pos_t = pos[:, 0][:, None] / pde.tmax
    variables = pos_t
    node_input = torch.cat((u, pos_x, pos_y, variables), -1)
    # embedding_mlp, gnn_2d.py:99-106
    h = _lin(sd, "embedding_mlp.0", node_input)
    h = _relu(sd, "embedding_mlp", "emb", _bn(sd, "embedding_mlp.1", h, train=train))
    h = _bn(sd, "embedding_mlp.4", _lin(sd, "embedding_mlp.3", h), train=train)
    hs = [h]
    for i in range(hidden_layer):
        h = gnn_layer(sd, f"gnn_layers.{i}", h, u, pos_x, pos_y, variables, edge_index,
                      train=train)
        hs.append(h)
    # output_mlp Conv1d head, gnn_2d.py:108-114,136
    d = h[:, None]
    d = torch.relu(F.conv1d(d, sd["output_mlp.0.weight"], sd["output_mlp.0.bias"], stride=3))
    d = torch.relu(F.conv1d(d, sd["output_mlp.2.weight"], sd["output_mlp.2.bias"], stride=3))
    d = F.conv1d(d, sd["output_mlp.4.weight"], sd["output_mlp.4.bias"], stride=2)
    diff = d.squeeze(1)
    dt = torch.ones(1, time_window) * pde.dt * 0.1          # gnn_2d.py:137-139
    dt = torch.cumsum(dt, dim=1)
    out = dt * diff
    if return_hidden:
        return out, hs
    return out


# ----------------------------------------------------------------------------
# DMM -- reference mesh/dmm_model.py
# ----------------------------------------------------------------------------
def densenet(sd, p, x, n_layers):
    """DenseNet.forward (normalize=False), dmm_model.py:31-45: tanh on all but the
    last layer; returns (out, last hidden)."""
    out = None
    for li in range(n_layers):
        if li != n_layers - 1:
            x = torch.tanh(_lin(sd, f"{p}.layers.{li}", x))
        else:
            out = _lin(sd, f"{p}.layers.{li}", x)
    return out, x


def convnet(sd, p, x):
    """ConvNet.forward (layers == 7), dmm_model.py:65-81. x=[B,1,s,s]."""
    ws = [(f"{p}.layers.{i}", st) for i, st in ((0, 2), (1, 1), (2, 1), (3, 2))]
    ori_x = None
    nl = len(ws)
    for i, (q, st) in enumerate(ws):
        if i != nl - 2:
            x = torch.tanh(F.conv2d(x, sd[q + ".weight"], sd[q + ".bias"], stride=st, padding=2))
        if i == 0:
            ori_x = x
        if i == nl - 2:
            x = torch.tanh(ori_x + F.conv2d(x, sd[q + ".weight"], sd[q + ".bias"], stride=st,
                                            padding=2))
    x = torch.flatten(x, 1)
    x = torch.tanh(_lin(sd, f"{p}.fc2", x))
    return _lin(sd, f"{p}.fc3", x)


def basecnn(sd, dt, u, tw):
    """BaseCNN.forward, models_cnn.py:66-83: circular-padded Conv2d stack with ELU
    and residuals (padding_mode='circular' = F.pad(mode='circular') + valid conv),
    then u[:, -1] + cumsum(dt) * x, squeezed.  u [B, tw, X, Y]."""
    def conv(i, x):
        w, b = sd[f"conv{i}.weight"], sd[f"conv{i}.bias"]
        p = w.shape[-1] // 2
        return F.conv2d(F.pad(x, (p, p, p, p), mode="circular"), w, b)

    x = F.elu(conv(1, u))
    for i in range(2, 8):
        x = x + F.elu(conv(i, x))
    x = conv(8, x)
    dtc = torch.cumsum(torch.ones(1, tw) * dt, dim=1)[None, :, :, None, None]
    out = u[:, -1, :, :][:, None, None, :, :].repeat(1, 1, tw, 1, 1) + dtc * x[:, None, :, :, :]
    return out.squeeze()


def dmm_gnn_layer(sd, p, x, u, pos_x, pos_y, edge_index, train=False):
    """DMM GNN_Layer_FS_2D (tanh), dmm_model.py:126-142 (train: BatchNorm on
    batch statistics, the DMM training forward)."""
    n = x.shape[0]

    def message(i, j):
        m = torch.cat((x[i], x[j], u[i] - u[j], pos_x[i] - pos_x[j], pos_y[i] - pos_y[j]),
                      dim=-1)
        m = torch.tanh(_lin(sd, p + ".message_net_1.0", m))
        return torch.tanh(_lin(sd, p + ".message_net_2.0", m))

    agg = propagate_mean(edge_index, n, message)
    upd = torch.tanh(_lin(sd, p + ".update_net_1.0", torch.cat((x, agg), dim=-1)))
    upd = torch.tanh(_lin(sd, p + ".update_net_2.0", upd))
    return _bn(sd, p + ".norm.module", x + upd, train=train)


def dmm_forward(sd, mode, u, grid, ori_grid=None, hidden_layer=3, grid_edge_index=None,
                train=False):
    """DMM.forward(u, grid), dmm_model.py:185-219.  `grid` is xi [B*N, 2].
    train=True: the train() forward of DMM training (BatchNorm on batch
    statistics, running buffers of `sd` updated)."""
    B = u.shape[0]
    if mode == "array":
        branch = convnet(sd, "branch", u.unsqueeze(1)).unsqueeze(1)
        branch = branch.repeat(1, int(grid.shape[0] / u.shape[0]), 1)
        trunk, _ = densenet(sd, "trunk", grid, 2)
    else:
        # create_graph, dmm_model.py:222-234 (kNN-35 on the fixed grid)
        N = ori_grid.shape[0]
        gpos = ori_grid[None].repeat(B, 1, 1).reshape(-1, 2)
        if grid_edge_index is None:
            grid_edge_index, _, _ = knn_graph(gpos, 35, B)
        x = u.reshape(-1, 1)
        pos_x = gpos[:, 0][:, None]
        pos_y = gpos[:, 1][:, None]
        h = _lin(sd, "embedding_mlp.0", torch.cat((x, pos_x, pos_y), -1))
        h = torch.tanh(_bn(sd, "embedding_mlp.1", h, train=train))
        h = _bn(sd, "embedding_mlp.4", _lin(sd, "embedding_mlp.3", h), train=train)
        for i in range(hidden_layer):
            h = dmm_gnn_layer(sd, f"gnn_layers.{i}", h, x, pos_x, pos_y, grid_edge_index,
                              train=train)
        h, _ = densenet(sd, "decoding_mlp", h, 2)
        b = h.reshape(B, 1, -1)
        b = torch.tanh(_lin(sd, "output_mlp.0", b))
        b = torch.tanh(_lin(sd, "output_mlp.2", b))
        b = _lin(sd, "output_mlp.4", b)
        branch = b.repeat(1, int(grid.shape[0] / u.shape[0]), 1)
        trunk, _ = densenet(sd, "trunk", grid, 2)
    out, _ = densenet(sd, "out_nn",
                      torch.cat((branch.reshape(-1, branch.shape[-1]),
                                 trunk.reshape(-1, branch.shape[-1])), dim=-1), 2)
    return out


# ----------------------------------------------------------------------------
# ItpNet -- reference interpolate.py:77-99
# ----------------------------------------------------------------------------
def itpnet(sd, neighbors, query_points, mode, data=None, burgers=False):
    if mode in ("1", "2"):
        pre = "layers" if mode == "1" else "layers2"
        x = torch.cat((neighbors, query_points), dim=-2).reshape(
            neighbors.shape[0], neighbors.shape[1], -1)
        for li in range(3):
            x = _lin(sd, f"{pre}.{li}", x)
            if li != 2:
                x = torch.tanh(x)
        return x
    if mode == "res_cut":
        if burgers:  # 4x Conv2d 5x5 pad 2 + Tanh after each (interpolate.py:63-72)
            for li in (0, 2, 4, 6):
                data = torch.tanh(F.conv2d(data, sd[f"down.{li}.weight"], sd[f"down.{li}.bias"],
                                           padding=2))
            return data
        # Linear 2521->2048->512->2048->2521, tanh on the first three (interpolate.py:74-82)
        for li in (0, 2, 4, 6):
            data = _lin(sd, f"down.{li}", data)
            if li != 6:
                data = torch.tanh(data)
        return data
    raise ValueError(mode)


# ----------------------------------------------------------------------------
# GraphCreator_FS_2D -- reference data_creator_2d.py
# ----------------------------------------------------------------------------
def interpolate(itp_sd, u, init_x, init_y, x, y, mode, burgers=False, return_idx=False,
                idx=None):
    """data_creator_2d.py:46-85 (per-trajectory sklearn kNN-30 + ItpNet weights)."""
    nu = u.shape[0]
    all_points = torch.cat((init_x, init_y), -1).reshape(nu, -1, 2)
    all_query_points = torch.cat((x, y), dim=-1).reshape(nu, -1, 2)
    if idx is None:
        idx = knn_query(all_points.reshape(-1, 2), all_query_points.reshape(-1, 2), nu, 30)
    neighbors, neighbor_labels = [], []
    for k in range(nu):
        labels = u[k].reshape(-1)
        neighbors.append(all_points[k][idx[k]])
        neighbor_labels.append(labels[idx[k]])
    neighbors = torch.stack(neighbors)
    neighbor_labels = torch.stack(neighbor_labels)
    weights = itpnet(itp_sd, neighbors, all_query_points.unsqueeze(-2), mode)
    out = torch.sum(weights * neighbor_labels, dim=-1).reshape(-1)
    if return_idx:
        return out, idx
    return out


def moving_mesh_tri(dmm_sd, u, grid_x, grid_y, ori_grid, grid_edge_index=None):
    """data_creator_2d.py:115-137 -- x = xi + d(phi)/d(xi) via two autograd.grad."""
    xi1, xi2 = grid_x.reshape(-1, 1).clone(), grid_y.reshape(-1, 1).clone()
    xi1.requires_grad = True
    xi2.requires_grad = True
    with torch.enable_grad():
        xi = torch.cat((xi1, xi2), dim=-1)
        phi = dmm_forward(dmm_sd, "graph", u, xi, ori_grid=ori_grid,
                          grid_edge_index=grid_edge_index)
        w = torch.ones(phi.shape)
        x1 = torch.autograd.grad(phi, xi1, grad_outputs=w, retain_graph=True,
                                 create_graph=True, allow_unused=True)[0] + xi1
        x2 = torch.autograd.grad(phi, xi2, grad_outputs=w, retain_graph=True,
                                 create_graph=True, allow_unused=True)[0] + xi2
    alpha = 1
    x1 = alpha * x1 + (1 - alpha) * xi1
    x2 = alpha * x2 + (1 - alpha) * xi2
    return x1.detach(), x2.detach()


def moving_mesh(dmm_sd, pde: PDEConst, u, n_grid_x, n_grid_y):
    """data_creator_2d.py:88-113 -- burgers; xi from np.meshgrid (xy order)."""
    grid_x = np.linspace(0, pde.Lx, n_grid_x)
    grid_y = np.linspace(0, pde.Ly, n_grid_y)
    grid = torch.tensor(np.array(np.meshgrid(grid_x, grid_y)), dtype=torch.float
                        ).reshape(2, -1).permute(1, 0)
    xi1 = grid[:, [0]].unsqueeze(0).repeat(u.shape[0], 1, 1).reshape(-1, 1)
    xi2 = grid[:, [1]].unsqueeze(0).repeat(u.shape[0], 1, 1).reshape(-1, 1)
    xi1 = xi1.detach().clone().requires_grad_(True)
    xi2 = xi2.detach().clone().requires_grad_(True)
    if pde.movingmesh_grid_size[-2] != n_grid_x or pde.movingmesh_grid_size[-1] != n_grid_y:
        u = F.interpolate(u.reshape(-1, 1, u.shape[-2], u.shape[-1]),
                          size=(pde.movingmesh_grid_size[-2], pde.movingmesh_grid_size[-1]),
                          mode="bilinear", align_corners=True).squeeze(1)
    with torch.enable_grad():
        xi = torch.cat((xi1, xi2), dim=-1)
        phi = dmm_forward(dmm_sd, "array", u, xi)
        w = torch.ones(phi.shape)
        x1 = torch.autograd.grad(phi, xi1, grad_outputs=w, retain_graph=True,
                                 create_graph=True, allow_unused=True)[0] + xi1
        x2 = torch.autograd.grad(phi, xi2, grad_outputs=w, retain_graph=True,
                                 create_graph=True, allow_unused=True)[0] + xi2
    return x1.detach(), x2.detach()


class Graph:
    """The fields of the PyG Data built at data_creator_2d.py:262-267."""

    def __init__(self, x, edge_index, y, pos, batch, nbr=None):
        self.x, self.edge_index, self.y, self.pos, self.batch = x, edge_index, y, pos, batch
        self.nbr = nbr


def create_data(datapoints, steps, tw=1):
    """data_creator_2d.py:139-154."""
    data, labels = [], []
    for dp, step in zip(datapoints, steps):
        data.append(dp[step - tw:step][None])
        labels.append(dp[step:tw + step][None])
    return torch.cat(data, 0), torch.cat(labels, 0)


def create_graph(pde: PDEConst, itp_sd, data, labels, steps, dmm_sd=None, neighbors=35, tw=1,
                 mesh_override=None, dmm_grid_edge_index=None):
    """data_creator_2d.py:157-267 (connect_edge='knn').  `mesh_override` lets a
    parity test inject an externally computed moved mesh [B*N, 2] so the kNN /
    GNN stages can be compared on identical coordinates."""
    B = data.shape[0]
    moved = dmm_sd is not None or mesh_override is not None
    if len(pde.grid_size) == 3:
        ori_nx, ori_ny = data.shape[-2], data.shape[-1]
        ori_x = torch.linspace(0, pde.Lx, ori_nx)
        ori_y = torch.linspace(0, pde.Ly, ori_ny)
        ori_grid_x, ori_grid_y = torch.meshgrid(ori_x, ori_y, indexing="ij")
        mm_nx, mm_ny = pde.movingmesh_grid_size[-2], pde.movingmesh_grid_size[-1]
        nt, nx, ny = pde.grid_size
        n = nx * ny
        t = torch.linspace(pde.tmin, pde.tmax, nt)
        x = torch.linspace(0, pde.Lx, nx)
        y = torch.linspace(0, pde.Ly, ny)
        grid_x, grid_y = torch.meshgrid(x, y, indexing="ij")
        grid = torch.stack((grid_x, grid_y), 2).float()
        grid = grid.view(-1, 2)[None].repeat(B, 1, 1)
        if moved:
            if mesh_override is not None:
                mesh_x, mesh_y = mesh_override[:, [0]], mesh_override[:, [1]]
            else:
                mesh_x, mesh_y = moving_mesh(
                    dmm_sd, pde,
                    data.reshape(-1, ori_nx, ori_ny)[:, ::int(ori_nx / mm_nx), ::int(ori_ny / mm_ny)],
                    nx, ny)
            mesh = torch.cat((mesh_x, mesh_y), dim=-1).reshape(-1, nx * ny, 2)
        else:
            mesh_x, mesh_y = grid[:, :, 0].reshape(-1, 1), grid[:, :, 1].reshape(-1, 1)
            mesh = grid
        if moved:
            gx = ori_grid_x[None].repeat(B, 1, 1).reshape(-1, 1)
            gy = ori_grid_y[None].repeat(B, 1, 1).reshape(-1, 1)
            data = interpolate(itp_sd, data.reshape(-1, ori_nx, ori_ny), gx, gy, mesh_x, mesh_y,
                               mode="1").reshape(-1, tw, nx, ny)
            # data_creator_2d.py:208-209 also interpolates `labels` the same way; the
            # result only feeds graph.y, which the MM-PDE step never reads.
            labels = interpolate(itp_sd, labels.reshape(-1, ori_nx, ori_ny), gx, gy, mesh_x,
                                 mesh_y, mode="1").reshape(-1, tw, nx, ny)
    else:
        n = pde.ori_grid_size[1]
        grid = pde.ori_grid[None].repeat(B, 1, 1)
        grid_x, grid_y = grid[:, :, 0], grid[:, :, 1]
        nt = pde.grid_size[0]
        t = torch.linspace(pde.tmin, pde.tmax, nt)
        if moved:
            if mesh_override is not None:
                mesh_x, mesh_y = mesh_override[:, [0]], mesh_override[:, [1]]
            else:
                mesh_x, mesh_y = moving_mesh_tri(dmm_sd, data.reshape(-1, n), grid_x, grid_y,
                                                 pde.ori_grid,
                                                 grid_edge_index=dmm_grid_edge_index)
            mesh = torch.cat((mesh_x, mesh_y), dim=-1).reshape(-1, n, 2)
        else:
            mesh = grid
    # per-trajectory node tensors, data_creator_2d.py:242-254
    u_new, x_new, y_new, t_new = [], [], [], []
    for b in range(B):
        u_new.append(torch.transpose(torch.cat([d.reshape(-1, n) for d in data[b]]), 0, 1))
        y_new.append(torch.transpose(torch.cat([l.reshape(-1, n) for l in labels[b]]), 0, 1))
        x_new.append(mesh[b])
        t_new.append(torch.ones(n) * t[steps[b]])
    u_new = torch.cat(u_new)
    x_new = torch.cat(x_new)
    y_new = torch.cat(y_new)
    t_new = torch.cat(t_new)
    batch = torch.arange(B).repeat_interleave(n)
    edge_index, nbr, _ = knn_graph(x_new, neighbors, B)      # data_creator_2d.py:260
    pos = torch.cat((t_new[:, None], x_new), 1)
    return Graph(u_new, edge_index, y_new, pos, batch, nbr=nbr)


def interpolate_pred(pde: PDEConst, itp_sd, pred, graph, data, return_idx=False):
    """data_creator_2d.py:270-305."""
    if len(pde.grid_size) == 3:
        ori_nx, ori_ny = pde.ori_grid_size[1], pde.ori_grid_size[2]
        ori_x = torch.linspace(0, pde.Lx, ori_nx)
        ori_y = torch.linspace(0, pde.Ly, ori_ny)
        ori_grid_x, ori_grid_y = torch.meshgrid(ori_x, ori_y, indexing="ij")
        nx, ny = pde.grid_size[1], pde.grid_size[2]
        nu = int(pred.shape[0] / (nx * ny))
        pg = interpolate(itp_sd, pred.reshape(-1, nx, ny), graph.pos[:, [1]], graph.pos[:, [2]],
                         ori_grid_x[None].repeat(nu, 1, 1).reshape(-1, 1),
                         ori_grid_y[None].repeat(nu, 1, 1).reshape(-1, 1), mode="2",
                         return_idx=return_idx)
        pg, idx = pg if return_idx else (pg, None)
        pred_grid = pg.reshape(-1, 1, ori_nx, ori_ny)
        out = itpnet(itp_sd, None, None, "res_cut", data=data, burgers=True
                     ).reshape(-1, 1, ori_nx, ori_ny) + pred_grid
    else:
        n = pde.ori_grid_size[1]
        nu = int(pred.shape[0] / n)
        gx, gy = pde.ori_grid[:, 0], pde.ori_grid[:, 1]
        pg = interpolate(itp_sd, pred.reshape(-1, n), graph.pos[:, [1]], graph.pos[:, [2]],
                         gx[None].repeat(nu, 1).reshape(-1, 1),
                         gy[None].repeat(nu, 1).reshape(-1, 1), mode="2", return_idx=return_idx)
        pg, idx = pg if return_idx else (pg, None)
        pred_grid = pg.reshape(-1, n)
        out = itpnet(itp_sd, None, None, "res_cut", data=data.reshape(-1, n)).reshape(-1, n) \
            + pred_grid
    if return_idx:
        return out.reshape(-1, 1), idx
    return out.reshape(-1, 1)


def mmpde_step(pde: PDEConst, sds, data, labels, steps, moving_mesh=True, mesh_override=None,
               graph_uni=None, dmm_grid_edge_index=None):
    """One MM-PDE forward step, train_helper_2d.py:174-185 (test_timestep_losses):
    pred = interpolate_pred(itp, model_b(graph), graph, data) + model(graph_uni).
    sds = dict(model=..., model_b=..., itp=..., dmm=...) state dicts."""
    with torch.no_grad():
        if moving_mesh:
            graph = create_graph(pde, sds["itp"], data, labels, steps, dmm_sd=sds["dmm"],
                                 mesh_override=mesh_override,
                                 dmm_grid_edge_index=dmm_grid_edge_index)
        if graph_uni is None:
            graph_uni = create_graph(pde, sds.get("itp"), data, labels, steps, dmm_sd=None)
        out_u = mp_pde_solver(sds["model"], pde, graph_uni.x, graph_uni.pos, graph_uni.edge_index)
        if not moving_mesh:
            return out_u, {"graph_uni": graph_uni}
        out_b = mp_pde_solver(sds["model_b"], pde, graph.x, graph.pos, graph.edge_index)
        ip = interpolate_pred(pde, sds["itp"], out_b, graph, data)
        return ip + out_u, {"graph": graph, "graph_uni": graph_uni, "out_b": out_b,
                            "out_u": out_u, "interp": ip}


def mmpde_train_loss(pde: PDEConst, sds, data, labels, steps, mesh_override=None,
                     moving_mesh=True):
    """The loss of one training iteration, train_helper_2d.py:107-121
    (training_loop_branch): graph / graph_uni built with grad enabled, model,
    model_b in train() mode, pred = interpolate_pred(itp, model_b(graph), graph,
    data) + model(graph_uni), MSELoss against the un-interpolated labels.  The
    caller backpropagates (train_helper_2d.py:126).  `sds` tensors that require
    grad receive their gradients; BatchNorm running buffers update in place."""
    graph_uni = create_graph(pde, sds.get("itp"), data, labels, steps, dmm_sd=None)
    out_u = mp_pde_solver(sds["model"], pde, graph_uni.x, graph_uni.pos, graph_uni.edge_index,
                          train=True)
    if not moving_mesh:
        return mse(out_u, labels), {"graph_uni": graph_uni, "pred": out_u}
    graph = create_graph(pde, sds["itp"], data, labels, steps, dmm_sd=sds.get("dmm"),
                         mesh_override=mesh_override)
    out_b = mp_pde_solver(sds["model_b"], pde, graph.x, graph.pos, graph.edge_index, train=True)
    pred = interpolate_pred(pde, sds["itp"], out_b, graph, data) + out_u
    return mse(pred, labels), {"graph": graph, "graph_uni": graph_uni, "pred": pred}


def mse(pred, labels):
    """mmpde.py:33-36."""
    return torch.nn.MSELoss()(pred, labels.reshape(-1, 1))


def test_timestep_losses(pde: PDEConst, sds, u, steps, moving_mesh=True, tw=1):
    """train_helper_2d.py:137-200 with the whole test set as one batch: for each
    step (mmpde.py:139, filter :167-168), create_data -> the MM-PDE step ->
    MSELoss(pred, labels) (mmpde.py:33-36).  Returns (per-step loss [S],
    per-trajectory MSE [S, B])."""
    B = u.shape[0]
    per_step, per_traj = [], []
    for s in steps:
        if s != tw and s % tw != 0:
            continue
        data, labels = create_data(u, [s] * B, tw)
        pred, _ = mmpde_step(pde, sds, data, labels, [s] * B, moving_mesh=moving_mesh)
        per_step.append(mse(pred, labels))
        d = pred.reshape(B, -1) - labels.reshape(B, -1)
        per_traj.append((d * d).mean(1))
    return torch.stack(per_step), torch.stack(per_traj)
