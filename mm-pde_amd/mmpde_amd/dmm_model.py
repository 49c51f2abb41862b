"""DMM mesh mover on the HIP kernels (drop-in for reference mesh/dmm_model.py).

Module tree and ``state_dict`` keys match the reference (including the unused
``DenseNet.fc0``, which also keeps the default-init RNG stream aligned), so
the reference checkpoints ``cy_checkpoint`` / ``burgers_checkpoint``
(``model_state_dict``) load unchanged.  Unlike the reference, nothing is
hard-wired to ``device="cuda"`` at construction (dmm_model.py:27-28).

The MM-PDE step never needs phi itself, only the moved mesh
x = xi + d(phi)/d(xi) that GraphCreator_FS_2D.moving_mesh[_tri] obtains with
two autograd.grad calls (data_creator_2d.py:106-107,130-131).  ``DMM.mesh``
returns exactly that through an analytic vector-Jacobian product
(mmpde_dmm_mesh_graph / mmpde_dmm_mesh_array; derivation in dmm.hip).
``DMM.forward`` (phi, and rf=True's second output) runs the branch and the
head on the same kernels (mmpde_dmm_branch_*, mmpde_dmm_phi); ``DenseNet`` /
``ConvNet`` forwards run on the skinny-linear and conv kernels.

In ``train()`` mode (DMM training, reference mesh/dmm_utils.py:391-1095,
SURVEY.md §8(f) row 4: ``mmpde_amd.dmm_train``) every forward is the
reference's computation as differentiable device torch ops -- BatchNorm on
batch statistics, twice differentiable in the grid (the Monge-Ampere loss
takes d2 phi / d xi2 through autograd) -- with the fixed grid's kNN-35 graph
from the HIP kernel and the mean aggregation over its fixed in-degree.
"""
from __future__ import annotations

import ctypes

import torch
from torch import nn

from . import _lib as L
from .gnn_2d import BatchNorm
from . import ops
from .ops import knn_graph_nbr




class DenseNet(nn.Module):
    """Reference dmm_model.py:9-45 (normalize=False): Linear layers with tanh on
    all but the last.  ``fc0`` is unused by the reference forward but is a
    parameter there, so it is kept for state_dict / RNG parity."""

    def __init__(self, layers, width=32, normalize=False):
        super().__init__()
        if normalize:
            raise NotImplementedError("DenseNet(normalize=True) is not used by MM-PDE")
        self.n_layers = len(layers) - 1
        assert self.n_layers >= 1
        self.layers = nn.ModuleList(nn.Linear(a, b) for a, b in zip(layers[:-1], layers[1:]))
        self.normalize = normalize
        self.width = width
        self.fc0 = nn.Linear(4, width)

    def forward(self, x):
        """dmm_model.py:31-45 (normalize=False): (out, x) with x the last hidden
        activation (the input of the last Linear)."""
        if self.training:   # differentiable torch ops (DMM training)
            for i, l in enumerate(self.layers):
                if i != self.n_layers - 1:
                    x = torch.tanh(l(x))
                else:
                    out = l(x)
            return out, x
        for i, l in enumerate(self.layers):
            if i != self.n_layers - 1:
                x = ops.linear_rows(x, l.weight, l.bias, L.ACT_TANH)
            else:
                out = ops.linear_rows(x, l.weight, l.bias, L.ACT_NONE)
        return out, x


class ConvNet(nn.Module):
    """Reference dmm_model.py:48-81 (layers == 7, the only configuration it builds)."""

    def __init__(self, s, layers):
        super().__init__()
        if layers != 7:
            raise NotImplementedError("ConvNet is only defined for layers == 7")
        self.layers = nn.ModuleList([
            nn.Conv2d(1, 8, 5, stride=2, padding=2), nn.Conv2d(8, 16, 5, padding=2),
            nn.Conv2d(16, 8, 5, padding=2), nn.Conv2d(8, 1, 5, stride=2, padding=2)])
        self.fc1 = None
        self.fc2 = nn.Linear(int(((s + 1) / 2 + 1) / 2) ** 2, 1024)
        self.fc3 = nn.Linear(1024, 512)
        self.s = s

    def forward(self, x):
        """dmm_model.py:65-81: x [B, 1, s, s] -> [B, 512]."""
        c = self.layers
        if self.training:   # differentiable torch ops (DMM training)
            x1 = torch.tanh(c[0](x))
            x3 = torch.tanh(x1 + c[2](torch.tanh(c[1](x1))))
            f = torch.flatten(torch.tanh(c[3](x3)), 1)
            return self.fc3(torch.tanh(self.fc2(f)))
        x1 = ops.conv2d(x, c[0].weight, c[0].bias, 2, 2, L.ACT_TANH)
        x2 = ops.conv2d(x1, c[1].weight, c[1].bias, 1, 2, L.ACT_TANH)
        x3 = ops.conv2d(x2, c[2].weight, c[2].bias, 1, 2, L.ACT_TANH, residual=x1)
        x4 = ops.conv2d(x3, c[3].weight, c[3].bias, 2, 2, L.ACT_TANH)
        f = torch.flatten(x4, 1)
        f = ops.linear_rows(f, self.fc2.weight, self.fc2.bias, L.ACT_TANH)
        return ops.linear_rows(f, self.fc3.weight, self.fc3.bias, L.ACT_NONE)


class GNN_Layer_FS_2D(nn.Module):  # noqa: N801 - reference name
    """The DMM branch's tanh GNN layer (reference dmm_model.py:94-142)."""

    def __init__(self, in_features, out_features, hidden_features):
        super().__init__()
        self.message_net_1 = nn.Sequential(nn.Linear(2 * in_features + 3, hidden_features),
                                           nn.Tanh())
        self.message_net_2 = nn.Sequential(nn.Linear(hidden_features, out_features), nn.Tanh())
        self.update_net_1 = nn.Sequential(nn.Linear(in_features + hidden_features,
                                                    hidden_features), nn.Tanh())
        self.update_net_2 = nn.Sequential(nn.Linear(hidden_features, out_features), nn.Tanh())
        self.norm = BatchNorm(hidden_features)

    def forward(self, x, u, pos_x, pos_y, nbr):
        """Training-mode layer (dmm_model.py:126-142) as differentiable torch ops:
        tanh messages cat(x_i, x_j, u_i - u_j, dx, dy) over the target-major
        neighbour table nbr [n, k] (every row k sources: PyG's mean is the mean
        over them), update x + U2 tanh(U1 cat(x, m)), BatchNorm.  The eval
        forward runs inside mmpde_dmm_mesh_graph."""
        n, k = nbr.shape
        j = nbr.reshape(-1).long()
        i = torch.arange(n, device=x.device).repeat_interleave(k)
        m = torch.cat((x[i], x[j], u[i] - u[j], pos_x[i] - pos_x[j], pos_y[i] - pos_y[j]), dim=-1)
        m = self.message_net_2(self.message_net_1(m)).reshape(n, k, -1).mean(1)
        return self.norm(x + self.update_net_2(self.update_net_1(torch.cat((x, m), dim=-1))))


class DMM(nn.Module):
    """Reference dmm_model.py:145-219."""

    def __init__(self, branch_layer, trunk_layer, grid=None, out_layer=None, s=None,
                 mode="array"):
        super().__init__()
        self.mode = mode
        self.ori_grid = grid
        if mode == "array":
            self.branch = ConvNet(s, branch_layer)
            self.trunk = DenseNet(trunk_layer)
            self.out_nn = DenseNet(out_layer)
        elif mode == "graph":
            self.hidden_features = branch_layer[0]
            self.hidden_layer = branch_layer[1]
            self.gnn_layers = nn.ModuleList(
                GNN_Layer_FS_2D(in_features=self.hidden_features,
                                hidden_features=self.hidden_features,
                                out_features=self.hidden_features)
                for _ in range(self.hidden_layer))
            self.embedding_mlp = nn.Sequential(
                nn.Linear(3, self.hidden_features), nn.BatchNorm1d(self.hidden_features),
                nn.Tanh(), nn.Linear(self.hidden_features, self.hidden_features),
                nn.BatchNorm1d(self.hidden_features))
            self.decoding_mlp = DenseNet([self.hidden_features, 128, 1])
            self.output_mlp = nn.Sequential(
                nn.Linear(grid.shape[0], 512), nn.Tanh(), nn.Linear(512, 256), nn.Tanh(),
                nn.Linear(256, trunk_layer[-1]))
            self.trunk = DenseNet(trunk_layer)
            self.out_nn = DenseNet(out_layer)
        else:
            raise ValueError(mode)
        self._pack_key = None
        self._pack = None
        self._grid_cache = {}

    def forward(self, u, grid, rf=False):
        """dmm_model.py:185-219: phi = out_nn(cat(branch(u), trunk(grid))), the
        branch of trajectory b repeated over its grid.shape[0] / B rows of grid.
        u: graph [B, N] (values on self.ori_grid), array [B, s, s]; grid [B*m, 2].
        Returns phi [B*m, 1], or (phi, second_out [B*m, L'], ones [B*m*L', 1])
        with rf=True."""
        L.require_device(u, grid)
        if self.training:
            return self._forward_train(u, grid, rf)
        bp, hd = self.device_params()
        u = L.f32c(u)
        grid = L.f32c(grid).reshape(-1, 2)
        B, ng = u.shape[0], grid.shape[0]
        if ng % B:
            raise ValueError("grid rows must be a multiple of the batch size")
        lib = L.lib()
        st = L.stream(u.device)
        branch = torch.empty((B, hd.latent), dtype=torch.float32, device=u.device)
        if self.mode == "graph":
            og = L.f32c(torch.as_tensor(self.ori_grid).to(u.device)).reshape(-1, 2)
            N = og.shape[0]
            nbr = self.grid_nbr(og)
            ws = torch.empty((lib.mmpde_dmm_workspace_bytes(B, N, hd.latent, hd.hidden) // 4,),
                             dtype=torch.float32, device=u.device)
            L.check(lib.mmpde_dmm_branch_graph(L.ptr(u), L.ptr(og), B, N, L.ptr(nbr), nbr.shape[1],
                                               ctypes.byref(bp), ctypes.byref(hd), L.ptr(ws),
                                               L.ptr(branch), st), "mmpde_dmm_branch_graph")
        else:
            s = self.branch.s
            ws = torch.empty((lib.mmpde_dmm_workspace_bytes(B, s * s, hd.latent, hd.hidden) // 4,),
                             dtype=torch.float32, device=u.device)
            L.check(lib.mmpde_dmm_branch_array(L.ptr(u), B, ctypes.byref(bp), ctypes.byref(hd),
                                               L.ptr(ws), L.ptr(branch), st), "mmpde_dmm_branch_array")
        nb = lib.mmpde_dmm_phi_workspace_bytes(B, ng, hd.latent, hd.hidden, hd.th)
        ws2 = torch.empty((nb // 4,), dtype=torch.float32, device=u.device)
        phi = torch.empty((ng, 1), dtype=torch.float32, device=u.device)
        second = (torch.empty((ng, hd.hidden), dtype=torch.float32, device=u.device)
                  if rf else None)
        ob = self.out_nn.layers[1].bias
        L.check(lib.mmpde_dmm_phi(L.ptr(branch), B, L.ptr(grid), ng, ctypes.byref(hd),
                                  L.ptr(L.f32c(ob)) if ob is not None else None, L.ptr(ws2),
                                  L.ptr(phi), L.ptr(second), st), "mmpde_dmm_phi")
        if not rf:
            return phi
        return phi, second, torch.ones_like(second).reshape(-1, 1)

    def _forward_train(self, u, grid, rf=False):
        """dmm_model.py:185-219 in train() mode: differentiable in the weights and
        in `grid` (to any order), BatchNorm on batch statistics."""
        B = u.shape[0]
        if grid.shape[0] % B:
            raise ValueError("grid rows must be a multiple of the batch size")
        if self.mode == "array":
            branch = self.branch(u.unsqueeze(1))
        else:
            og = torch.as_tensor(self.ori_grid).to(u.device, torch.float32).reshape(-1, 2)
            N = og.shape[0]
            nbr = self.grid_nbr(og.contiguous())                       # [N, 35] local
            gnbr = (nbr[None].long() + N * torch.arange(B, device=u.device)[:, None, None])
            gnbr = gnbr.reshape(B * N, -1)
            x = u.reshape(-1, 1)
            pos = og[None].expand(B, N, 2).reshape(-1, 2)
            pos_x, pos_y = pos[:, :1], pos[:, 1:]
            h = self.embedding_mlp(torch.cat((x, pos_x, pos_y), -1))
            for layer in self.gnn_layers:
                h = layer(h, x, pos_x, pos_y, gnbr)
            h, _ = self.decoding_mlp(h)
            branch = self.output_mlp(h.reshape(B, -1))
        rep = grid.shape[0] // B
        branch = branch[:, None, :].expand(B, rep, branch.shape[-1]).reshape(-1, branch.shape[-1])
        trunk, _ = self.trunk(grid)
        out, second = self.out_nn(torch.cat((branch, trunk.reshape(-1, branch.shape[-1])), dim=-1))
        if not rf:
            return out
        return out, second, torch.ones_like(second).reshape(-1, 1)

    # ----------------------------------------------------------------- packing
    def _check(self):
        if self.training:
            raise NotImplementedError("the HIP head is eval-mode: call .eval() (train() "
                                      "mode runs DMM.forward as torch ops)")
        tl = self.trunk.layers
        ol = self.out_nn.layers
        if len(tl) != 2 or len(ol) != 2 or ol[1].out_features != 1:
            raise NotImplementedError("trunk DenseNet[2, th, L] / out_nn DenseNet[2L, L', 1] only")
        if self.mode == "graph" and (self.hidden_features != 4 or self.hidden_layer > 3):
            raise NotImplementedError("graph branch: hidden 4, <= 3 layers (cy checkpoint)")

    def _tensors(self):
        tl, ol = self.trunk.layers, self.out_nn.layers
        head = [tl[0].weight, tl[0].bias, tl[1].weight, tl[1].bias, ol[0].weight, ol[0].bias,
                ol[1].weight]
        if self.mode == "graph":
            e = self.embedding_mlp
            br = [e[0].weight, e[0].bias, e[1].weight, e[1].bias, e[1].running_mean,
                  e[1].running_var, e[3].weight, e[3].bias, e[4].weight, e[4].bias,
                  e[4].running_mean, e[4].running_var]
            for g in self.gnn_layers:
                br += [g.message_net_1[0].weight, g.message_net_1[0].bias,
                       g.message_net_2[0].weight, g.message_net_2[0].bias,
                       g.update_net_1[0].weight, g.update_net_1[0].bias,
                       g.update_net_2[0].weight, g.update_net_2[0].bias,
                       g.norm.module.weight, g.norm.module.bias, g.norm.module.running_mean,
                       g.norm.module.running_var]
            d, o = self.decoding_mlp.layers, self.output_mlp
            br += [d[0].weight, d[0].bias, d[1].weight, d[1].bias, o[0].weight, o[0].bias,
                   o[2].weight, o[2].bias, o[4].weight, o[4].bias]
        else:
            b = self.branch
            br = [b.layers[0].weight, b.layers[0].bias, b.layers[1].weight, b.layers[1].bias,
                  b.layers[2].weight, b.layers[2].bias, b.layers[3].weight, b.layers[3].bias,
                  b.fc2.weight, b.fc2.bias, b.fc3.weight, b.fc3.bias]
        return head, br

    def device_params(self):
        self._check()
        head, br = self._tensors()
        key = tuple((t.data_ptr(), t._version) for t in head + br)
        if key == self._pack_key:
            return self._pack[0]
        fh = [L.f32c(t) for t in head]
        fb = [L.f32c(t) for t in br]
        tl, ol = self.trunk.layers, self.out_nn.layers
        hd = L.DmmHead(fh[0].data_ptr(), fh[1].data_ptr(), fh[2].data_ptr(), fh[3].data_ptr(),
                       tl[0].out_features, tl[1].out_features, fh[4].data_ptr(),
                       fh[5].data_ptr(), fh[6].data_ptr(), ol[0].out_features)
        if self.mode == "graph":
            p = [t.data_ptr() for t in fb]
            nl = self.hidden_layer
            per = [p[12 + 12 * i: 24 + 12 * i] for i in range(nl)]
            arrs = []
            for fld in range(12):
                vals = [per[i][fld] if i < nl else None for i in range(3)]
                arrs.append(L._P3(*vals))
            tail = p[12 + 12 * nl:]
            bn_eps = float(self.embedding_mlp[1].eps)
            bp = L.DmmGraphBranch(*p[:12], *arrs, nl, *tail, bn_eps)
        else:
            bp = L.DmmArrayBranch(*[t.data_ptr() for t in fb], self.branch.s)
        self._pack = ((bp, hd), fh + fb)
        self._pack_key = key
        return self._pack[0]

    def grid_nbr(self, grid: torch.Tensor, k: int = 35) -> torch.Tensor:
        """kNN-35 table of the fixed grid (reference dmm_model.py:222-234 builds it
        every call on B identical copies; it depends only on the grid, so it is
        built once per grid here).  LOCAL indices [N, k] int32."""
        # the entry holds the grid tensor itself, so its storage cannot be freed
        # and reused by another grid while the entry lives: (address, version,
        # shape) then identifies the content
        key = (grid.data_ptr(), grid._version, tuple(grid.shape), str(grid.device), k)
        hit = self._grid_cache.get(key)
        if hit is None:
            hit = (grid, knn_graph_nbr(grid, 1, k))
            self._grid_cache = {key: hit}
        return hit[1]

    # ----------------------------------------------------------------- the API
    def head_cache(self, xi: torch.Tensor, workspace: torch.Tensor | None = None) -> torch.Tensor:
        """The grid side of the head (trunk(xi), Q, J = dQ/dxi): a function of xi
        and the weights only, prepared once for a rollout over a fixed grid and
        passed to mesh(..., head_cache=).  Recompute it after changing weights."""
        L.require_device(xi)
        _, hd = self.device_params()
        xi = L.f32c(xi).reshape(-1, 2)
        N = xi.shape[0]
        if workspace is None:
            nb = L.lib().mmpde_dmm_workspace_bytes(1, N, hd.latent, hd.hidden)
            workspace = torch.empty((nb // 4,), dtype=torch.float32, device=xi.device)
        cache = torch.empty((L.lib().mmpde_dmm_head_cache_bytes(N, hd.hidden) // 4,),
                            dtype=torch.float32, device=xi.device)
        L.check(L.lib().mmpde_dmm_head_prepare(L.ptr(xi), N, ctypes.byref(hd), L.ptr(workspace),
                                               L.ptr(cache), L.stream(xi.device)),
                "mmpde_dmm_head_prepare")
        return cache

    def mesh(self, u: torch.Tensor, xi: torch.Tensor, out: torch.Tensor | None = None,
             workspace: torch.Tensor | None = None,
             head_cache: torch.Tensor | None = None) -> torch.Tensor:
        """Moved mesh x = xi + d(phi)/d(xi) for every trajectory.
        u: graph mode [B, N] (values on the fixed grid), array mode [B, s, s];
        xi: [N, 2] grid shared by all trajectories (graph: self.ori_grid;
        array: the np.meshgrid 'xy' grid of data_creator_2d.py:94-100);
        head_cache: head_cache(xi) of the same xi and weights, or None.
        Returns [B*N, 2] fp32."""
        L.require_device(u, xi)
        bp, hd = self.device_params()
        u = L.f32c(u)
        xi = L.f32c(xi).reshape(-1, 2)
        B, N = u.shape[0], xi.shape[0]
        if workspace is None:
            ne = N if self.mode == "graph" else max(N, self.branch.s ** 2)  # array: xi may be coarser
            nb = L.lib().mmpde_dmm_workspace_bytes(B, ne, hd.latent, hd.hidden)
            workspace = torch.empty((nb // 4,), dtype=torch.float32, device=u.device)
        if out is None:
            out = torch.empty((B * N, 2), dtype=torch.float32, device=u.device)
        if head_cache is not None:
            L.require_device(head_cache)
            if head_cache.numel() * 4 < L.lib().mmpde_dmm_head_cache_bytes(N, hd.hidden):
                raise ValueError("head_cache is smaller than mmpde_dmm_head_cache_bytes")
        hc = L.ptr(head_cache) if head_cache is not None else None
        st = L.stream(u.device)
        if self.mode == "graph":
            nbr = self.grid_nbr(xi)
            L.check(L.lib().mmpde_dmm_mesh_graph_cached(
                L.ptr(u), L.ptr(xi), B, N, L.ptr(nbr), nbr.shape[1], ctypes.byref(bp),
                ctypes.byref(hd), hc, L.ptr(workspace), L.ptr(out), st), "mmpde_dmm_mesh_graph")
        else:
            L.check(L.lib().mmpde_dmm_mesh_array_cached(
                L.ptr(u), L.ptr(xi), B, N, ctypes.byref(bp), ctypes.byref(hd), hc,
                L.ptr(workspace), L.ptr(out), st), "mmpde_dmm_mesh_array")
        return out
