"""Synthetic inputs for the benchmark and the parity tests.

The reference's datasets (mesh/data/cylinder_rot_tri, burgers_192.npy) and DMM
checkpoints are not available offline, so every input is synthetic and seeded:

* ``cy_synth_mesh``: 2521 points uniform in [0,1]^2 outside the disk of centre
  (0.25, 0.5) and radius 0.05 (a cylinder wake domain), from
  ``torch.Generator().manual_seed(0)`` -- general position, so no distance ties.
  A copy ships as ``data/cy_synth_mesh.npy`` and is what the engine loads.
* ``fields``: u(b, t, x, y) = sin(2 pi (x + phi_b + 0.02 t)) cos(2 pi y) + 0.05 N(0, 1).
* ``build_models``: reference architectures constructed in the reference's
  order under ``torch.manual_seed(seed)`` (default PyTorch init), BatchNorm
  statistics/affines randomised so eval-mode BN is exercised.  With default
  init the DMM already moves mesh points by O(1e-2) (about half the cylinder
  mesh spacing), so its ``out_nn`` is left unscaled (``dmm_scale``).
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")


def generate_cy_mesh(n=2521, seed=0):
    g = torch.Generator().manual_seed(seed)
    pts = []
    have = 0
    while have < n:
        p = torch.rand((4 * n, 2), generator=g)
        keep = ((p[:, 0] - 0.25) ** 2 + (p[:, 1] - 0.5) ** 2) > 0.05 ** 2
        p = p[keep]
        pts.append(p)
        have += p.shape[0]
    return torch.cat(pts)[:n].contiguous()


def cy_synth_mesh() -> torch.Tensor:
    """The committed 2521 x 2 fp32 fixture (regenerated if missing)."""
    path = os.path.join(_DATA, "cy_synth_mesh.npy")
    if os.path.exists(path):
        return torch.from_numpy(np.load(path)).float()
    return generate_cy_mesh()


def burgers_grid_points(s=48):
    """Uniform 'ij' grid of the Burgers solution (data_creator_2d.py:187-194)."""
    x = torch.linspace(0, 1, s)
    gx, gy = torch.meshgrid(x, x, indexing="ij")
    return torch.stack((gx, gy), 2).reshape(-1, 2)


def fields(points: torch.Tensor, batches: int, t_len: int, seed=1) -> torch.Tensor:
    """u [batches, t_len, N] on the given points."""
    g = torch.Generator().manual_seed(seed)
    phi = torch.rand((batches, 1, 1), generator=g)
    t = torch.arange(t_len, dtype=torch.float32)[None, :, None]
    x = points[:, 0][None, None, :]
    y = points[:, 1][None, None, :]
    u = torch.sin(2 * math.pi * (x + phi + 0.02 * t)) * torch.cos(2 * math.pi * y)
    u = u + 0.05 * torch.randn(u.shape, generator=g)
    return u.float().contiguous()


def _randomise_bn(module: torch.nn.Module, g: torch.Generator):
    for m in module.modules():
        if isinstance(m, torch.nn.BatchNorm1d):
            c = m.num_features
            with torch.no_grad():
                m.running_mean.copy_(0.1 * torch.randn(c, generator=g))
                m.running_var.copy_(0.5 + torch.rand(c, generator=g))
                m.weight.copy_(0.8 + 0.4 * torch.rand(c, generator=g))
                m.bias.copy_(0.1 * torch.randn(c, generator=g))


def build_models(kind: str, grid: torch.Tensor | None = None, seed: int = 0,
                 moving_mesh: bool = True, dmm_scale: float = 1.0):
    """Construct (pde, model, model_b, itp, dmm, graph_creator) exactly as
    mmpde.main does (mmpde.py:161-253) with the README's DMM settings:
    cy: --base_resolution 30,2521, DMM(graph, branch 4,3, trunk [2,16,512],
    out [1024,512,1]); burgers: base_resolution 31,48,48, DMM(array, s=48,
    branch 7, trunk [2,32,512])."""
    from .data_creator_2d import GraphCreator_FS_2D
    from .dmm_model import DMM
    from .gnn_2d import MP_PDE_Solver_2D
    from .interpolate import ItpNet
    from .pdes import burgers, cy

    torch.manual_seed(seed)
    if kind == "cy":
        grid = cy_synth_mesh() if grid is None else grid
        pde = cy(ori_grid=grid)
        res = [30, grid.shape[0]]
    elif kind == "burgers":
        pde = burgers()
        res = [31, 48, 48]
    else:
        raise ValueError(kind)
    pde.grid_size = res
    pde.movingmesh_grid_size = res
    pde.ori_grid_size = res
    itp = dmm = model_b = None
    if moving_mesh:
        if kind == "cy":
            itp = ItpNet(res[1], None, [128, 64], [128, 64], [1, 4, 16, 4, 1])
            dmm = DMM(mode="graph", grid=grid, branch_layer=[4, 3], trunk_layer=[2, 16, 512],
                      out_layer=[1024, 512, 1])
        else:
            itp = ItpNet(res[-2], res[-1], [128, 64], [128, 64], [1, 4, 16, 4, 1])
            dmm = DMM(s=48, mode="array", branch_layer=7, trunk_layer=[2, 32, 512],
                      out_layer=[1024, 512, 1])
    gc = GraphCreator_FS_2D(pde=pde, neighbors=35, connect_edge="knn", time_window=1,
                            t_resolution=res[0])
    model = MP_PDE_Solver_2D(pde=pde, time_window=1, eq_variables={})
    if moving_mesh:
        model_b = MP_PDE_Solver_2D(pde=pde, time_window=1, eq_variables={})
    g = torch.Generator().manual_seed(seed + 1000)
    for m in (model, model_b, dmm):
        if m is not None:
            _randomise_bn(m, g)
    if dmm is not None and dmm_scale != 1.0:
        with torch.no_grad():
            dmm.out_nn.layers[-1].weight.mul_(dmm_scale)
    for m in (model, model_b, itp, dmm):
        if m is not None:
            m.eval()
    return pde, model, model_b, itp, dmm, gc
