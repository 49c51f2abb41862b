"""PDE descriptors: same class names, constructor arguments and attributes as
the reference (PDEs.py:9-67) -- tmin/tmax, Lx/Ly, the three grid sizes, dt and
(cy) the fixed mesh ``ori_grid``.  Pure constants, read by the models and the
GraphCreator.

Note the reference computes ``dt`` from the grid size passed to the
constructor (defaults: burgers (31, 96, 96) -> dt = 1.0, cy (30, 2521) ->
dt = 0.1) and ``mmpde.main`` later overwrites the grid sizes with
--base_resolution without touching dt; the same happens here.
"""
from __future__ import annotations

from torch import nn

_DEFAULTS = {
    # name: (tmin, tmax, default grid, separate movingmesh/ori defaults)
    "burgers": (0, 30, (31, 96, 96)),
    "cy": (0, 2.9, (30, 2521)),
}


class PDE(nn.Module):
    """Generic PDE template (PDEs.py:9-17)."""

    def __init__(self):
        super().__init__()

    def __repr__(self):
        return "PDE"

    def _setup(self, kind, tmin, tmax, grid_size, L, device):
        t0, t1, g = _DEFAULTS[kind]
        self.tmin = t0 if tmin is None else tmin
        self.tmax = t1 if tmax is None else tmax
        self.Lx = self.Ly = 1 if L is None else L
        self.grid_size = g if grid_size is None else grid_size
        self.dt = self.tmax / (self.grid_size[0] - 1)
        self.device = device


class burgers(PDE):  # noqa: N801 - reference class name
    """2-D Burgers' equation on [0, L]^2, t in [0, 30] (PDEs.py:20-41)."""

    def __init__(self, tmin=None, tmax=None, grid_size=None, L=None, flux_splitting=None,
                 device="cpu"):
        super().__init__()
        self._setup("burgers", tmin, tmax, grid_size, L, device)
        # the reference keeps these at the default regardless of grid_size
        self.movingmesh_grid_size = _DEFAULTS["burgers"][2]
        self.ori_grid_size = _DEFAULTS["burgers"][2]


class cy(PDE):  # noqa: N801 - reference class name
    """Flow past a cylinder on a fixed unstructured mesh (PDEs.py:44-67)."""

    def __init__(self, tmin=None, tmax=None, grid_size=None, ori_grid=None, L=None,
                 flux_splitting=None, device="cpu"):
        super().__init__()
        self._setup("cy", tmin, tmax, grid_size, L, device)
        self.ori_grid_size = self.grid_size
        self.movingmesh_grid_size = self.grid_size
        self.ori_grid = ori_grid
