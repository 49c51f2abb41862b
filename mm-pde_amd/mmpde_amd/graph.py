"""Minimal stand-in for the PyG ``Data`` object the reference builds at
data_creator_2d.py:262-267 (PyG is not a dependency of this engine).

Fields the reference sets and the models read: ``x`` [n, tw], ``pos`` [n, 3] =
(t, x, y), ``edge_index`` int64 [2, n*k] (row 0 source, row 1 target), ``batch``
int64 [n] and ``y`` [n, tw].  The engine adds ``nbr`` -- the same graph as an
int32 target-major [n, k] table, which is what the HIP kernels consume, and
``seg_n`` -- the nodes per trajectory (every batch segment has that many; no
edge leaves its segment).  Any
object with the PyG fields (including a real ``torch_geometric.data.Data``) is
accepted by the models; ``nbr`` is then derived from ``edge_index``.
"""
from __future__ import annotations

import torch


class Data:
    def __init__(self, x=None, edge_index=None, **kwargs):
        self.x = x
        self._edge_index = edge_index
        self.y = None
        self.pos = None
        self.batch = None
        self.nbr = None
        self.nbr_checked = False  # nbr built by the engine's graph kernels (sources in range)
        self.deg = None   # ragged graphs (radius): in-degree per target, nbr rows padded
        self.seg_n = None  # nodes per trajectory (batch segment), when all are equal
        for k, v in kwargs.items():
            setattr(self, k, v)

    @property
    def edge_index(self):
        """PyG edge_index, materialised lazily from ``nbr`` (int64 widening kernel)."""
        if self._edge_index is None and self.nbr is not None:
            from .ops import edge_index_from_nbr
            self._edge_index = edge_index_from_nbr(self.nbr, self.deg)
        return self._edge_index

    @edge_index.setter
    def edge_index(self, v):
        self._edge_index = v

    @property
    def num_nodes(self):
        return None if self.x is None else self.x.shape[0]

    def to(self, device):
        for k in ("x", "_edge_index", "y", "pos", "batch", "nbr", "deg"):
            v = getattr(self, k)
            if isinstance(v, torch.Tensor):
                setattr(self, k, v.to(device))
        return self

    def __repr__(self):
        parts = []
        for k in ("x", "edge_index", "y", "pos", "batch", "nbr"):
            v = self._edge_index if k == "edge_index" else getattr(self, k)
            if isinstance(v, torch.Tensor):
                parts.append(f"{k}={list(v.shape)}")
        return f"Data({', '.join(parts)})"
