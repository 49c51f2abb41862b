"""Regenerate the committed golden fixtures (run from the repo root):

    python tests/golden/make_golden.py

* sklearn_knn30.npz -- scikit-learn (1.7.2 here; the reference pins 1.3.0,
  env.yml:135) NearestNeighbors(30).fit(src).kneighbors(qry) on tie-free random
  inputs, per trajectory: the independent pin of the kNN-30 restatement
  (reference data_creator_2d.py:66-78).
* knn35_lattice.npz -- kNN-35 graph of an integer lattice (exact fp32
  distances, heavy ties) computed with exact integer arithmetic in pure Python
  under the (d2, index) rule of torch_cluster's insertion sort: a hand KAT for
  the knn_graph restatement (data_creator_2d.py:260).
* gnn_small.npz -- the oracle's MP_PDE_Solver_2D output for a small seeded case
  (regression pin of the restatement itself; weights are rebuilt from the seed
  by mmpde_amd.synth.build_models, as in tests/test_golden.py).

No reference code is imported or executed here.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mm-pde_amd")]


def sklearn_knn30():
    from sklearn.neighbors import NearestNeighbors

    rng = np.random.default_rng(7)
    B, ns, nq = 2, 257, 131
    src = rng.random((B, ns, 2), dtype=np.float64).astype(np.float32)
    qry = rng.random((B, nq, 2), dtype=np.float64).astype(np.float32)
    qry[:, :5] = src[:, 10:15]          # queries that coincide with a source point
    idx = np.empty((B, nq, 30), dtype=np.int64)
    dist = np.empty((B, nq, 30), dtype=np.float64)
    for b in range(B):
        nn_ = NearestNeighbors(n_neighbors=30).fit(src[b])
        d, i = nn_.kneighbors(qry[b])
        idx[b], dist[b] = i, d
    # tie-free check: consecutive neighbour distances differ
    assert np.all(np.diff(dist, axis=-1) > 0)
    np.savez_compressed(os.path.join(HERE, "sklearn_knn30.npz"), src=src, qry=qry, idx=idx,
                        dist=dist)


def lattice_knn35():
    s = 12
    pts = [(float(i), float(j)) for i in range(s) for j in range(s)]
    n, k = len(pts), 35
    nbr = np.empty((n, k), dtype=np.int64)
    for q in range(n):
        qx, qy = pts[q]
        cand = sorted(((int((px - qx) ** 2 + (py - qy) ** 2), j) for j, (px, py) in enumerate(pts)))
        cand = cand[:k + 1]
        nbr[q] = [j for _, j in cand if j != q][:k]
    np.savez_compressed(os.path.join(HERE, "knn35_lattice.npz"),
                        pos=np.asarray(pts, dtype=np.float32), nbr=nbr)


def gnn_small():
    from mmpde_amd.synth import build_models
    from oracle import refcpu

    torch.manual_seed(3)
    pde, model, _, _, _, _ = build_models("cy", grid=torch.rand(64, 2), moving_mesh=False)
    B, n = 2, 64
    pos_xy = pde.ori_grid.repeat(B, 1)
    u = torch.randn(B * n, 1)
    t = torch.full((B * n, 1), 0.7)
    pos = torch.cat((t, pos_xy), 1)
    ei, _, _ = refcpu.knn_graph(pos_xy, 35, B)
    sd = {k: v.detach() for k, v in model.state_dict().items()}
    opde = refcpu.PDEConst("cy", [30, n], ori_grid=pde.ori_grid)
    out = refcpu.mp_pde_solver(sd, opde, u, pos, ei)
    np.savez_compressed(os.path.join(HERE, "gnn_small.npz"), u=u.numpy(), pos=pos.numpy(),
                        edge_index=ei.numpy(), out=out.numpy())


if __name__ == "__main__":
    sklearn_knn30()
    lattice_knn35()
    gnn_small()
    print("fixtures written to", HERE)
