"""Exact-tie exposure of the kNN-30 query (sklearn kneighbors replacement,
reference data_creator_2d.py:66-78, :75-76).

On exact fp64 distance ties sklearn's order is its KD-tree's traversal order,
which the engine does not reproduce (it takes ties in index order, DESIGN.md
§2): those queries are where parity with the reference is unpinned.  The
query kernels count them (include/mmpde_hip.h mmpde_knn_query `ties`): a query
counts when its sorted fp64 keys hold an equal pair inside the first k or
between ranks k-1 and k.  The expected counts here are computed in numpy from
the same fp64 keys (dx*dx + dy*dy of the fp32 coordinates, no fma) over every
source point -- an independent brute force, not the kernels' candidate lists.

Bars: counts exact; the index maps stay bit-exact against the C oracle.
"""
import numpy as np
import pytest
import torch

from oracle import refcpu

pytestmark = pytest.mark.gpu


def tie_queries(src, qry, B, k=30):
    """Number of queries whose sorted fp64 distances tie inside the first k
    or at rank k (numpy brute force)."""
    s = src.double().numpy().reshape(B, -1, 2)
    q = qry.double().numpy().reshape(B, -1, 2)
    n = 0
    for b in range(B):
        dx = q[b][:, None, 0] - s[b][None, :, 0]
        dy = q[b][:, None, 1] - s[b][None, :, 1]
        d = np.sort(dx * dx + dy * dy, axis=1)[:, :k + 1]
        n += int(np.any(d[:, 1:] == d[:, :-1], axis=1).sum())
    return n


def _query(ops, src, qry, B, dev):
    ties = torch.zeros((1,), dtype=torch.int32, device=dev)
    idx = ops.knn_query(src.to(dev), qry.to(dev), B, 30, ties=ties)
    ref = refcpu.knn_query(src, qry, B, 30)
    assert torch.equal(idx.cpu().long().reshape(ref.shape), ref)
    return int(ties.item())


def test_ties_lattice_all_and_random_none(dev):
    from mmpde_amd import ops
    from mmpde_amd.synth import burgers_grid_points, cy_synth_mesh

    grid = burgers_grid_points()                                # 48 x 48 lattice
    # lattice queries on the lattice: almost every query ties (4 points at
    # d^2 = h^2, ...; linspace's fp32 spacing is not exactly uniform, so a few
    # do not: 2290 of 2304)
    want = tie_queries(grid, grid, 1)
    assert want > 0.9 * grid.shape[0]
    assert _query(ops, grid, grid, 1, dev) == want
    # cell centres and a jittered copy: some tie, some do not
    g = torch.Generator().manual_seed(5)
    qry = grid[torch.randperm(grid.shape[0], generator=g)[:500]].clone()
    qry[:250] += 0.5 / 47.0                                     # cell centres (ties)
    qry[250:] += 1e-3 * torch.rand(250, 2, generator=g)         # generic (no ties)
    want = tie_queries(grid, qry, 1)
    assert 0 < want < 500
    assert _query(ops, grid, qry, 1, dev) == want
    # the cylinder mesh (general position): none
    mesh = cy_synth_mesh()
    assert tie_queries(mesh, mesh, 1) == 0
    assert _query(ops, mesh.repeat(2, 1), mesh.repeat(2, 1), 2, dev) == 0


def test_ties_exhaustive_and_radix_paths(dev):
    """Long candidate lists: coincident sources (the exhaustive-rank and the
    radix-select branches of the selection) tie by construction."""
    from mmpde_amd import ops

    torch.manual_seed(12)
    src, qry = torch.rand(2 * 1000, 2), torch.rand(2 * 300, 2)
    src[0:700] = 0.5                                            # 700 coincident sources
    qry[0:100] = 0.5
    src[1000:1150] = 0.25                                       # 150 coincident: ranked list
    qry[300:340] = 0.25 + 1e-4
    want = tie_queries(src, qry, 2)
    assert want >= 140
    assert _query(ops, src, qry, 2, dev) == want


def test_ties_candidate_table_path(dev):
    """The moved-mesh query (knn_query_moved: candidate table + fallback), as
    the rollout runs it: the fixed lattice queried onto a lattice mesh moved
    by nothing (every query ties, answered from the table) and by a small
    random field (a mix), each query counted once."""
    from mmpde_amd import ops
    from mmpde_amd.synth import burgers_grid_points

    B = 3
    grid = burgers_grid_points()                                # queries ('ij' order)
    s = 48
    xi = grid.reshape(s, s, 2).transpose(0, 1).reshape(-1, 2).contiguous()   # 'xy' order
    g = torch.Generator().manual_seed(9)
    disp = torch.zeros(B, xi.shape[0], 2)
    disp[1] = 1e-4 * torch.randn(xi.shape[0], 2, generator=g)
    disp[2, :300] = 2e-3 * torch.randn(300, 2, generator=g)
    src = (xi[None] + disp).reshape(-1, 2)
    qry = grid.repeat(B, 1)
    cand = ops.knn_candidates(xi.to(dev), ref=grid.to(dev))
    ties = torch.zeros((1,), dtype=torch.int32, device=dev)
    idx = ops.knn_query_moved(src.to(dev), qry.to(dev), xi.to(dev), cand, B, 30, ref=grid.to(dev),
                              ties=ties)
    ref = refcpu.knn_query(src, qry, B, 30)
    assert torch.equal(idx.cpu().long().reshape(ref.shape), ref)
    want = tie_queries(src, qry, B)
    assert want > 0.9 * xi.shape[0]                             # trajectory 0: almost all
    assert int(ties.item()) == want


def test_rollout_reports_no_ties_on_bench_geometry(dev):
    """The bench rollout (cy, 16 trajectories): no kNN-30 query of the moved
    meshes meets an exact tie, so every step's interpolation is pinned."""
    from mmpde_amd.rollout import MMPDERollout
    from mmpde_amd.synth import build_models, fields

    pde, model, model_b, itp, dmm, gc = build_models("cy")
    for m in (model, model_b, itp, dmm):
        m.to(dev)
    B = 16
    eng = MMPDERollout("cy", model, model_b, itp, dmm, gc, B, dev)
    u = fields(pde.ori_grid, B, 30)[:, 0].to(dev)
    for s in (1, 2, 3):
        u = eng.step(u, s)
    assert eng.knn_query_ties() == 0
