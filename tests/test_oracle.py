"""CPU tests of the oracle itself: golden vectors, hand KATs, properties.
The oracle is trusted as the parity checker only after these pass."""
import math
import os

import numpy as np
import pytest
import torch
from hypothesis import given, settings
from hypothesis import strategies as st

from conftest import GOLDEN
from oracle import refcpu


# ----------------------------------------------------------------------------- kNN graph
def test_knn_graph_lattice_kat():
    """Integer lattice: exact fp32 distances with many ties at the k=35 cut;
    expected list from exact integer arithmetic (tests/golden/make_golden.py)."""
    g = np.load(os.path.join(GOLDEN, "knn35_lattice.npz"))
    ei, nbr, deg = refcpu.knn_graph(torch.from_numpy(g["pos"]), 35, 1)
    assert deg == 0
    assert torch.equal(nbr, torch.from_numpy(g["nbr"]))
    # PyG layout: row 0 source, row 1 target, grouped by target
    assert torch.equal(ei[1], torch.arange(nbr.shape[0]).repeat_interleave(35))
    assert torch.equal(ei[0], nbr.reshape(-1))


def _np_knn(pos, k):
    """numpy float64 reference: stable sort by distance (ties by index)."""
    d = ((pos[None, :, :].astype(np.float64) - pos[:, None, :]) ** 2).sum(-1)
    order = np.argsort(d, axis=1, kind="stable")
    return d, order


def test_knn_graph_random_batches():
    rng = np.random.default_rng(0)
    B, n, k = 3, 200, 35
    pos = rng.random((B * n, 2)).astype(np.float32)
    _, nbr, deg = refcpu.knn_graph(torch.from_numpy(pos), k, B)
    assert deg == 0
    for b in range(B):
        p = pos[b * n:(b + 1) * n]
        d, order = _np_knn(p, k)
        for q in range(n):
            exp = [j for j in order[q][:k + 1] if j != q][:k]
            got = (nbr[b * n + q] - b * n).tolist()
            # sets agree unless the cut falls on a float32-level near-tie
            gap = d[q, order[q][k + 1]] - d[q, order[q][k]]
            if gap > 1e-6:
                assert sorted(got) == sorted(exp)
            assert all(0 <= j < n and j != q for j in got)
            # neighbours ordered by non-decreasing distance
            dd = d[q, got]
            assert np.all(np.diff(dd) >= -1e-6)


def test_knn_graph_duplicates_are_degenerate():
    pos = torch.zeros((50, 2))
    pos[:, 0] = torch.arange(50) * 0.1
    pos[5:45] = pos[0]         # 41 coincident points {0, 5..44}
    _, nbr, deg = refcpu.knn_graph(pos, 35, 1)
    # the 36 nearest of each are {0, 5..39} (index order at d = 0): queries 40..44 lose
    # their self loop -> ragged degree (36) in the reference
    assert deg == 5
    assert (nbr >= 0).all()
    assert 39 not in nbr[39].tolist()          # self dropped
    assert nbr[40].tolist() == [0] + list(range(5, 39))


# ----------------------------------------------------------------------------- kNN-30 query
def test_knn_query_matches_sklearn_fixture():
    g = np.load(os.path.join(GOLDEN, "sklearn_knn30.npz"))
    src, qry, idx = g["src"], g["qry"], g["idx"]
    B = src.shape[0]
    got = refcpu.knn_query(torch.from_numpy(src.reshape(-1, 2)),
                           torch.from_numpy(qry.reshape(-1, 2)), B, 30)
    assert torch.equal(got, torch.from_numpy(idx))


def test_knn_query_matches_live_sklearn():
    from sklearn.neighbors import NearestNeighbors

    rng = np.random.default_rng(11)
    src = rng.random((300, 2)).astype(np.float32)
    qry = rng.random((90, 2)).astype(np.float32)
    d, i = NearestNeighbors(n_neighbors=30).fit(src).kneighbors(qry)
    assert np.all(np.diff(d, axis=-1) > 0)
    got = refcpu.knn_query(torch.from_numpy(src), torch.from_numpy(qry), 1, 30)[0]
    assert np.array_equal(got.numpy(), i)


def test_knn_query_ties_by_index():
    pos = torch.tensor([[float(i), float(j)] for i in range(8) for j in range(8)])
    q = torch.tensor([[3.0, 3.0]])
    got = refcpu.knn_query(pos, q, 1, 30)[0, 0].tolist()
    keys = sorted(((int((x - 3) ** 2 + (y - 3) ** 2), j) for j, (x, y) in enumerate(pos.tolist())))
    assert got == [j for _, j in keys[:30]]


@settings(max_examples=25, deadline=None)
@given(st.integers(min_value=31, max_value=120), st.integers(min_value=0, max_value=2 ** 31 - 1))
def test_knn_query_property_sorted_and_minimal(n, seed):
    """Property: the 30 returned are the 30 smallest (float64) distances, sorted."""
    rng = np.random.default_rng(seed)
    src = rng.random((n, 2)).astype(np.float32)
    qry = rng.random((5, 2)).astype(np.float32)
    got = refcpu.knn_query(torch.from_numpy(src), torch.from_numpy(qry), 1, 30)[0].numpy()
    d = ((src[None].astype(np.float64) - qry[:, None].astype(np.float64)) ** 2).sum(-1)
    for q in range(5):
        sel = d[q, got[q]]
        assert np.all(np.diff(sel) >= 0)
        rest = np.delete(d[q], got[q])
        assert sel.max() <= rest.min()


# ----------------------------------------------------------------------------- GNN restatement
def test_propagate_mean_kat():
    n, k = 6, 3
    ei = torch.stack([torch.tensor([1, 2, 3, 0, 2, 4, 5, 0, 1, 3, 4, 5, 0, 1, 2, 2, 3, 4]),
                      torch.arange(n).repeat_interleave(k)])
    x = torch.arange(n, dtype=torch.float32)[:, None]
    out = refcpu.propagate_mean(ei, n, lambda i, j: x[j])
    exp = torch.tensor([[2.0], [2.0], [2.0], [4.0], [1.0], [3.0]])  # means of j-groups of 3
    assert torch.allclose(out, exp)
    # a node without in-edges gets 0 (count clamped to 1)
    out = refcpu.propagate_mean(ei[:, :3], n, lambda i, j: x[j])
    assert out[1:].abs().sum() == 0


def test_gnn_zero_weights_kat():
    """All weights zero: out = dt * 0.1 * output_mlp.4.bias (gnn_2d.py:136-139)."""
    from mmpde_amd.synth import build_models

    pde, model, _, _, _, _ = build_models("cy", grid=torch.rand(50, 2), moving_mesh=False)
    sd = {k: torch.zeros_like(v) for k, v in model.state_dict().items()}
    for k in sd:
        if k.endswith("running_var"):
            sd[k] = torch.ones_like(sd[k])
    sd["output_mlp.4.bias"] = torch.tensor([0.37])
    n = 100
    ei, _, _ = refcpu.knn_graph(pde.ori_grid.repeat(2, 1), 35, 2)
    pos = torch.cat((torch.full((n, 1), 0.3), pde.ori_grid.repeat(2, 1)), 1)
    out = refcpu.mp_pde_solver(sd, refcpu.PDEConst("cy", [30, 50]), torch.randn(n, 1), pos, ei)
    scale = float((torch.ones(1, 1) * (2.9 / 29) * 0.1)[0, 0])
    assert torch.allclose(out, torch.full((n, 1), scale * 0.37))


def test_message_factorisation_identity():
    """The engine splits message_net_1 into target / source halves; check the
    identity on the oracle's own layer in float64."""
    from mmpde_amd.synth import build_models

    _, model, _, _, _, _ = build_models("cy", grid=torch.rand(40, 2), moving_mesh=False)
    W = model.gnn_layers[0].message_net_1[0].weight.double()
    b = model.gnn_layers[0].message_net_1[0].bias.double()
    h = torch.randn(2, 128, dtype=torch.float64)
    u, x, y, t = torch.randn(4, 2, dtype=torch.float64)
    full = W @ torch.cat((h[0], h[1], (u[0] - u[1])[None], (x[0] - x[1])[None],
                          (y[0] - y[1])[None], t[0][None])) + b
    a = W[:, :128] @ h[0] + W[:, 256] * u[0] + W[:, 257] * x[0] + W[:, 258] * y[0] \
        + W[:, 259] * t[0] + b
    bb = W[:, 128:256] @ h[1] - W[:, 256] * u[1] - W[:, 257] * x[1] - W[:, 258] * y[1]
    assert torch.allclose(full, a + bb, atol=1e-12)


# ----------------------------------------------------------------------------- DMM restatement
def test_dmm_mesh_matches_finite_differences():
    """x - xi from the oracle's two autograd.grad calls equals a central finite
    difference of phi (float64 copy of the weights)."""
    from mmpde_amd.synth import build_models

    torch.manual_seed(5)
    grid = torch.rand(60, 2)
    _, _, _, _, dmm, _ = build_models("cy", grid=grid)
    sd = {k: v.detach().double() for k, v in dmm.state_dict().items()}
    B = 2
    u = torch.randn(B, 60, dtype=torch.float64)
    gx, gy = grid[:, 0].double()[None].repeat(B, 1), grid[:, 1].double()[None].repeat(B, 1)
    ei, _, _ = refcpu.knn_graph(grid.repeat(B, 1), 35, B)
    x1, x2 = refcpu.moving_mesh_tri(sd, u, gx, gy, grid.double(), grid_edge_index=ei)
    xi = torch.stack((gx.reshape(-1), gy.reshape(-1)), -1)
    eps = 1e-6
    for d, got in ((0, x1), (1, x2)):
        dp, dm = xi.clone(), xi.clone()
        dp[:, d] += eps
        dm[:, d] -= eps
        fp = refcpu.dmm_forward(sd, "graph", u, dp, ori_grid=grid.double(), grid_edge_index=ei)
        fm = refcpu.dmm_forward(sd, "graph", u, dm, ori_grid=grid.double(), grid_edge_index=ei)
        fd = (fp - fm)[:, 0] / (2 * eps)
        assert torch.allclose(got[:, 0] - xi[:, d], fd, atol=1e-7, rtol=1e-5)


def test_create_data_window():
    u = torch.arange(2 * 10 * 3, dtype=torch.float32).reshape(2, 10, 3)
    d, l = refcpu.create_data(u, [4, 7], tw=1)
    assert torch.equal(d[0, 0], u[0, 3]) and torch.equal(l[1, 0], u[1, 7])


def test_gnn_out_scale_fp32():
    scale = float(torch.cumsum(torch.ones(1, 1) * (2.9 / 29) * 0.1, dim=1)[0, 0])
    assert math.isclose(scale, 0.01, rel_tol=1e-6)
