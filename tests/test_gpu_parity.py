"""GPU parity: every HIP stage against the CPU oracle on identical inputs.

Bars (stated per test):
* neighbour index maps (knn_graph, knn_query): bit-exact;
* fp32 floating point: max|hip - oracle| <= RTOL * max|oracle| + ATOL with the
  tolerance written in each test (fp32 MFMA products are exact; differences
  come from summation order and the factored message_net_1).
"""
import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import refcpu

pytestmark = pytest.mark.gpu


def _close(got, ref, rtol, atol=0.0, what=""):
    got = got.detach().float().cpu().reshape(-1)
    ref = ref.detach().float().cpu().reshape(-1)
    err = (got - ref).abs().max().item()
    bound = rtol * ref.abs().max().item() + atol
    print(f"{what}: max|err| {err:.3e} bound {bound:.3e} max|ref| {ref.abs().max().item():.3e}")
    assert err <= bound, (what, err, bound)


def _sds(**mods):
    return {k: {n: t.detach().cpu() for n, t in m.state_dict().items()} for k, m in mods.items()}


# ============================================================================ kNN graph
def _graph_case(pos, B, dev, k=35):
    from mmpde_amd import ops

    nbr, deg = ops.knn_graph_nbr(pos.to(dev), B, k, count_degenerate=True)
    _, ref, rdeg = refcpu.knn_graph(pos, k, B)
    assert int(deg.item()) == rdeg
    assert torch.equal(nbr.cpu().long(), ref)


def test_knn_graph_cy_mesh_bit_exact(dev):
    from mmpde_amd.synth import cy_synth_mesh

    g = cy_synth_mesh()
    moved = g + 0.01 * torch.sin(7 * g.flip(1))            # a moved-mesh-like input
    _graph_case(torch.cat((g, moved)), 2, dev)


def test_knn_graph_burgers_grid_ties_bit_exact(dev):
    from mmpde_amd.synth import burgers_grid_points

    _graph_case(burgers_grid_points().repeat(2, 1), 2, dev)   # linspace grid: ties at the cut


@pytest.mark.gpu
def test_knn_moved_cells_record_vs_numpy(dev):
    """The per-trajectory displacement record of the candidate path
    (mmpde_knn_moved_cells): per 16 x 16 cell of xi's box the largest |x_j - xi_j|
    (empty: -1), the trajectory's largest, and the median over the non-empty
    cells (the skip threshold's statistic) against a numpy restatement.  The
    kernel rounds each distance up by 2^-20 relative (a bound), so values match
    to that factor."""
    from mmpde_amd import ops
    from mmpde_amd.synth import cy_synth_mesh

    xi = cy_synth_mesh()
    N, B = xi.shape[0], 3
    g = torch.Generator().manual_seed(7)
    disp = torch.stack([0.004 * torch.randn((N, 2), generator=g),
                        0.02 * torch.randn((N, 2), generator=g),
                        torch.zeros((N, 2))])
    disp[2, 11] = 0.3                                       # one far-moved node
    pos = (xi[None] + disp).reshape(-1, 2)
    rec = ops.knn_moved_cells(pos.to(dev), xi.to(dev), B).cpu().numpy().reshape(B, -1)
    x32 = xi.numpy().astype(np.float32)
    lo, hi = x32.min(0), x32.max(0)
    h = ((hi - lo) / np.float32(16)).astype(np.float32)    # the kernel's fp32 cell assignment
    ih = (np.float32(1) / h).astype(np.float32)
    cell = np.clip(((x32 - lo) * ih).astype(np.int64), 0, 15)
    cid = cell[:, 1] * 16 + cell[:, 0]
    x = x32.astype(np.float64)
    for b in range(B):
        d = np.sqrt(((pos.numpy()[b * N:(b + 1) * N].astype(np.float64) - x) ** 2).sum(1))
        dcell = np.full(256, -1.0)
        for c in range(256):
            m = cid == c
            if m.any():
                dcell[c] = d[m].max()
        got = rec[b, :256]
        assert np.array_equal(got < 0, dcell < 0), f"empty cells of trajectory {b}"
        ne = dcell >= 0
        np.testing.assert_allclose(got[ne], dcell[ne], rtol=4e-6, atol=1e-9)
        np.testing.assert_allclose(rec[b, 256 + 5], d.max(), rtol=4e-6, atol=1e-9)
        med = np.sort(dcell[ne])[ne.sum() // 2]
        np.testing.assert_allclose(rec[b, 256 + 6], med, rtol=4e-6, atol=1e-9)


@pytest.mark.parametrize("kind", ["cy", "burgers"])
def test_knn_graph_moved_candidates_bit_exact(dev, kind):
    """The candidate-table graph and kNN-30 query (mmpde_knn_graph_cand /
    mmpde_knn_query_cand) against the oracle and the full search, on
    trajectories that exercise every branch: unmoved (ties at the cut on the
    burgers lattice), small smooth and small random displacements (the table
    answers), random displacements of 0.02 (mixed: some queries answered, the
    rest by the full search in the same workgroups), one node moved far (the
    per-cell bound keeps the table for the queries away from it) and a large
    smooth displacement (the bound fails, the full search answers).  The
    tables' answered shares are asserted so that each regime is really hit."""
    from mmpde_amd import ops
    from mmpde_amd.synth import burgers_grid_points, cy_synth_mesh

    xi = cy_synth_mesh() if kind == "cy" else burgers_grid_points()
    N = xi.shape[0]
    gen = torch.Generator().manual_seed(5)
    one_far = xi.clone()
    one_far[N // 3] += torch.tensor([0.08, -0.05])
    moved = [xi, xi + 0.004 * torch.sin(9 * xi.flip(1)),
             xi + 0.002 * torch.randn(xi.shape, generator=gen),
             xi + 0.02 * torch.randn(xi.shape, generator=gen),
             one_far,
             xi + 0.3 * torch.sin(3 * xi.flip(1))]
    B = len(moved)
    pos = torch.cat(moved)
    xd, pd = xi.to(dev), pos.to(dev)
    cand = ops.knn_candidates(xd)
    assert cand is not None and cand.shape == (N, ops.KNN_CAND)
    cells = ops.knn_moved_cells(pd, xd, B)
    nbr, deg = ops.knn_graph_moved(pd, xd, cand, B, 35, count_degenerate=True, cells=cells)
    share = ops.knn_table_share(cells, B, N)[:, 0].cpu()
    print(f"{kind} graph: table share per trajectory {share.tolist()}")
    _, ref, rdeg = refcpu.knn_graph(pos, 35, B)
    assert int(deg.item()) == rdeg
    assert torch.equal(nbr.cpu().long(), ref)
    assert torch.equal(nbr, ops.knn_graph_nbr(pd, B, 35))
    assert share[1] > 0.99 and share[2] > 0.99           # small displacements: the table
    assert 0.0 < share[3] < 1.0                           # mixed
    assert share[4] > 0.7                                 # one far node: its cells only
    assert share[5] < 0.05                                # large: the full search
    # the skip threshold sends the trajectories moved far everywhere (3 and 5)
    # straight to the full search, not the one with a single far node (4);
    # same tables bit for bit
    thr = ops.knn_skip_threshold(xd, cand, 36, moved_queries=True)
    assert 0.0 < thr < 0.1
    cells = ops.knn_moved_cells(pd, xd, B)
    nbr_s = ops.knn_graph_moved(pd, xd, cand, B, 35, cells=cells, skip_above=thr)
    share_s = ops.knn_table_share(cells, B, N)[:, 0].cpu()
    print(f"{kind} graph, skip above {thr:.4f}: table share {share_s.tolist()}")
    assert torch.equal(nbr_s, nbr)
    assert share_s[3] == 0.0 and share_s[5] == 0.0 and share_s[4] > 0.7
    assert share_s[1] > 0.99 and share_s[2] > 0.99
    # the kNN-30 query of fixed points onto the moved meshes: queries at xi
    # (table of xi), moved off xi (the bound takes the offset), and the queries
    # in another order than xi -- burgers: the 'ij' grid against the 'xy' xi,
    # cy: a permutation -- once with a table built for that order (answered
    # from the table) and once with xi's table (offsets large: full search)
    if kind == "burgers":
        s = int(round(N ** 0.5))
        perm = torch.arange(N).reshape(s, s).t().reshape(-1)   # 'ij' index -> 'xy' index
    else:
        perm = torch.randperm(N, generator=gen)
    other = xi[perm]
    cand_o = ops.knn_candidates(xd, ref=other.to(dev))
    cases = [(xi.repeat(B, 1), cand, None, 1),
             (xi.repeat(B, 1) + 0.003 * torch.cos(5 * xi.repeat(B, 1)), cand, None, 1),
             (other.repeat(B, 1), cand_o, other, 1),
             (other.repeat(B, 1), cand, None, 0)]
    for qry, cq, rq, expect_table in cases:
        cells = ops.knn_moved_cells(pd, xd, B)             # fresh miss counters
        idx = ops.knn_query_moved(pd, qry.to(dev), xd, cq, B, 30,
                                  ref=None if rq is None else rq.to(dev), cells=cells)
        qs = ops.knn_table_share(cells, B, N)[:, 1].cpu()
        print(f"{kind} query: table share per trajectory {qs.tolist()}")
        assert torch.equal(idx, ops.knn_query(pd, qry.to(dev), B, 30))
        ref_q = refcpu.knn_query(pos, qry, B, 30)
        assert torch.equal(idx.cpu().long().reshape(ref_q.shape), ref_q)
        if expect_table:
            assert qs[1] > 0.99 and qs[2] > 0.99
        else:
            assert qs[1] < 0.5


def test_knn_graph_integer_lattice_golden(dev):
    from mmpde_amd import ops

    g = np.load(f"{GOLDEN}/knn35_lattice.npz")
    nbr = ops.knn_graph_nbr(torch.from_numpy(g["pos"]).to(dev), 1, 35)
    assert np.array_equal(nbr.cpu().numpy(), g["nbr"])


@pytest.mark.parametrize("n,B", [(36, 3), (100, 5), (640, 2), (4096, 1), (3000, 2),
                                 (4097, 1), (9216, 2), (16384, 1)])   # > 4096: knn_large_kernel
def test_knn_graph_sizes(dev, n, B):
    torch.manual_seed(n)
    _graph_case(torch.rand(n * B, 2), B, dev)


def test_knn_graph_duplicates(dev):
    pos = torch.rand(200, 2)
    pos[50:100] = pos[3]                                       # 51 coincident points
    pos[120:125] = pos[7]
    _graph_case(pos, 1, dev)


def test_knn_graph_candidate_overflow_fallback(dev):
    # > 512 points tie with the kk-th lane minimum: the LDS candidate list
    # overflows and the kernel takes the full radix-select path.
    torch.manual_seed(11)
    pos = torch.rand(2 * 1500, 2)
    pos[100:800] = pos[5]                                      # 701 coincident points
    pos[1500 + 200:1500 + 1400] = 0.25                         # 1200 coincident points
    _graph_case(pos, 2, dev)


# ============================================================================ kNN-30 query
def test_knn_query_sklearn_golden(dev):
    from mmpde_amd import ops

    g = np.load(f"{GOLDEN}/sklearn_knn30.npz")
    B = g["src"].shape[0]
    idx = ops.knn_query(torch.from_numpy(g["src"]).to(dev), torch.from_numpy(g["qry"]).to(dev),
                        B, 30)
    assert np.array_equal(idx.cpu().numpy().reshape(g["idx"].shape), g["idx"])


@pytest.mark.parametrize("ns,nq,B", [(2521, 2521, 2), (30, 7, 2), (2304, 2304, 1), (4096, 50, 1),
                                     (9216, 2304, 2), (16384, 300, 1)])
def test_knn_query_bit_exact(dev, ns, nq, B):
    from mmpde_amd import ops

    torch.manual_seed(ns + nq)
    src, qry = torch.rand(B * ns, 2), torch.rand(B * nq, 2)
    qry[:3] = src[:3]                                          # zero-distance hits
    idx = ops.knn_query(src.to(dev), qry.to(dev), B, 30)
    ref = refcpu.knn_query(src, qry, B, 30)
    assert torch.equal(idx.cpu().long().reshape(ref.shape), ref)


def test_knn_large_candidate_overflow_fallback(dev):
    # > 4096 points per trajectory with hundreds of coincident points: the
    # large-set kernel's chunked compaction overflows the LDS list and takes
    # the radix-select path, for the graph and the query variant.
    from mmpde_amd import ops

    torch.manual_seed(13)
    pos = torch.rand(2 * 6000, 2)
    pos[100:900] = pos[5]                                      # 801 coincident points
    pos[6000 + 4000:6000 + 5300] = 0.25                        # 1300 coincident points
    _graph_case(pos, 2, dev)
    qry = torch.rand(2 * 200, 2)
    qry[:50] = pos[5]
    qry[200:260] = 0.25
    idx = ops.knn_query(pos.to(dev), qry.to(dev), 2, 30)
    ref = refcpu.knn_query(pos, qry, 2, 30)
    assert torch.equal(idx.cpu().long().reshape(ref.shape), ref)


def test_knn_query_candidate_overflow_fallback(dev):
    from mmpde_amd import ops

    torch.manual_seed(12)
    src, qry = torch.rand(2 * 1000, 2), torch.rand(2 * 300, 2)
    src[0:700] = 0.5                                           # 700 coincident sources
    qry[0:100] = 0.5
    idx = ops.knn_query(src.to(dev), qry.to(dev), 2, 30)
    ref = refcpu.knn_query(src, qry, 2, 30)
    assert torch.equal(idx.cpu().long().reshape(ref.shape), ref)


@pytest.mark.parametrize("ring", [90, 400])
def test_knn_query_fp32_filter_margin(dev, ring):
    # `ring` sources at radius 0.1 (+- 1e-7 relative) from each query: their
    # fp32 squared distances tie or misorder, only the fp64 keys separate
    # them, so the candidate filter's rounding margin decides the answer.
    # ring=90 takes the bitonic path, ring=400 the exhaustive-rank path.
    from mmpde_amd import ops

    g = torch.Generator().manual_seed(ring)
    nq, nfar = 6, 1200
    qry = 0.3 + 0.4 * torch.rand(nq, 2, generator=g)
    src = []
    for q in qry:
        th = 2 * np.pi * torch.rand(ring, generator=g, dtype=torch.float64)
        r = 0.1 * (1 + 1e-7 * torch.randn(ring, generator=g, dtype=torch.float64))
        src.append(q.double() + torch.stack((r * th.cos(), r * th.sin()), 1))
    src.append(0.5 + 2.0 * (torch.rand(nfar, 2, generator=g, dtype=torch.float64) - 0.5) + 0.3)
    src = torch.cat(src).float()
    idx = ops.knn_query(src.to(dev), qry.to(dev), 1, 30)
    assert torch.equal(idx.cpu().long(), refcpu.knn_query(src, qry, 1, 30)[0])


def test_knn_query_lattice_ties(dev):
    from mmpde_amd import ops

    src = torch.tensor([[float(i), float(j)] for i in range(10) for j in range(10)])
    qry = src[torch.randperm(100)[:20]] + 0.5 * (torch.rand(20, 2) > 0.5)
    idx = ops.knn_query(src.to(dev), qry.to(dev), 1, 30)
    assert torch.equal(idx.cpu().long(), refcpu.knn_query(src, qry, 1, 30)[0])


# ============================================================================ GNN
def _gnn_inputs(kind, B, seed=0):
    from mmpde_amd.synth import build_models, burgers_grid_points

    pde, model, _, _, _, gc = build_models(kind, moving_mesh=False, seed=seed)
    pts = pde.ori_grid if kind == "cy" else burgers_grid_points()
    torch.manual_seed(seed + 7)
    n = B * pts.shape[0]
    pos = torch.cat((torch.full((n, 1), float(gc.time_grid()[5])), pts.repeat(B, 1)), 1)
    u = torch.randn(n, 1)
    ei, nbr, _ = refcpu.knn_graph(pts.repeat(B, 1), 35, B)
    return pde, model, u, pos, ei, nbr


@pytest.mark.parametrize("kind", ["cy", "burgers"])
def test_gnn_forward_matches_oracle(dev, kind):
    from mmpde_amd.rollout import _Nodes

    pde, model, u, pos, ei, nbr = _gnn_inputs(kind, 2)
    opde = refcpu.PDEConst(kind, pde.grid_size, ori_grid=getattr(pde, "ori_grid", None))
    ref, hs = refcpu.mp_pde_solver(_sds(m=model)["m"], opde, u, pos, ei, return_hidden=True)
    model.to(dev)
    out = model(_Nodes(u.to(dev), pos.to(dev), nbr.int().to(dev)))
    # fp32 tolerance for 6 BN'd layers + head: 1e-5 of the output range
    _close(out, ref, 1e-5, 1e-9, f"gnn {kind}")
    # the rollout's position form: (x, y) rows + one t (host value or device
    # slot) gives the same bits as the (t, x, y) rows, in both GEMM modes
    t = float(pos[0, 0])
    xy = pos[:, 1:].contiguous().to(dev)
    for mode in ("f32", "f16x3"):
        model.edge_gemm = mode
        full = model(_Nodes(u.to(dev), pos.to(dev), nbr.int().to(dev), seg_n=pos.shape[0] // 2))
        a = model(_Nodes(u.to(dev), xy, nbr.int().to(dev), seg_n=pos.shape[0] // 2, t=t))
        b = model(_Nodes(u.to(dev), xy, nbr.int().to(dev), seg_n=pos.shape[0] // 2,
                         t_slot=torch.tensor([t], device=dev)))
        assert torch.equal(a, full) and torch.equal(b, full), mode


def test_gnn_layer_api_and_edge_index_input(dev):
    """Layer-level reference API (x, u, pos_x, pos_y, variables, edge_index, batch)
    and a PyG-style edge_index input both run the HIP path."""
    pde, model, u, pos, ei, nbr = _gnn_inputs("cy", 1)
    sd = _sds(m=model)["m"]
    h = torch.randn(u.shape[0], 128)
    px, py, pt = pos[:, 1:2], pos[:, 2:3], pos[:, 0:1] / 2.9
    ref = refcpu.gnn_layer(sd, "gnn_layers.0", h, u, px, py, pt, ei)
    model.to(dev)
    got = model.gnn_layers[0](h.to(dev), u.to(dev), px.to(dev), py.to(dev), pt.to(dev),
                              ei.to(dev), None)
    _close(got, ref, 5e-5, 1e-6, "gnn layer")

    g = type("G", (), {"x": u.to(dev), "pos": pos.to(dev), "edge_index": ei.to(dev),
                       "nbr": None})
    ref2 = refcpu.mp_pde_solver(sd, refcpu.PDEConst("cy", pde.grid_size), u, pos, ei)
    _close(model(g()), ref2, 1e-5, 1e-9, "gnn edge_index input")


@pytest.mark.parametrize("tw", [1, 3])
def test_gnn_layer_api_any_time_window_ragged_edge_index(dev, tw):
    """The layer API on what the fused launch does not take: time_window 3, and
    a ragged, ungrouped edge_index (every 7th edge dropped, edges shuffled, one
    node without in-edges): the HIP EdgeMean path, against the oracle."""
    from mmpde_amd.gnn_2d import GNN_Layer_FS_2D

    torch.manual_seed(4)
    layer = GNN_Layer_FS_2D(128, 128, 128, time_window=tw, n_variables=1).eval()
    with torch.no_grad():
        layer.norm.module.running_mean.normal_(0, 0.1)
        layer.norm.module.running_var.uniform_(0.5, 1.5)
    sd = {"L." + k: v.detach() for k, v in layer.state_dict().items()}
    n, k = 700, 12
    g = torch.Generator().manual_seed(5)
    pts = torch.rand(n, 2, generator=g)
    ei, _, _ = refcpu.knn_graph(pts, k, 1)
    keep = torch.ones(ei.shape[1], dtype=torch.bool)
    keep[::7] = False
    keep[ei[1] == 5] = False                       # node 5: no in-edges (mean 0)
    ei = ei[:, keep][:, torch.randperm(int(keep.sum()), generator=g)]
    h = torch.randn(n, 128, generator=g)
    u = torch.randn(n, tw, generator=g)
    px, py, pt = pts[:, :1], pts[:, 1:], torch.rand(n, 1, generator=g)
    ref = refcpu.gnn_layer(sd, "L", h, u, px, py, pt, ei)
    layer.to(dev)
    got = layer(h.to(dev), u.to(dev), px.to(dev), py.to(dev), pt.to(dev), ei.to(dev), None)
    _close(got, ref, 2e-5, 1e-6, f"gnn layer tw={tw}, ragged edge_index")


def test_edge_mean_vs_torch_fp32(dev):
    """The hot kernel alone against a plain torch fp32 evaluation of
    mean_e relu(W2 relu(a_i + b_nbr) + b2)."""
    from mmpde_amd import _lib as L

    torch.manual_seed(1)
    n, k = 3000, 35
    a, b = torch.randn(n, 128), torch.randn(n, 128)
    nbr = torch.randint(0, n, (n, k), dtype=torch.int32)
    w2, b2 = torch.randn(128, 128) / 11, torch.randn(128) / 10
    m1 = torch.relu(a[:, None, :] + b[nbr.long()])
    ref = torch.relu(m1 @ w2.T + b2).mean(1)
    d = [t.to(dev) for t in (a, b, nbr, w2, b2)]
    out = torch.empty(n, 128, device=dev)
    L.check(L.lib().mmpde_gnn_edge_mean(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), n, k,
                                        d[3].data_ptr(), d[4].data_ptr(), out.data_ptr(),
                                        L.stream(dev)), "edge_mean")
    _close(out, ref, 1e-5, 1e-6, "edge_mean")


# ============================================================================ DMM
def test_dmm_mesh_graph_matches_autograd(dev):
    from mmpde_amd.synth import build_models, fields

    pde, _, _, _, dmm, _ = build_models("cy")
    grid = pde.ori_grid
    B = 3
    u = fields(grid, B, 30)[:, 4]
    ref_x, ref_y = refcpu.moving_mesh_tri(_sds(d=dmm)["d"], u, grid[None, :, 0].repeat(B, 1),
                                         grid[None, :, 1].repeat(B, 1), grid)
    ref = torch.cat((ref_x, ref_y), -1)
    dmm.to(dev)
    got = dmm.mesh(u.to(dev), grid.to(dev))
    torch.cuda.synchronize()
    disp = (ref - grid.repeat(B, 1)).abs().max().item()
    assert disp > 1e-3                                         # the mesh actually moves
    _close(got, ref, 0.0, 2e-6, "dmm graph mesh")              # absolute, coords in [0,1]


def test_dmm_mesh_array_matches_autograd(dev):
    from mmpde_amd.synth import build_models, burgers_grid_points, fields

    pde, _, _, _, dmm, gc = build_models("burgers")
    B = 3
    u = fields(burgers_grid_points(), B, 31).reshape(B, 31, 48, 48)[:, 4]
    ox, oy = refcpu.moving_mesh(_sds(d=dmm)["d"], refcpu.PDEConst("burgers", [31, 48, 48]), u,
                                48, 48)
    ref = torch.cat((ox, oy), -1)
    dmm.to(dev)
    got = dmm.mesh(u.to(dev).contiguous(), gc.xi_grid_xy(48, 48, dev))
    torch.cuda.synchronize()
    _close(got, ref, 0.0, 2e-6, "dmm array mesh")


@pytest.mark.parametrize("kind", ["cy", "burgers"])
def test_dmm_head_cache_identical(dev, kind):
    """A prepared grid-side head (trunk, Q, J of the fixed xi) gives the same mesh,
    bit for bit, as computing it inside the call."""
    from mmpde_amd.synth import build_models, burgers_grid_points, fields

    pde, _, _, _, dmm, gc = build_models(kind)
    B = 4
    dmm.to(dev)
    if kind == "cy":
        xi = pde.ori_grid.to(dev)
        u = fields(pde.ori_grid, B, 30)[:, 7].to(dev).contiguous()
    else:
        xi = gc.xi_grid_xy(48, 48, dev)
        u = fields(burgers_grid_points(), B, 31).reshape(B, 31, 48, 48)[:, 7].to(dev).contiguous()
    cache = dmm.head_cache(xi)
    a = dmm.mesh(u, xi)
    b = dmm.mesh(u, xi, head_cache=cache)
    assert torch.equal(a, b)


# ============================================================================ ItpNet
@pytest.mark.parametrize("mode", ["1", "2"])
def test_itp_interp_matches_oracle(dev, mode):
    from mmpde_amd import ops
    from mmpde_amd.synth import build_models

    pde, _, _, itp, _, _ = build_models("cy")
    B, N = 2, pde.ori_grid.shape[0]
    torch.manual_seed(2)
    src = pde.ori_grid.repeat(B, 1) + 0.01 * torch.randn(B * N, 2)
    qry = pde.ori_grid.repeat(B, 1)
    vals = torch.randn(B, N)
    ref, idx = refcpu.interpolate(_sds(i=itp)["i"], vals, src[:, :1], src[:, 1:], qry[:, :1],
                                  qry[:, 1:], mode, return_idx=True)
    itp.to(dev)
    got = ops.itp_interp(src.to(dev), vals.to(dev), qry.to(dev),
                         idx.reshape(B * N, 30).int().to(dev), B, itp.packed(mode))
    _close(got, ref, 2e-5, 1e-6, f"itp mode {mode}")


@pytest.mark.parametrize("kind", ["cy", "burgers"])
def test_res_cut_matches_oracle(dev, kind):
    from mmpde_amd.synth import build_models

    _, _, _, itp, _, _ = build_models(kind)
    torch.manual_seed(4)
    x = torch.randn(3, 2521) if kind == "cy" else torch.randn(3, 1, 48, 48)
    ref = refcpu.itpnet(_sds(i=itp)["i"], None, None, "res_cut", data=x, burgers=kind != "cy")
    itp.to(dev)
    _close(itp(None, None, "res_cut", data=x.to(dev)), ref, 1e-5, 1e-6, f"res_cut {kind}")


# ============================================================================ full step
@pytest.mark.parametrize("kind", ["cy", "burgers"])
def test_mmpde_step_matches_oracle(dev, kind):
    """One MM-PDE step (train_helper_2d.py:174-185) through the rollout engine vs
    the oracle; the oracle uses the engine's moved mesh (mesh_override) so the
    kNN stages see identical coordinates -- the mesh itself is checked above."""
    from mmpde_amd.rollout import MMPDERollout
    from mmpde_amd.synth import build_models, burgers_grid_points, fields

    pde, model, model_b, itp, dmm, gc = build_models(kind)
    B, step = 2, 6
    if kind == "cy":
        data = fields(pde.ori_grid, B, 30)[:, step - 1:step]
        opde = refcpu.PDEConst("cy", pde.grid_size, ori_grid=pde.ori_grid)
    else:
        data = fields(burgers_grid_points(), B, 31).reshape(B, 31, 48, 48)[:, step - 1:step]
        opde = refcpu.PDEConst("burgers", pde.grid_size)
    sds = _sds(model=model, model_b=model_b, itp=itp, dmm=dmm)
    for m in (model, model_b, itp, dmm):
        m.to(dev)
    eng = MMPDERollout(kind, model, model_b, itp, dmm, gc, B, dev)
    pred = eng.step(data[:, 0].to(dev), step)
    ref, aux = refcpu.mmpde_step(opde, sds, data, data, [step] * B, mesh_override=eng.mesh.cpu())
    assert torch.equal(eng.nbr_u.cpu().long(), aux["graph_uni"].nbr)
    _close(pred, ref, 2e-5, 1e-6, f"mmpde step {kind}")


def test_gnn_only_step_matches_oracle(dev):
    from mmpde_amd.rollout import MMPDERollout
    from mmpde_amd.synth import build_models, fields

    pde, model, _, _, _, gc = build_models("cy", moving_mesh=False)
    B, step = 3, 3
    data = fields(pde.ori_grid, B, 30)[:, step - 1:step]
    ref, _ = refcpu.mmpde_step(refcpu.PDEConst("cy", pde.grid_size, ori_grid=pde.ori_grid),
                               _sds(model=model), data, data, [step] * B, moving_mesh=False)
    model.to(dev)
    eng = MMPDERollout("cy", model, None, None, None, gc, B, dev, moving_mesh=False)
    _close(eng.step(data[:, 0].to(dev), step), ref, 1e-5, 1e-9, "gnn-only step")


def test_burgers_gnn_default_resolution_api_matches_oracle(dev):
    """BASELINE configs[0]'s shape on the GPU: the Burgers GNN baseline
    (moving_mesh=False) at the PDE's default resolution (31, 96, 96), 9216
    nodes per trajectory (the large-set kNN kernel), through the drop-in API
    (create_graph(..., None) -> model(graph), train_helper_2d.py:177-181)."""
    from mmpde_amd.synth import build_models, burgers_grid_points, fields

    pde, model, _, _, _, gc = build_models("burgers", moving_mesh=False, seed=4)
    res = [31, 96, 96]
    pde.grid_size = pde.movingmesh_grid_size = pde.ori_grid_size = res
    B, step = 1, 7
    u = fields(burgers_grid_points(96), B, 31, seed=5).reshape(B, 31, 96, 96)
    data, labels = gc.create_data(u, [step] * B)
    opde = refcpu.PDEConst("burgers", res)
    ref, aux = refcpu.mmpde_step(opde, _sds(model=model), data, labels, [step] * B, moving_mesh=False)
    model.to(dev)
    graph = gc.create_graph(None, data, labels, [step] * B, dev, None)
    assert torch.equal(graph.edge_index.cpu(), aux["graph_uni"].edge_index), "kNN-35 graph, 9216 nodes"
    _close(model(graph), ref, 1e-5, 1e-9, "burgers GNN 96x96")


def test_graph_creator_api_equals_engine(dev):
    """The drop-in GraphCreator path (create_graph / interpolate_pred) and the
    rollout engine compose the same kernels: identical bits.  (Oracle parity of
    that path, cy and burgers: tests/test_gpu_api.py.)"""
    from mmpde_amd.rollout import MMPDERollout
    from mmpde_amd.synth import build_models, fields

    pde, model, model_b, itp, dmm, gc = build_models("cy")
    for m in (model, model_b, itp, dmm):
        m.to(dev)
    B, step = 2, 4
    u = fields(pde.ori_grid, B, 30)
    data, labels = gc.create_data(u, [step] * B)
    graph = gc.create_graph(itp, data, labels, [step] * B, dev, dmm)
    graph_uni = gc.create_graph(itp, data, labels, [step] * B, dev, None)
    pred = gc.interpolate_pred(itp, model_b(graph), graph, data, dev) + model(graph_uni)
    eng = MMPDERollout("cy", model, model_b, itp, dmm, gc, B, dev)
    pe = eng.step(data[:, 0].to(dev), step)
    assert torch.equal(pred.reshape(-1), pe.reshape(-1))
    ei = graph.edge_index
    assert ei.dtype == torch.int64 and ei.shape == (2, B * 2521 * 35)
    assert torch.equal(ei[0].reshape(-1, 35).int(), graph.nbr)


# ============================================================================ full size
def test_full_size_properties(dev):
    """BASELINE config 4 size (16 x 2521 nodes): properties the oracle is too slow
    to check end to end -- graph validity, determinism, finite rollout."""
    from mmpde_amd import ops
    from mmpde_amd.rollout import MMPDERollout
    from mmpde_amd.synth import build_models, fields

    pde, model, model_b, itp, dmm, gc = build_models("cy")
    for m in (model, model_b, itp, dmm):
        m.to(dev)
    B, N = 16, 2521
    eng = MMPDERollout("cy", model, model_b, itp, dmm, gc, B, dev)
    u0 = fields(pde.ori_grid, B, 30)[:, 0].to(dev)
    p1 = eng.step(u0, 1)
    mesh = eng.mesh.clone()
    p2 = eng.step(u0, 1)
    assert torch.equal(p1, p2)                                  # bitwise deterministic
    nbr = ops.knn_graph_nbr(mesh, B, 35).long().cpu()
    rows = torch.arange(B * N)[:, None]
    assert ((nbr // N) == rows // N).all()                      # within own trajectory
    assert (nbr != rows).all()                                  # no self loops
    m = mesh.cpu().double()
    d = ((m[nbr] - m[:, None, :]) ** 2).sum(-1)
    assert (d[:, 1:] >= d[:, :-1] - 1e-12).all()                # sorted by distance
    # spot-check trajectory 11 against the oracle bit for bit
    _, ref, _ = refcpu.knn_graph(mesh[11 * N:12 * N].cpu(), 35, 1)
    assert torch.equal(nbr[11 * N:12 * N] - 11 * N, ref)
    u = eng.rollout(u0, 1, 29)
    assert torch.isfinite(u).all()


# ============================================================================ layer kernels: odd sizes
@pytest.mark.parametrize("k", [1, 3, 4, 5, 8, 35])
@pytest.mark.parametrize("mode", ["f32", "f16x3"])
def test_gnn_forward_ragged_k(dev, k, mode):
    """Degrees that leave partial rounds of neighbour slots (k % 4 != 0, k < 4)
    and node counts that leave partial edge tiles / node tiles (3 x 37 rows),
    in both arithmetic modes, against the oracle."""
    from mmpde_amd.rollout import _Nodes
    from mmpde_amd.synth import build_models

    pde, model, _, _, _, _ = build_models("cy", moving_mesh=False, seed=3)
    B, N = 3, 37
    torch.manual_seed(k)
    pts = torch.rand(B * N, 2)
    pos = torch.cat((torch.full((B * N, 1), 0.7), pts), 1)
    u = torch.randn(B * N, 1)
    ei, nbr, _ = refcpu.knn_graph(pts, k, B)
    opde = refcpu.PDEConst("cy", pde.grid_size, ori_grid=pde.ori_grid)
    ref = refcpu.mp_pde_solver(_sds(m=model)["m"], opde, u, pos, ei)
    model.to(dev)
    model.edge_gemm = mode
    out = model(_Nodes(u.to(dev), pos.to(dev), nbr.int().to(dev)))
    _close(out, ref, 1e-5, 1e-9, f"gnn k={k} {mode}")


@pytest.mark.parametrize("mode", ["f32", "f16x3"])
def test_gnn_forward_segments_cross_tiles(dev, mode):
    """Trajectory segments of 37 rows, so 16-row range blocks and 32-row node
    tiles straddle segment boundaries (the node epilogue's second-segment
    maxima, the edge kernel's per-segment units and side blocks): against the
    oracle, and each trajectory of the batch bitwise equal to it launched alone."""
    from mmpde_amd.rollout import _Nodes
    from mmpde_amd.synth import build_models

    pde, model, _, _, _, _ = build_models("cy", moving_mesh=False, seed=5)
    B, N, k = 3, 37, 35
    torch.manual_seed(11)
    pts = torch.rand(B * N, 2)
    pos = torch.cat((torch.full((B * N, 1), 0.4), pts), 1)
    u = torch.randn(B * N, 1)
    ei, nbr, _ = refcpu.knn_graph(pts, k, B)
    opde = refcpu.PDEConst("cy", pde.grid_size, ori_grid=pde.ori_grid)
    ref = refcpu.mp_pde_solver(_sds(m=model)["m"], opde, u, pos, ei)
    model.to(dev)
    model.edge_gemm = mode
    out = model(_Nodes(u.to(dev), pos.to(dev), nbr.int().to(dev), seg_n=N))
    _close(out, ref, 1e-5, 1e-9, f"gnn 3 x 37-row segments {mode}")
    for j in range(B):
        rows = slice(j * N, (j + 1) * N)
        alone = model(_Nodes(u[rows].to(dev), pos[rows].to(dev), (nbr[rows] - j * N).int().to(dev), seg_n=N))
        assert torch.equal(out[rows], alone), (mode, j)


# ============================================================================ hipGraph replay
@pytest.mark.parametrize("kind", ["cy", "burgers"])
def test_graph_replay_matches_eager(dev, kind):
    """The captured step (all three streams in one hipGraph, t read from a device
    slot) replayed over an autoregressive rollout equals the eager rollout bit
    for bit (every kernel is deterministic), across step indices."""
    from mmpde_amd.rollout import MMPDERollout
    from mmpde_amd.synth import build_models, burgers_grid_points, fields

    pde, model, model_b, itp, dmm, gc = build_models(kind)
    B = 2
    if kind == "cy":
        u0 = fields(pde.ori_grid, B, 30)[:, 3]
    else:
        u0 = fields(burgers_grid_points(), B, 31).reshape(B, 31, 48, 48)[:, 3]
    for m in (model, model_b, itp, dmm):
        m.to(dev)
    for m in (model, model_b):
        m.edge_gemm = "f16x3"
    eng = MMPDERollout(kind, model, model_b, itp, dmm, gc, B, dev)
    u0 = u0.to(dev).contiguous()
    ref, u = [], u0
    for s in range(4, 8):
        u = eng.step(u, s)
        ref.append(u.clone())
    eng.enable_graph(u0)
    u = u0
    for i, s in enumerate(range(4, 8)):
        u = eng.graph_step(u, s)
        assert torch.equal(u, ref[i]), f"{kind} graph step {s}: max|diff| {(u - ref[i]).abs().max()}"


@pytest.mark.parametrize("kind", ["cy", "burgers"])
def test_stream_priorities_match_default(dev, kind):
    """The step with stream priorities on (the moving-mesh chain on its own
    high-priority stream, model(u) low: MMPDERollout.set_priorities) equals the
    default streams bit for bit over an autoregressive rollout: which stream a
    kernel runs on changes no sum."""
    from mmpde_amd.rollout import MMPDERollout
    from mmpde_amd.synth import build_models, burgers_grid_points, fields

    pde, model, model_b, itp, dmm, gc = build_models(kind)
    B = 2
    if kind == "cy":
        u0 = fields(pde.ori_grid, B, 30)[:, 3]
    else:
        u0 = fields(burgers_grid_points(), B, 31).reshape(B, 31, 48, 48)[:, 3]
    for m in (model, model_b, itp, dmm):
        m.to(dev)
    for m in (model, model_b):
        m.edge_gemm = "f16x3"
    eng = MMPDERollout(kind, model, model_b, itp, dmm, gc, B, dev)
    u0 = u0.to(dev).contiguous()
    outs = {}
    for on in (False, True):
        eng.set_priorities(on)
        u, outs[on] = u0, []
        for s in range(4, 8):
            u = eng.step(u, s)
            outs[on].append(u.clone())
    torch.cuda.synchronize(dev)
    for i, (a, b) in enumerate(zip(outs[False], outs[True])):
        assert torch.equal(a, b), f"{kind} step {4 + i}: max|diff| {(a - b).abs().max()}"


# ============================================================================ full size vs oracle
@pytest.mark.parametrize("edge_gemm", ["f16x3", "f32"])
def test_full_size_step_matches_oracle_sampled(dev, edge_gemm):
    """BASELINE config 4 at its full size (16 trajectories x 2521 nodes, the
    bench's launch geometry: 2521 edge tiles per layer over the persistent grid)
    against the oracle on sampled trajectories (first, middle, last; trajectories
    are independent, so the oracle on a subset is the full oracle restricted):
    the DMM mesh against autograd, the moved-mesh kNN-35 rows bit for bit and the
    step output at the parity tolerance."""
    from mmpde_amd import ops
    from mmpde_amd.rollout import MMPDERollout
    from mmpde_amd.synth import build_models, fields

    pde, model, model_b, itp, dmm, gc = build_models("cy")
    grid = pde.ori_grid
    B, N, step = 16, grid.shape[0], 7
    data = fields(grid, B, 30)[:, step - 1:step]
    sds = _sds(model=model, model_b=model_b, itp=itp, dmm=dmm)
    for m in (model, model_b, itp, dmm):
        m.to(dev)
    model.edge_gemm = model_b.edge_gemm = edge_gemm
    eng = MMPDERollout("cy", model, model_b, itp, dmm, gc, B, dev)
    pred = eng.step(data[:, 0].to(dev), step).cpu().reshape(B, N)
    torch.cuda.synchronize()
    mesh = eng.mesh.cpu().reshape(B, N, 2)
    # the rollout's own moved-mesh tables (candidate path), whole batch against
    # the full search, sampled trajectories against the oracle below
    nbr = eng.nbr_m.long().cpu().reshape(B, N, 35)
    idx2 = eng.idx2.long().cpu().reshape(B, N, 30)
    assert torch.equal(eng.nbr_m, ops.knn_graph_nbr(eng.mesh, B, 35))
    assert torch.equal(eng.idx2, ops.knn_query(eng.mesh, eng.grid_rep, B, 30))
    share = eng.knn_table_share()
    print(f"full size: candidate tables answered {share[0]:.4f} (graph) {share[1]:.4f} (query)")
    # the same tables at bench geometry with one trajectory moved far: the
    # fallback runs inside the B = 16 launch, bit for bit
    far = eng.mesh.clone().reshape(B, N, 2)
    far[5] += 0.04 * torch.sin(11 * far[5].flip(1))
    far = far.reshape(-1, 2)
    cells = ops.knn_moved_cells(far, eng.xi, B)
    nbr_far = ops.knn_graph_moved(far, eng.xi, eng.knn_cand, B, 35, cells=cells)
    fs = ops.knn_table_share(cells, B, N)[:, 0]
    print(f"far trajectory: table share {fs[5].item():.3f}, others min {fs[torch.arange(B) != 5].min().item():.3f}")
    assert fs[5] < 0.9
    assert torch.equal(nbr_far, ops.knn_graph_nbr(far, B, 35))
    idx_far = ops.knn_query_moved(far, eng.grid_rep, eng.xi, eng.knn_cand_q, B, 30, ref=eng.grid,
                                  cells=cells)
    assert torch.equal(idx_far, ops.knn_query(far, eng.grid_rep, B, 30))
    pick = [0, 7, 15]
    sub = data[pick]
    ref_x, ref_y = refcpu.moving_mesh_tri(sds["dmm"], sub.reshape(len(pick), -1),
                                          grid[None, :, 0].repeat(len(pick), 1),
                                          grid[None, :, 1].repeat(len(pick), 1), grid)
    ref_mesh = torch.cat((ref_x, ref_y), -1).reshape(len(pick), N, 2)
    _close(mesh[pick], ref_mesh, 1e-5, 1e-6, "full-size DMM mesh")
    for i, b in enumerate(pick):
        _, ref_nbr, _ = refcpu.knn_graph(mesh[b], 35, 1)
        assert torch.equal(nbr[b] - b * N, ref_nbr), f"kNN-35 rows of trajectory {b}"
        ref_idx = refcpu.knn_query(mesh[b], grid, 1, 30)
        assert torch.equal(idx2[b], ref_idx.reshape(N, 30)), f"kNN-30 rows of trajectory {b}"
    opde = refcpu.PDEConst("cy", [30, N], ori_grid=grid)
    ref, aux = refcpu.mmpde_step(opde, sds, sub, sub, [step] * len(pick),
                                 mesh_override=mesh[pick].reshape(-1, 2))
    _close(pred[pick], ref, 2.5e-5, 1e-7, f"full-size mmpde step {edge_gemm}")
    # each GNN against its own output range (|out| ~ 2e-3, about 1 % of the summed
    # step's range): an error in a GNN cannot hide under res_cut / interpolation
    out_u = eng.out_u.cpu().reshape(B, N)[pick]
    out_b = eng.out_b.cpu().reshape(B, N)[pick]
    _close(out_u, aux["out_u"], 1e-5, 1e-9, f"full-size model(graph_uni) {edge_gemm}")
    _close(out_b, aux["out_b"], 1e-5, 1e-9, f"full-size model_b(graph) {edge_gemm}")


def test_full_size_burgers_step_properties_and_oracle(dev):
    """BASELINE config 2 at its full size (32 trajectories x 48 x 48 nodes,
    array-mode DMM, mode-'1' interpolation onto the moved mesh, Conv2d res_cut):
    kNN validity on every trajectory's moved mesh, bitwise determinism, a finite
    30-step autoregressive rollout, and the step against the oracle on sampled
    trajectories (mesh vs autograd, moved-mesh kNN-35 rows bit for bit, each GNN
    against its own range, the summed step)."""
    from mmpde_amd import ops
    from mmpde_amd.rollout import MMPDERollout
    from mmpde_amd.synth import build_models, burgers_grid_points, fields

    pde, model, model_b, itp, dmm, gc = build_models("burgers")
    B, s, step = 32, 48, 11
    N = s * s
    u_all = fields(burgers_grid_points(), B, 31).reshape(B, 31, s, s)
    data = u_all[:, step - 1:step]
    sds = _sds(model=model, model_b=model_b, itp=itp, dmm=dmm)
    for m in (model, model_b, itp, dmm):
        m.to(dev)
    for m in (model, model_b):
        m.edge_gemm = "f16x3"
    eng = MMPDERollout("burgers", model, model_b, itp, dmm, gc, B, dev)
    u0 = data[:, 0].to(dev).contiguous()
    p1 = eng.step(u0, step)
    mesh = eng.mesh.clone()
    out_u, out_b = eng.out_u.clone(), eng.out_b.clone()
    # the rollout's own moved-mesh tables (candidate path): kNN-35 graph, kNN-30
    # of the moved mesh onto the grid (mode '1') and of the grid onto the
    # moved mesh (mode '2', the grid in 'ij' order against the 'xy' mesh)
    torch.cuda.synchronize()
    nbr_m, idx1, idx2 = eng.nbr_m.clone(), eng.idx1.clone(), eng.idx2.clone()
    share = eng.knn_table_share()
    print(f"burgers: candidate tables answered {share[0]:.4f} (graph) {share[1]:.4f} (query), "
          f"{share[2]:.4f} (mode-1 query)")
    assert share[1] > 0.9     # the query table is built for the grid's own order
    assert torch.equal(nbr_m, ops.knn_graph_nbr(mesh, B, 35))
    assert torch.equal(idx1, ops.knn_query(eng.grid_rep, mesh, B, 30))
    assert torch.equal(idx2, ops.knn_query(mesh, eng.grid_rep, B, 30))
    p2 = eng.step(u0, step)
    assert torch.equal(p1, p2)                                  # bitwise deterministic
    nbr = nbr_m.long().cpu()
    rows = torch.arange(B * N)[:, None]
    assert ((nbr // N) == rows // N).all() and (nbr != rows).all()
    m = mesh.cpu().double()
    d = ((m[nbr] - m[:, None, :]) ** 2).sum(-1)
    # sorted by the fp32 key (fmaf(dy, dy, dx*dx)): in fp64 the near-uniform grid's
    # near-ties may swap by an fp32 rounding (exact order: oracle rows below)
    assert (d[:, 1:] >= d[:, :-1] * (1 - 1e-6)).all()
    pick = [0, 13, 31]
    mesh_c = mesh.cpu().reshape(B, N, 2)
    opde = refcpu.PDEConst("burgers", [31, s, s])
    sub = data[pick]
    ox, oy = refcpu.moving_mesh(sds["dmm"], opde, sub.reshape(len(pick), s, s), s, s)
    _close(mesh_c[pick], torch.cat((ox, oy), -1), 0.0, 2e-6, "full-size burgers DMM mesh")
    grid_c = eng.grid.cpu()
    for b in pick:
        _, ref_nbr, _ = refcpu.knn_graph(mesh_c[b], 35, 1)
        assert torch.equal(nbr.reshape(B, N, 35)[b] - b * N, ref_nbr), f"kNN-35 rows of {b}"
        r1 = refcpu.knn_query(grid_c, mesh_c[b], 1, 30).reshape(N, 30)
        assert torch.equal(idx1.long().cpu().reshape(B, N, 30)[b], r1), f"kNN-30 (mode 1) rows of {b}"
        r2 = refcpu.knn_query(mesh_c[b], grid_c, 1, 30).reshape(N, 30)
        assert torch.equal(idx2.long().cpu().reshape(B, N, 30)[b], r2), f"kNN-30 (mode 2) rows of {b}"
    ref, aux = refcpu.mmpde_step(opde, sds, sub, sub, [step] * len(pick),
                                 mesh_override=mesh_c[pick].reshape(-1, 2))
    _close(p1.cpu().reshape(B, N)[pick], ref, 2.5e-5, 1e-7, "full-size burgers step")
    _close(out_u.cpu().reshape(B, N)[pick], aux["out_u"], 1e-5, 1e-9, "full-size burgers model")
    _close(out_b.cpu().reshape(B, N)[pick], aux["out_b"], 1e-5, 1e-9, "full-size burgers model_b")
    u = eng.rollout(u0, 1, 30)
    assert torch.isfinite(u).all()
