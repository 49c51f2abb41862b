"""connect_edge='radius' (SURVEY.md §8(f) row 3): torch_cluster radius_graph and
the ragged-degree GNN built on it.

CPU tests pin the oracle's radius semantics on hand-checked cases and the host
table conversions; GPU tests compare the HIP radius kernel (bit-exact) and the
ragged-degree GNN (fp32 tolerance) with the oracle.  The torch_cluster boundary
is "parity unpinned" (no fixture, reference not runnable).
"""
import pytest
import torch

from oracle import refcpu


def test_radius_oracle_truncates_in_index_order():
    # 8 points on a line, spacing 1; r = 2.5 covers |i - j| <= 2.  With
    # max_num_neighbors = 2 the scan keeps the first 3 hits in index order,
    # itself included, then drops itself.
    x = torch.stack((torch.arange(8, dtype=torch.float32), torch.zeros(8)), 1)
    _, nbr, deg = refcpu.radius_graph(x, 2.5, 1, max_num_neighbors=2)
    assert nbr[0].tolist() == [1, 2, -1] and deg[0] == 2      # hits 0,1,2 -> self dropped
    assert nbr[3].tolist() == [1, 2, -1] and deg[3] == 2      # hits 1,2,3 (4, 5 cut)
    assert nbr[7].tolist() == [5, 6, -1] and deg[7] == 2      # hits 5,6,7
    _, nbr, deg = refcpu.radius_graph(x, 2.5, 1, max_num_neighbors=32)
    assert nbr[3, :4].tolist() == [1, 2, 4, 5] and deg[3] == 4
    # strict '<': a point exactly at distance r is outside
    _, nbr, deg = refcpu.radius_graph(x, 1.0, 1)
    assert deg.tolist() == [0] * 8


def test_radius_oracle_segments_and_edge_index():
    x = torch.tensor([[0.0, 0.0], [0.1, 0.0], [5.0, 5.0], [0.0, 0.0], [0.05, 0.0], [9.0, 9.0]])
    ei, nbr, deg = refcpu.radius_graph(x, 0.5, 2)
    assert deg.tolist() == [1, 1, 0, 1, 1, 0]
    assert nbr[:, 0].tolist() == [1, 0, -1, 4, 3, -1]          # never across segments
    assert ei.tolist() == [[1, 0, 4, 3], [0, 1, 3, 4]]          # source row 0, target row 1


def test_table_conversions_on_host():
    from mmpde_amd.ops import edge_index_from_nbr, nbr_table_from_edge_index

    ei = torch.tensor([[3, 1, 0, 2, 4, 1], [0, 2, 1, 2, 0, 0]])
    nbr, deg = nbr_table_from_edge_index(ei, 5)
    assert deg.tolist() == [3, 1, 2, 0, 0]
    assert nbr.tolist() == [[3, 4, 1], [0, -1, -1], [1, 2, -1], [-1] * 3, [-1] * 3]
    back = edge_index_from_nbr(nbr, deg)
    assert back.tolist() == [[3, 4, 1, 0, 1, 2], [0, 0, 0, 1, 2, 2]]
    fixed = torch.tensor([[1, 2, 0, 2, 0, 1], [0, 0, 1, 1, 2, 2]])
    nbr, deg = nbr_table_from_edge_index(fixed, 3)
    assert deg is None and nbr.tolist() == [[1, 2], [0, 2], [0, 1]]


def test_graph_creator_radius_value():
    from mmpde_amd.synth import build_models

    _, _, _, _, _, gc = build_models("burgers", moving_mesh=False)
    gc.e = "radius"
    x = torch.linspace(0, 1, 48)
    dx = x[1] - x[0]
    assert gc.radius() == float(35 * torch.sqrt(dx ** 2 + dx ** 2) + 0.0001)


# ------------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("case", ["mesh_saturated", "small_r", "tiny_r", "duplicates"])
def test_radius_graph_bit_exact(dev, case):
    from mmpde_amd import ops
    from mmpde_amd.synth import cy_synth_mesh

    torch.manual_seed(7)
    if case == "mesh_saturated":        # the reference's r covers the domain: 32/33 per row
        g = cy_synth_mesh()
        pts, B, r = torch.cat((g, g + 0.001 * torch.randn_like(g))), 2, 1.05
    elif case == "small_r":
        pts, B, r = torch.rand(3 * 700, 2), 3, 0.06
    elif case == "tiny_r":              # many empty rows
        pts, B, r = torch.rand(2 * 500, 2), 2, 0.01
    else:
        pts = torch.rand(400, 2)
        pts[100:180] = pts[3]          # 81 coincident points: saturation by index order
        B, r = 1, 0.05
    nbr, deg = ops.radius_graph_nbr(pts.to(dev), B, r, 32)
    _, rn, rd = refcpu.radius_graph(pts, r, B, 32)
    assert torch.equal(deg.cpu().long(), rd)
    assert torch.equal(nbr.cpu().long(), rn)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["f32", "f16x3"])
def test_gnn_forward_radius_graph(dev, mode):
    """Ragged in-degree (radius graph, 0..33 neighbours per node, partial edge
    tiles) against the oracle's PyG mean aggregation over the same edges."""
    from mmpde_amd.graph import Data
    from mmpde_amd.synth import build_models

    pde, model, _, _, _, _ = build_models("cy", moving_mesh=False, seed=4)
    B, N = 3, 301
    torch.manual_seed(11)
    pts = torch.rand(B * N, 2)
    pts[:60] = 0.5 + 0.01 * torch.rand(60, 2)     # a cluster: rows saturate at 32 / 33
    pts[N + 5] = torch.tensor([3.0, 3.0])           # an isolated node: degree 0
    pos = torch.cat((torch.full((B * N, 1), 0.9), pts), 1)
    u = torch.randn(B * N, 1)
    ei, nbr, deg = refcpu.radius_graph(pts, 0.09, B, 32)
    assert int(deg.min()) == 0 and int(deg.max()) == 33
    opde = refcpu.PDEConst("cy", pde.grid_size, ori_grid=pde.ori_grid)
    ref = refcpu.mp_pde_solver({k: v.detach().cpu() for k, v in model.state_dict().items()},
                               opde, u, pos, ei)
    model.to(dev)
    model.edge_gemm = mode
    g = Data(x=u.to(dev))
    g.pos = pos.to(dev)
    g.nbr = nbr.int().to(dev)
    g.deg = deg.int().to(dev)
    out = model(g)
    err = (out.cpu() - ref).abs().max().item()
    bound = 2e-4 * ref.abs().max().item() + 1e-7
    print(f"gnn radius {mode}: max|err| {err:.3e} bound {bound:.3e}")
    assert err <= bound
    # the same graph handed over as a PyG edge_index
    g2 = Data(x=u.to(dev), edge_index=ei.to(dev))
    g2.pos = pos.to(dev)
    out2 = model(g2)
    assert (out2.cpu() - ref).abs().max().item() <= bound


@pytest.mark.gpu
def test_graph_creator_radius(dev):
    from mmpde_amd.synth import build_models, fields

    pde, model, _, _, _, gc = build_models("cy", moving_mesh=False)
    gc.e = "radius"
    model.to(dev)
    B, step = 2, 3
    u = fields(pde.ori_grid, B, 30)
    data, labels = gc.create_data(u, [step] * B)
    graph = gc.create_graph(None, data, labels, [step] * B, dev, None)
    _, rn, rd = refcpu.radius_graph(pde.ori_grid.repeat(B, 1), gc.radius(), B, 32)
    assert torch.equal(graph.deg.cpu().long(), rd)
    assert torch.equal(graph.nbr.cpu().long(), rn)
    ei = graph.edge_index
    assert ei.shape[1] == int(rd.sum())
    assert torch.isfinite(model(graph)).all()
