"""MP_PDE_Solver_2D with time_window > 1: u has tw
channels (embedding input tw + 3, message_net_1 input 256 + tw + 3) and the
head scales one output by cumsum(dt * 0.1) into tw (gnn_2d.py:72-141).
Against the oracle's op-for-op forward, both edge-GEMM modes."""
import pytest
import torch

from oracle import refcpu


def _solver(tw, seed):
    from mmpde_amd.gnn_2d import MP_PDE_Solver_2D
    from mmpde_amd.synth import _randomise_bn, cy_synth_mesh
    from mmpde_amd.pdes import cy

    torch.manual_seed(seed)
    grid = cy_synth_mesh()
    pde = cy(ori_grid=grid)
    pde.grid_size = [30, grid.shape[0]]
    model = MP_PDE_Solver_2D(pde=pde, time_window=tw, eq_variables={})
    _randomise_bn(model, torch.Generator().manual_seed(seed + 1))
    return pde, model.eval()


def test_head_scales_and_padding_on_host():
    pde, model = _solver(3, 0)
    s = model.out_scales()
    assert s.shape == (3,) and torch.equal(s, torch.cumsum(torch.ones(1, 3) * pde.dt * 0.1, 1)[0])
    p = model.gnn_layers[0]._params()
    assert p.msg1_ld == 264                     # 259 + 3 columns padded to a multiple of 4


@pytest.mark.gpu
@pytest.mark.parametrize("tw,mode", [(2, "f32"), (2, "f16x3"), (5, "f16x3"), (1, "f16x3")])
def test_gnn_forward_time_window(dev, tw, mode):
    from mmpde_amd.graph import Data

    pde, model = _solver(tw, tw)
    B, N = 2, 200
    pts = torch.rand(B * N, 2)
    pos = torch.cat((torch.full((B * N, 1), 1.3), pts), 1)
    u = torch.randn(B * N, tw)
    ei, nbr, _ = refcpu.knn_graph(pts, 35, B)
    opde = refcpu.PDEConst("cy", pde.grid_size, ori_grid=pde.ori_grid)
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    ref = refcpu.mp_pde_solver(sd, opde, u, pos, ei, time_window=tw)
    assert ref.shape == (B * N, tw)
    model.to(dev)
    model.edge_gemm = mode
    g = Data(x=u.to(dev))
    g.pos = pos.to(dev)
    g.nbr = nbr.int().to(dev)
    out = model(g)
    assert out.shape == (B * N, tw)
    err = (out.cpu() - ref).abs().max().item()
    bound = 2e-4 * ref.abs().max().item() + 1e-7
    print(f"gnn tw={tw} {mode}: max|err| {err:.3e} bound {bound:.3e}")
    assert err <= bound
