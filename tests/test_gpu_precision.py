"""Arithmetic of the message_net_2 edge GEMM: exact fp32 MFMA ("f32") vs the
fp32-emulating fp16 hi/lo split ("f16x3", include/mmpde_hip.h).

Both are measured against a float64 evaluation of the same oracle
(oracle/refcpu.py run on float64 weights and inputs), beside the CPU fp32
oracle itself (the reference's own fp32 arithmetic, torch CPU).  The bar for
f16x3: its error vs fp64 is within 4x of the larger of the two fp32 errors,
and inside the fp32 parity tolerance of tests/test_gpu_parity.py.
"""
import pytest
import torch

from oracle import refcpu

pytestmark = pytest.mark.gpu


def _gnn_case(kind, B, seed=0):
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
def test_edge_gemm_f16x3_vs_fp64(dev, kind):
    from mmpde_amd.rollout import _Nodes

    pde, model, u, pos, ei, nbr = _gnn_case(kind, 2)
    opde = refcpu.PDEConst(kind, pde.grid_size, ori_grid=getattr(pde, "ori_grid", None))
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
    ref64 = refcpu.mp_pde_solver(sd64, opde, u.double(), pos.double(), ei).reshape(-1)
    ref32 = refcpu.mp_pde_solver(sd, opde, u, pos, ei).reshape(-1).double()
    model.to(dev)
    g = _Nodes(u.to(dev), pos.to(dev), nbr.int().to(dev))
    outs = {"cpu-f32": ref32}
    for mode in ("f32", "f16x3"):
        model.edge_gemm = mode
        outs[mode] = model(g).reshape(-1).double().cpu()
    model.edge_gemm = "f32"
    errs = {m: (o - ref64).abs().max().item() for m, o in outs.items()}
    rms = {m: (o - ref64).pow(2).mean().sqrt().item() for m, o in outs.items()}
    scale = ref64.abs().max().item()
    print(f"{kind}: max|ref| {scale:.3e}; vs fp64 max|err| / rms err: "
          + ", ".join(f"{m} {errs[m]:.3e} / {rms[m]:.3e}" for m in outs)
          + f"; f16x3 vs f32 max|diff| {(outs['f16x3'] - outs['f32']).abs().max().item():.3e}")
    assert errs["f16x3"] <= 4.0 * max(errs["f32"], errs["cpu-f32"]) + 1e-12
    assert rms["f16x3"] <= 4.0 * max(rms["f32"], rms["cpu-f32"]) + 1e-12
    assert errs["f16x3"] <= 2e-4 * scale + 1e-7


def test_edge_gemm_f16x3_mmpde_step(dev):
    """Whole cylinder MM-PDE step with the split edge GEMM in both GNNs, against
    the fp32 oracle at the parity tolerance of test_mmpde_step_matches_oracle."""
    from mmpde_amd.rollout import MMPDERollout
    from mmpde_amd.synth import build_models, fields

    B, step = 2, 5
    pde, model, model_b, itp, dmm, gc = build_models("cy")
    grid = pde.ori_grid
    data = fields(grid, B, 30)[:, step - 1:step]
    sds = {k: {n: t.detach().cpu() for n, t in m.state_dict().items()}
           for k, m in (("model", model), ("model_b", model_b), ("itp", itp), ("dmm", dmm))}
    for m in (model, model_b, itp, dmm):
        m.to(dev)
    model.edge_gemm = model_b.edge_gemm = "f16x3"
    eng = MMPDERollout("cy", model, model_b, itp, dmm, gc, B, dev)
    pred = eng.step(data[:, 0].to(dev), step).cpu().reshape(-1)
    mesh = eng.mesh.cpu()
    opde = refcpu.PDEConst("cy", [30, grid.shape[0]], ori_grid=grid)
    ref, _ = refcpu.mmpde_step(opde, sds, data, data, [step] * B, mesh_override=mesh)
    err = (pred - ref.reshape(-1)).abs().max().item()
    bound = 2.5e-5 * ref.abs().max().item() + 1e-7
    print(f"mmpde step f16x3: max|err| {err:.3e} bound {bound:.3e}")
    assert err <= bound
