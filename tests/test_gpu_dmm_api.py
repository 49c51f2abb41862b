"""GPU parity of the DMM API surfaces outside the MM-PDE step, against the CPU
oracle (reference mesh/dmm_model.py, data_creator_2d.py:88-113):

- DMM.forward -> phi (and rf=True's second output), graph and array mode, on
  a grid that is NOT the branch's grid (the trunk runs on any rows);
- DenseNet.forward (trunk, decoding_mlp) and ConvNet.forward (array branch);
- F.interpolate(bilinear, align_corners=True) (mmpde_resample_bilinear) and
  GraphCreator_FS_2D.moving_mesh with the pre-resampling of u to a DMM grid
  of another size (data_creator_2d.py:102-103).

Bars: phi / DenseNet / ConvNet 2e-5 of max|ref| + 1e-6 (fp32 chains of tanh
layers; observed errors are ~1e-7 relative); resampling 1e-6 absolute on O(1)
values; the moved mesh 2e-6 absolute (coordinates in [0, 1]), the bar of
test_gpu_api.py.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import refcpu

pytestmark = pytest.mark.gpu


def _close(got, ref, rtol, atol=0.0, what=""):
    got = got.detach().double().cpu().reshape(-1)
    ref = ref.detach().double().cpu().reshape(-1)
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    err = (got - ref).abs().max().item()
    bound = rtol * ref.abs().max().item() + atol
    print(f"{what}: max|err| {err:.3e} bound {bound:.3e} max|ref| {ref.abs().max().item():.3e}")
    assert err <= bound, (what, err, bound)


def _dmm(kind):
    from mmpde_amd.synth import build_models

    pde, _, _, _, dmm, gc = build_models(kind, seed=3)
    dmm.eval()
    sd = {k: v.detach().cpu() for k, v in dmm.state_dict().items()}
    return pde, dmm, gc, sd


def _u(kind, pde, B, seed=5):
    from mmpde_amd.synth import burgers_grid_points, fields

    if kind == "cy":
        return fields(pde.ori_grid, B, 3, seed=seed)[:, 1]              # [B, N]
    return fields(burgers_grid_points(), B, 3, seed=seed)[:, 1].reshape(B, 48, 48)


@pytest.mark.parametrize("kind", ["cy", "burgers"])
def test_dmm_forward_phi_vs_oracle(dev, kind):
    pde, dmm, gc, sd = _dmm(kind)
    B = 2
    u = _u(kind, pde, B)
    g = torch.Generator().manual_seed(11)
    if kind == "cy":
        base = pde.ori_grid
    else:
        base = gc.xi_grid_xy(48, 48, "cpu")
    # m rows per trajectory, perturbed off the branch's grid
    grid = (base.repeat(B, 1) + 0.01 * torch.randn(B * base.shape[0], 2, generator=g)).float()
    ref = refcpu.dmm_forward(sd, "graph" if kind == "cy" else "array", u, grid,
                             ori_grid=pde.ori_grid if kind == "cy" else None)
    dmm.to(dev)
    phi = dmm(u.to(dev), grid.to(dev))
    assert phi.shape == ref.shape == (B * base.shape[0], 1)
    _close(phi, ref, 2e-5, 1e-6, f"{kind} DMM.forward phi")
    phi2, second, ones = dmm(u.to(dev), grid.to(dev), rf=True)
    assert torch.equal(phi2, phi), "rf=True phi differs"
    L2 = dmm.out_nn.layers[1]
    assert second.shape == (grid.shape[0], L2.in_features)
    assert ones.shape == (second.numel(), 1) and bool((ones == 1).all())
    # second_out is the tanh layer that produced phi
    lin = second.double().cpu() @ L2.weight.detach().double().cpu().t() + L2.bias.detach().double().cpu()
    _close(phi, lin, 1e-6, 1e-6, f"{kind} phi = out_nn.layers.1(second_out)")
    assert float(second.abs().max()) <= 1.0


def test_densenet_convnet_forward_vs_oracle(dev):
    _, dmm_c, _, sd_c = _dmm("cy")
    _, dmm_b, _, sd_b = _dmm("burgers")
    g = torch.Generator().manual_seed(2)
    x = torch.rand(5000, 2, generator=g)                      # > 4096 rows: two row blocks
    dmm_c.to(dev)
    out, hid = dmm_c.trunk(x.to(dev))
    rout, rhid = refcpu.densenet(sd_c, "trunk", x, 2)
    _close(out, rout, 2e-5, 1e-6, "trunk DenseNet out")
    _close(hid, rhid, 2e-5, 1e-6, "trunk DenseNet hidden")
    h = torch.randn(300, 4, generator=g)
    out, hid = dmm_c.decoding_mlp(h.to(dev))
    rout, rhid = refcpu.densenet(sd_c, "decoding_mlp", h, 2)
    _close(out, rout, 2e-5, 1e-6, "decoding_mlp DenseNet out")
    _close(hid, rhid, 2e-5, 1e-6, "decoding_mlp DenseNet hidden")
    u = torch.randn(3, 1, 48, 48, generator=g)
    dmm_b.to(dev)
    br = dmm_b.branch(u.to(dev))
    rbr = refcpu.convnet(sd_b, "branch", u)
    assert br.shape == rbr.shape == (3, 512)
    _close(br, rbr, 2e-5, 1e-6, "ConvNet.forward")
    dmm_b.train()       # DMM training's differentiable torch path (no BatchNorm inside)
    _close(dmm_b.branch(u.to(dev)), rbr, 2e-5, 1e-6, "ConvNet.forward (train mode)")


def _bilinear_f32(x, oh, ow):
    """align_corners=True bilinear in fp32 step by step: scale (in-1)/(out-1)
    in fp32, source coordinate = rounded fp32 product, lambdas, then
    hy (hx a + lx b) + ly (hx c + lx d) (PyTorch's upsample_bilinear2d)."""
    x = x.numpy()
    h, w = x.shape[-2:]
    f32 = np.float32

    def coord(n_in, n_out):
        sc = f32(n_in - 1) / f32(n_out - 1) if n_out > 1 else f32(0)
        c = np.array([f32(sc * f32(i)) for i in range(n_out)], dtype=np.float32)
        i0 = c.astype(np.int64)
        i1 = np.minimum(i0 + 1, n_in - 1)
        lam = (c - i0.astype(np.float32)).astype(np.float32)
        return i0, i1, lam, (f32(1) - lam).astype(np.float32)

    y0, y1, ly, hy = coord(h, oh)
    x0, x1, lx, hx = coord(w, ow)
    a, b = x[:, y0][:, :, x0], x[:, y0][:, :, x1]
    c, d = x[:, y1][:, :, x0], x[:, y1][:, :, x1]
    hy, ly = hy[:, None], ly[:, None]
    return torch.from_numpy(hy * (hx * a + lx * b) + ly * (hx * c + lx * d))


@pytest.mark.parametrize("size", [(32, 40), (64, 64), (1, 7), (48, 48)])
def test_resample_bilinear_vs_torch(dev, size):
    """Against the fp32 step-by-step restatement and torch's CPU F.interpolate
    (which agree to 2.4e-7).  The kernel forms the same fp32 source coordinates
    (tools/resample_diag.py: identical on ramps) but its blend is contracted
    differently: up to 2.7e-6 of max|ref| measured, bar 5e-6."""
    from mmpde_amd import ops

    g = torch.Generator().manual_seed(size[0])
    u = torch.randn(3, 48, 48, generator=g)
    got = ops.resample_bilinear(u.to(dev), *size)
    _close(got, _bilinear_f32(u, *size), 5e-6, 1e-6, f"bilinear 48x48 -> {size} (fp32 restatement)")
    ref = F.interpolate(u[:, None], size=size, mode="bilinear", align_corners=True)[:, 0]
    _close(got, ref, 5e-6, 1e-6, f"bilinear 48x48 -> {size} (torch CPU)")


def test_moving_mesh_with_resampling_vs_oracle(dev):
    """Data on a 32 x 32 grid, DMM trained at 48 x 48 (pde.movingmesh_grid_size):
    xi is the 32 x 32 grid and u is resampled to 48 x 48 first."""
    from mmpde_amd.synth import fields

    pde, dmm, gc, sd = _dmm("burgers")
    B = 2
    gx = np.linspace(0, 1, 32)
    pts = torch.tensor(np.array(np.meshgrid(gx, gx, indexing="ij")), dtype=torch.float
                       ).reshape(2, -1).t()
    u = fields(pts, B, 3, seed=9)[:, 1].reshape(B, 32, 32)
    opde = refcpu.PDEConst("burgers", (31, 32, 32))
    opde.movingmesh_grid_size = (31, 48, 48)
    gc.pde.movingmesh_grid_size = [31, 48, 48]
    rx, ry = refcpu.moving_mesh(sd, opde, u, 32, 32)
    dmm.to(dev)
    x1, x2 = gc.moving_mesh(u.to(dev), dmm, 32, 32)
    assert x1.shape == rx.shape == (B * 1024, 1)
    _close(x1, rx, 0.0, 2e-6, "moving_mesh x1 (resampled u)")
    _close(x2, ry, 0.0, 2e-6, "moving_mesh x2 (resampled u)")
