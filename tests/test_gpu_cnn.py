"""BaseCNN baseline (reference models_cnn.py:8-83, ``--model BaseCNN``) on the
HIP conv kernels against the CPU oracle: circular padding, ELU, the
post-activation residuals and the cumsum(dt) output, for the reference's
default time_window 1 (mmpde.py:363-364) and the class default 25.
Bar: 2e-5 of max|ref| + 1e-6 (fp32 sums of up to 40 x 81 products per output).
Also: the seeded construction reproduces torch's own nn.Conv2d init order
(state_dict keys / shapes as the reference's).

Training (train_helper_2d.py:107-125, the non-GNN branch of
training_loop_branch; reference models_cnn.py:66-83 under loss.backward()):
the conv weight gradient kernel against torch autograd (zero and circular
padding, ks 3 / 5 / 9: 1e-5 of max|ref| + 1e-6), and every parameter gradient
of a BaseCNN training step against float64 autograd through the oracle:
relative L2 <= max(1e-4, 2 x the fp32 oracle's own); the loop runs seeded,
finite and reproducible bit for bit."""
import pytest
import torch

from oracle import refcpu

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("tw,B", [(1, 2), (25, 2), (1, 1)])
def test_basecnn_forward_vs_oracle(dev, tw, B):
    from mmpde_amd import BaseCNN, burgers

    pde = burgers()
    torch.manual_seed(0)
    m = BaseCNN(pde, time_window=tw, hidden_channels=40).eval()
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    assert sorted(sd) == sorted([f"conv{i}.{p}" for i in range(1, 9) for p in ("weight", "bias")])
    g = torch.Generator().manual_seed(tw + B)
    u = torch.randn(B, tw, 48, 48, generator=g)
    ref = refcpu.basecnn(sd, pde.dt, u, tw)
    m.to(dev)
    out = m(u.to(dev))
    assert out.shape == ref.shape
    err = (out.cpu().double() - ref.double()).abs().max().item()
    bound = 2e-5 * ref.abs().max().item() + 1e-6
    print(f"BaseCNN tw={tw} B={B}: max|err| {err:.3e} bound {bound:.3e}")
    assert err <= bound


def test_conv2d_circular_elu_residual_vs_torch(dev):
    from mmpde_amd import _lib as L, ops
    import torch.nn.functional as F

    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 6, 13, 11, generator=g)
    w = torch.randn(6, 6, 5, 5, generator=g) * 0.2
    b = torch.randn(6, generator=g)
    ref = x + F.elu(F.conv2d(F.pad(x, (2, 2, 2, 2), mode="circular"), w, b))
    got = ops.conv2d(x.to(dev), w.to(dev), b.to(dev), 1, 2, L.ACT_ELU, residual=x.to(dev), circular=True,
                     res_after_act=True)
    assert (got.cpu() - ref).abs().max().item() <= 2e-5 * ref.abs().max().item()


@pytest.mark.parametrize("ks,circ", [(3, True), (5, False), (9, True), (9, False)])
def test_conv2d_grad_weight_vs_autograd(dev, ks, circ):
    from mmpde_amd import ops
    import torch.nn.functional as F

    g = torch.Generator().manual_seed(ks)
    x = torch.randn(3, 5, 12, 10, generator=g, dtype=torch.float64)
    w = (torch.randn(4, 5, ks, ks, generator=g, dtype=torch.float64) * 0.1).requires_grad_()
    b = torch.randn(4, generator=g, dtype=torch.float64).requires_grad_()
    p = ks // 2
    xx = F.pad(x, (p, p, p, p), mode="circular") if circ else F.pad(x, (p, p, p, p))
    y = F.conv2d(xx, w, b)
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    y.backward(dy)
    dw, db = ops.conv2d_grad_weight(x.float().to(dev), dy.float().to(dev), ks, p, circ)
    for got, ref in ((dw, w.grad), (db, b.grad)):
        err = (got.cpu().double() - ref).abs().max().item()
        assert err <= 1e-5 * ref.abs().max().item() + 1e-6, err
    # the input gradient: the same convolution of dy with the flipped kernel
    xg = x.clone().float().to(dev).requires_grad_()
    wg = w.detach().float().to(dev).requires_grad_()
    out = ops.Conv2dSame.apply(xg, wg, b.detach().float().to(dev), circ)
    out.backward(dy.float().to(dev))
    xr = x.clone().requires_grad_()
    xxr = F.pad(xr, (p, p, p, p), mode="circular") if circ else F.pad(xr, (p, p, p, p))
    F.conv2d(xxr, w.detach(), b.detach()).backward(dy)
    err = (xg.grad.cpu().double() - xr.grad).abs().max().item()
    assert err <= 1e-5 * xr.grad.abs().max().item() + 1e-6, err


def _rel_l2(a, b):
    a, b = a.detach().double().cpu().reshape(-1), b.detach().double().cpu().reshape(-1)
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


@pytest.mark.parametrize("tw,B", [(1, 4), (25, 2)])
def test_basecnn_training_gradients_vs_fp64(dev, tw, B):
    from mmpde_amd import BaseCNN, burgers

    pde = burgers()
    torch.manual_seed(1)
    m = BaseCNN(pde, time_window=tw, hidden_channels=40)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    g = torch.Generator().manual_seed(7 + tw)
    u = torch.randn(B, tw, 48, 48, generator=g)
    lab = torch.randn(B, 1, tw, 48, 48, generator=g)
    m.to(dev).train()
    loss = torch.nn.functional.mse_loss(m(u.to(dev)), lab.to(dev).squeeze())
    loss.backward()
    grads = {n: p.grad for n, p in m.named_parameters()}

    def oracle(dtype):
        sdt = {k: v.to(dtype).requires_grad_() for k, v in sd.items()}
        out = refcpu.basecnn(sdt, pde.dt, u.to(dtype), tw)
        l = torch.nn.functional.mse_loss(out, lab.to(dtype).squeeze())
        l.backward()
        return l, {k: v.grad for k, v in sdt.items()}

    l64, g64 = oracle(torch.float64)
    _, g32 = oracle(torch.float32)
    assert abs(loss.item() - l64.item()) <= 1e-5 * abs(l64.item())
    for n, gg in grads.items():
        e = _rel_l2(gg, g64[n])
        e32 = _rel_l2(g32[n], g64[n])
        print(f"BaseCNN tw={tw} {n}: rel-L2 {e:.2e} (fp32 oracle {e32:.2e})")
        assert e <= max(1e-4, 2 * e32), (n, e, e32)


def test_basecnn_training_loop_reproducible(dev):
    """training_loop_branch's non-GNN branch (train_helper_2d.py:107-125) with
    BaseCNN and AdamW, twice from the same seed: finite losses, identical bit
    for bit (every kernel of the step is deterministic)."""
    import random

    from mmpde_amd import BaseCNN, burgers
    from mmpde_amd.data_creator_2d import GraphCreator_FS_2D
    from mmpde_amd.train import training_loop_branch

    pde = burgers()
    pde.grid_size = pde.movingmesh_grid_size = pde.ori_grid_size = [31, 48, 48]
    g = torch.Generator().manual_seed(3)
    u = torch.randn(4, 31, 48, 48, generator=g) * 0.5

    def run():
        torch.manual_seed(0)
        m = BaseCNN(pde, time_window=1, hidden_channels=40).to(dev).train()
        opt = torch.optim.AdamW(m.parameters(), lr=1e-3)
        gc = GraphCreator_FS_2D(pde, neighbors=35, time_window=1, t_resolution=31)
        loader = torch.utils.data.DataLoader(torch.utils.data.TensorDataset(u, u), batch_size=2, shuffle=False)
        random.seed(5)
        ls = torch.cat([training_loop_branch(m, None, None, None, [0], 2, opt, None, loader, gc,
                                             torch.nn.MSELoss(), dev) for _ in range(2)])
        return ls.cpu(), {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}

    l1, p1 = run()
    l2, p2 = run()
    assert torch.isfinite(l1).all() and l1.numel() == 4
    assert torch.equal(l1, l2)
    assert all(torch.equal(p1[k], p2[k]) for k in p1)
