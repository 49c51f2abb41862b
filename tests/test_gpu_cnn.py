"""BaseCNN baseline (reference models_cnn.py:8-83, ``--model BaseCNN``) on the
HIP conv kernels against the CPU oracle: circular padding, ELU, the
post-activation residuals and the cumsum(dt) output, for the reference's
default time_window 1 (mmpde.py:363-364) and the class default 25.
Bar: 2e-5 of max|ref| + 1e-6 (fp32 sums of up to 40 x 81 products per output).
Also: the seeded construction reproduces torch's own nn.Conv2d init order
(state_dict keys / shapes as the reference's), and train() raises."""
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
    m.train()
    with pytest.raises(NotImplementedError):
        m(u.to(dev))


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
