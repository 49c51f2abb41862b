"""Skinny linear (mmpde_linear_skinny_ws, dense.hip): the res_cut / DMM-branch
GEMMs with K split over the chip and the partial tiles added in z order inside
the launch.

Bar: exact-fp32 products, so max|err| vs float64 <= 1e-6 x (1 + |ref|max)
times sqrt(k)/sqrt(512) slack; repeated calls bit-identical; one workspace
reused across shapes (the cylinder res_cut chain 2521-2048-512-2048-2521, then
shapes whose partial tiles cover other shapes' ticket words) stays exact and
leaves its ticket words at zero.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(16, 2521, 2048), (16, 2048, 2521), (3, 2048, 2521), (3, 2521, 2048), (2, 512, 2048),
          (32, 2521, 512), (2, 4096, 64), (1, 100, 7), (64, 1024, 1000)]


def _ref(x, w, b, act):
    r = x.double() @ w.double().t() + b.double()
    return torch.tanh(r) if act == 1 else r


def _bound(ref, k):
    return 1e-6 * (1 + ref.abs().max().item()) * max(1.0, math.sqrt(k / 512))


@pytest.mark.parametrize("m,k,n", SHAPES)
def test_linear_skinny_vs_fp64(dev, m, k, n):
    from mmpde_amd import ops

    g = torch.Generator().manual_seed(m * 7 + k + n)
    x = torch.randn(m, k, generator=g).to(dev)
    w = (torch.randn(n, k, generator=g) * 0.02).to(dev)
    b = torch.randn(n, generator=g).to(dev)
    for act in (0, 1):
        ref = _ref(x, w, b, act)
        outs = [ops.linear_skinny(x, w, b, act) for _ in range(3)]
        err = (outs[0].double() - ref.to(dev)).abs().max().item()
        assert err <= _bound(ref, k), (m, k, n, act, err)
        assert all(torch.equal(outs[0], o) for o in outs[1:]), "run-to-run"


def test_linear_skinny_workspace_reuse(dev):
    from mmpde_amd import _lib as L, ops

    g = torch.Generator().manual_seed(3)
    widths = [2521, 2048, 512, 2048, 2521]
    layers = [((torch.randn(b_, a_, generator=g) * 0.02).to(dev), torch.randn(b_, generator=g).to(dev))
              for a_, b_ in zip(widths, widths[1:])]
    for m in (2, 3, 16):
        x = torch.randn(m, 2521, generator=g).to(dev)
        for _ in range(2):
            h, r = x, x.double()
            for i, (w, b) in enumerate(layers):
                act = 1 if i < 3 else 0
                h = ops.linear_skinny(h, w, b, act)
                r = _ref(r, w, b, act)
                err = (h.double() - r).abs().max().item()
                assert err <= _bound(r, w.shape[1]), (m, i, err)
    torch.cuda.synchronize()
    assert L.lib().mmpde_linear_skinny_workspace_bytes(16, 2521, 2048) > 4096 * 4
    for ws in ops._SKINNY_WS.values():
        assert int(ws[:4096].view(torch.int32).abs().sum()) == 0, "ticket words left non-zero"


@pytest.mark.parametrize("m", [600, 40])
def test_linear_skinny_rows_independent(dev, m):
    """A row's result does not depend on the rows launched beside it (the K
    split depends on (n, k) only): the res_cut shape at m = 600 (more output
    tiles than one split launch's ticket block: row blocks of the same split)
    and m = 40, every row slice bitwise equal to the full launch."""
    from mmpde_amd import ops

    g = torch.Generator().manual_seed(11)
    x = torch.randn(m, 2048, generator=g).to(dev)
    w = (torch.randn(2521, 2048, generator=g) * 0.02).to(dev)
    b = torch.randn(2521, generator=g).to(dev)
    full = ops.linear_skinny(x, w, b, 1)
    ref = _ref(x, w, b, 1)
    assert (full.double() - ref).abs().max().item() <= _bound(ref, 2048)
    for lo, hi in ((0, 8), (8, 16), (5, 6), (m - 3, m)):
        assert torch.equal(full[lo:hi], ops.linear_skinny(x[lo:hi].contiguous(), w, b, 1)), (lo, hi)
