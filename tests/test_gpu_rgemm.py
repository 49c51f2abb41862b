"""Row GEMMs of the training path (csrc/rgemm.hip, mmpde_amd/rows.py): every
train-mode Linear of the GNN and ItpNet (gnn_2d.py:53-69,99-106,
interpolate.py:79-93) and their gradients, against float64 torch.

Bars: exact-fp32-product GEMMs with fp32 accumulation over K <= 2048 (or n
rows for the weight gradients, summed in fixed 256-row chunks): max|err| <=
2e-5 of max|ref| (1e-5 for K <= 260), the same order as torch's fp32 GEMMs.
Layer-level: GnnLayerTrain against float64 autograd through the oracle's
train-mode layer (oracle/refcpu.py gnn_layer, train=True).
"""
import pytest
import torch

from oracle import refcpu

pytestmark = pytest.mark.gpu


def _close(got, ref, rtol, what):
    got = got.detach().double().cpu()
    ref = ref.detach().double().cpu()
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    err = (got - ref).abs().max().item()
    scale = ref.abs().max().item()
    print(f"{what}: max|err| {err:.3e} max|ref| {scale:.3e}")
    assert err <= rtol * scale + 1e-30, (what, err, scale)


@pytest.mark.parametrize("n,k,nout", [(40336, 128, 128), (1000, 257, 128), (777, 62, 128), (5000, 128, 64),
                                      (3000, 64, 30), (300, 4, 128), (2049, 16, 4), (513, 132, 256),
                                      (64, 260, 300), (100, 3, 5)])
def test_linear_rows_vs_fp64(dev, n, k, nout):
    from mmpde_amd.ops import LinearRows

    g = torch.Generator().manual_seed(n + k + nout)
    x = torch.randn(n, k, generator=g)
    w = torch.randn(nout, k, generator=g) / k ** 0.5
    b = torch.randn(nout, generator=g)
    dy = torch.randn(n, nout, generator=g)
    ref = [t.double().requires_grad_() for t in (x, w, b)]
    yr = torch.addmm(ref[2], ref[0], ref[1].t())
    (yr * dy.double()).sum().backward()
    got = [t.to(dev).requires_grad_() for t in (x, w, b)]
    y = LinearRows.apply(*got)
    (y * dy.to(dev)).sum().backward()
    tol = 1e-5 if k <= 260 else 2e-5
    _close(y, yr, tol, f"y n={n} k={k} N={nout}")
    _close(got[0].grad, ref[0].grad, tol, "dx")
    _close(got[1].grad, ref[1].grad, 2e-5, "dW")
    _close(got[2].grad, ref[2].grad, 2e-5, "db")


def test_rgemm_masks_accumulate_and_small_segments(dev):
    """The fused forms GnnLayerTrain uses: two input tensors side by side, the
    <= 4-column small segment with a sign, ReLU, input / output ReLU-backward
    masks, accumulation into an existing output, two output parts."""
    from mmpde_amd import _lib as L
    from mmpde_amd import rows

    g = torch.Generator().manual_seed(7)
    n = 4133
    h, m = torch.randn(n, 128, generator=g), torch.randn(n, 128, generator=g)
    xs = torch.randn(n, 4, generator=g)
    w = torch.randn(128, 260, generator=g) / 16
    bias = torch.randn(128, generator=g)
    hd, md, xsd, wd, bd = (t.to(dev) for t in (h, m, xs, w, bias))
    P = rows._p
    st = L.stream(dev)
    # NT: y = relu([h | m] W[:, :256]^T + xs[:, 3] W[:, 256] + b); z = h W[:, 128:256]^T - xs[:, :3] W[:, 256:259]
    y = torch.empty(n, 128, device=dev)
    z = torch.empty(n, 128, device=dev)
    rows.rgemm(n, 128, L.RGEMM_NT, (P(wd), P(wd, 128)), 260, (P(hd), P(md)), (128, 128),
               [dict(out=P(y), ldo=128, ncols=128, bias=P(bd), ns=1, xw=P(wd, 256))],
               relu=True, xs=P(xsd, 3), ldxs=4, ldxw=260, stream=st)
    rows.rgemm(n, 64, L.RGEMM_NT, (P(wd), P(wd, 64)), 260, (P(hd), P(hd, 64)), (128, 128),
               [dict(out=P(z), ldo=128, wk=128, ncols=128, ns=3, xw=P(wd, 256), xscale=-1.0)],
               xs=P(xsd), ldxs=4, ldxw=260, stream=st)
    H, M, X, W, B = (t.double() for t in (h, m, xs, w, bias))
    yr = torch.relu(torch.cat((H, M), 1) @ W[:, :256].t() + X[:, 3:4] @ W[:, 256:257].t() + B)
    zr = H @ W[:, 128:256].t() - X[:, :3] @ W[:, 256:259].t()
    _close(y, yr, 1e-5, "NT two tensors + t + relu")
    _close(z, zr, 1e-5, "NT half + small segment with sign")
    # NN with an input mask, an output mask, two parts, one accumulating
    gr = torch.randn(n, 128, generator=g)
    up = torch.randn(n, 128, generator=g)
    vm = torch.randn(n, 128, generator=g)
    acc0 = torch.randn(n, 128, generator=g)
    grd, upd, vmd = gr.to(dev), up.to(dev), vm.to(dev)
    out0 = acc0.clone().to(dev)
    out1 = torch.empty(n, 128, device=dev)
    rows.rgemm(n, 64, L.RGEMM_NN, (P(wd), P(wd, 64 * 260)), 260, (P(grd), P(grd, 64)), (128, 128),
               [dict(out=P(out0), ldo=128, wc=0, ncols=128, acc=True),
                dict(out=P(out1), ldo=128, wc=128, ncols=128, omask=P(vmd), ldom=128)],
               amask=(P(upd), P(upd, 64)), stream=st)
    Gm = gr.double() * (up > 0).double()
    _close(out0, acc0.double() + Gm @ W[:, :128], 1e-5, "NN masked input, accumulate")
    _close(out1, (Gm @ W[:, 128:256]) * (vm > 0).double(), 1e-5, "NN output mask, second part")


def test_rgemm_tn_segments_and_signs(dev):
    from mmpde_amd import _lib as L
    from mmpde_amd import rows

    g = torch.Generator().manual_seed(9)
    n = 40336 + 17
    G = torch.randn(n, 128, generator=g)
    gm = torch.randn(n, 128, generator=g)
    h, m = torch.randn(n, 128, generator=g), torch.randn(n, 128, generator=g)
    xs = torch.randn(n, 4, generator=g)
    Gd, gmd, hd, md, xsd = (t.to(dev) for t in (G, gm, h, m, xs))
    P = rows._p
    dw = torch.full((128, 260), 0.5, device=dev)
    db = torch.empty(128, device=dev)
    rows.rgemm_tn(n, P(Gd), 128, 128, [(P(hd), 128, 128, 0), (P(md), 128, 128, 128)], dw, 260, db=db,
                  gmask=P(gmd), xs=P(xsd), ldxs=4, ns=3, dwcol_s=256, stream=L.stream(dev))
    rows.rgemm_tn(n, P(Gd), 128, 128, [(P(hd), 128, 128, 0)], dw, 260, xs=P(xsd), ldxs=4, ns=4,
                  dwcol_s=256, sign_s=-1.0, accumulate_s=True, gmask=P(gmd), stream=L.stream(dev))
    Gm = G.double() * (gm > 0).double()
    X = xs.double()
    ref = torch.empty(128, 260, dtype=torch.float64)
    ref[:, :128] = Gm.t() @ h.double()
    ref[:, 128:256] = Gm.t() @ m.double()
    ref[:, 256:260] = -(Gm.t() @ X)
    ref[:, 256:259] += Gm.t() @ X[:, :3]
    ref[:, 259] += 0.5                    # the first call's 3 columns left column 259 as it was
    _close(dw[:, :256], ref[:, :256], 2e-5, "TN segments")
    # 256:259 cancel to ~0 by construction: compare absolutely against the summands' scale
    err = (dw[:, 256:].double().cpu() - ref[:, 256:]).abs().max().item()
    assert err <= 2e-5 * (Gm.t().abs() @ X.abs()).max().item()
    _close(db, Gm.sum(0), 2e-5, "TN db")


@pytest.mark.parametrize("edge_gemm", ["f32", "f16x3"])
def test_gnn_layer_train_vs_fp64(dev, edge_gemm):
    """GnnLayerTrain (forward, input / weight / BatchNorm gradients, running
    statistics) against float64 autograd through refcpu.gnn_layer(train=True),
    on a cy kNN-35 graph; u requires grad (the Burgers path, where ItpNet
    interpolates u onto the moved mesh).  Bar per quantity: max|err| / max|ref|
    within 4x the fp32 oracle's own (refcpu in float32 on the CPU: the message
    gradients sum ~1e5 ReLU-gated per-edge terms, several of them within fp32
    rounding of the kink), or 2e-6 (the BatchNorm running statistics 1e-5)."""
    from mmpde_amd.gnn_2d import GNN_Layer_FS_2D, EdgeGraph
    from mmpde_amd.synth import _randomise_bn, cy_synth_mesh

    torch.manual_seed(0)
    lay = GNN_Layer_FS_2D(128, 128, 128, 1, 1)
    _randomise_bn(lay, torch.Generator().manual_seed(1))
    lay.train()
    pts = cy_synth_mesh()
    B = 2
    n = B * pts.shape[0]
    ei, nbr, _ = refcpu.knn_graph(pts.repeat(B, 1), 35, B)
    g = torch.Generator().manual_seed(3)
    h = torch.randn(n, 128, generator=g)
    ext = torch.cat((torch.randn(n, 1, generator=g), pts.repeat(B, 1), torch.full((n, 1), 0.3)), 1)
    dy = torch.randn(n, 128, generator=g)

    def ref(dtype):
        sd = {("." + k): v.detach().to(dtype).clone() for k, v in lay.state_dict().items()}
        for k, v in sd.items():
            if k.endswith(("weight", "bias")):
                v.requires_grad_()
        hr, er = h.to(dtype).clone().requires_grad_(), ext.to(dtype).clone().requires_grad_()
        yr = refcpu.gnn_layer(sd, "", hr, er[:, 0:1], er[:, 1:2], er[:, 2:3], er[:, 3:4], ei, train=True)
        (yr * dy.to(dtype)).sum().backward()
        out = {"h'": yr, "dL/dh": hr.grad, "dL/du": er.grad[:, 0]}
        out.update({k[1:]: v.grad for k, v in sd.items() if v.grad is not None})
        out.update({k[1:]: v for k, v in sd.items() if k.endswith(("running_mean", "running_var"))})
        return out

    r64, r32 = ref(torch.float64), ref(torch.float32)
    lay.to(dev)
    hd, ed = h.to(dev).requires_grad_(), ext.to(dev).requires_grad_()
    y = lay.train_forward_fused(hd, ed, EdgeGraph(nbr.int().to(dev)), edge_gemm)
    (y * dy.to(dev)).sum().backward()
    got = {"h'": y, "dL/dh": hd.grad, "dL/du": ed.grad[:, 0]}
    got.update({k: p.grad for k, p in lay.named_parameters()})
    got.update({k: b for k, b in lay.named_buffers() if k.endswith(("running_mean", "running_var"))})

    def rel(a, b):
        return ((a.detach().double().cpu() - b.double()).abs().max() / b.double().abs().max()).item()

    for k, r in r64.items():
        e, f = rel(got[k], r), rel(r32[k], r)
        print(f"{edge_gemm} {k}: rel max err {e:.2e} (fp32 oracle {f:.2e})")
        bar = 1e-5 if k.startswith("norm.module.running") else max(4 * f, 2e-6)
        assert e <= bar, (k, e, f)


@pytest.mark.parametrize("conv,B", [(False, 16), (True, 16), (False, 33)])
def test_res_cut_train_vs_fp64(dev, conv, B):
    """ItpNet.res_cut in train mode (interpolate.py:54-60,95-97) on the HIP
    kernels (cy: ResCutMlp on mmpde_linear_skinny / _outer_rows / _transpose /
    _tanh_bwd; Burgers: ops.Conv2dSame + tanh) against float64 autograd through
    the module itself: output and every parameter gradient within 1e-5 of
    max|ref| (exact fp32 products, K <= 2521).  B = 33: the weight gradient's
    row sum (mmpde_outer_rows) runs over more than one 32-row pass."""
    from mmpde_amd.interpolate import ItpNet

    torch.manual_seed(0)
    itp = ItpNet(48, 48, [128, 64], [128, 64], [1, 4, 16, 4, 1]) if conv else \
        ItpNet(2521, None, [128, 64], [128, 64], [1, 4, 16, 4, 1])
    g = torch.Generator().manual_seed(5)
    data = torch.randn(B, 1, 48, 48, generator=g) if conv else torch.randn(B, 2521, generator=g)
    dy = torch.randn(B, 1, 48, 48, generator=g) if conv else torch.randn(B, 2521, generator=g)
    ref = ItpNet(48, 48, [128, 64], [128, 64], [1, 4, 16, 4, 1]) if conv else \
        ItpNet(2521, None, [128, 64], [128, 64], [1, 4, 16, 4, 1])
    ref.load_state_dict(itp.state_dict())
    ref.double().train()
    yr = ref.down(data.double())
    (yr * dy.double()).sum().backward()
    itp.to(dev).train()
    y = itp.res_cut(data.to(dev))
    (y * dy.to(dev)).sum().backward()
    _close(y, yr, 1e-5, "res_cut train forward")
    for (name, p), (_, pr) in zip(itp.down.named_parameters(), ref.down.named_parameters()):
        _close(p.grad, pr.grad, 1e-5, f"d/d down.{name}")
