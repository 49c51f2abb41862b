"""Row reductions of the training path (csrc/train_rows.hip) against float64
torch: the skinny weight gradients (mmpde_rows_grad_weight: the Conv1d head's
window GEMMs and the embedding Linear, gnn_2d.py:99-114) and BatchNorm1d in
train mode with the fused residual add (mmpde_batch_norm_rows_*,
gnn_2d.py:51,69,101,105; nn.BatchNorm1d semantics incl. the running
statistics and num_batches_tracked).

Bars: fp32 sums over up to 1.5e6 rows against float64 -- 2e-5 of max|ref| for
the weight gradients and 1e-5 for BatchNorm outputs / statistics; the input
gradient 2e-5 of max|ref|.  Determinism: a second call gives the same bits.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _close(got, ref, rtol, what):
    got = got.detach().double().cpu().reshape(-1)
    ref = ref.detach().double().cpu().reshape(-1)
    err = (got - ref).abs().max().item()
    scale = ref.abs().max().item()
    print(f"{what}: max|err| {err:.3e} max|ref| {scale:.3e}")
    assert err <= rtol * scale, (what, err, rtol * scale)


@pytest.mark.parametrize("rows,k,nout,bias,ldx", [
    (5000, 16, 4, True, 16),            # head conv1 windows (small)
    (1532768, 16, 4, True, 16),         # head conv1 at cy B=16 (40336 x 38)
    (363024, 48, 8, True, 48),          # head conv2 (40336 x 9)
    (40336, 64, 1, True, 64),           # head conv3
    (40336, 4, 128, True, 4),           # embedding Linear(4, 128)
    (9999, 5, 100, False, 7),           # strided rows, no bias, ragged last tile
    (50000, 0, 128, True, 0),           # bias only (the node GEMMs' db)
    (7, 16, 8, True, 16),               # column-lane kernel: fewer rows than one pass
    (100003, 32, 2, False, 36),         # column-lane kernel: strided 16-byte rows, ragged
    (70001, 64, 4, True, 64),           # column-lane kernel: k = 64
])
def test_rows_grad_weight_vs_fp64(dev, rows, k, nout, bias, ldx):
    from mmpde_amd import ops

    g = torch.Generator().manual_seed(rows + k)
    xb = torch.randn(rows, max(ldx, 1), generator=g)
    x = xb[:, :k]
    dy = torch.randn(rows, nout, generator=g)
    xd, dyd = xb.to(dev)[:, :k], dy.to(dev)
    gw, gb = ops.rows_grad_weight(xd, dyd, k, bias)
    torch.cuda.synchronize()
    if k:
        _close(gw, dy.double().t() @ x.double(), 2e-5, f"dW rows={rows} k={k} n={nout}")
    else:
        assert gw is None
    if bias:
        _close(gb, dy.double().sum(0), 2e-5, f"db rows={rows}")
    else:
        assert gb is None
    gw2, gb2 = ops.rows_grad_weight(xd, dyd, k, bias)
    assert (gw is None or torch.equal(gw, gw2)) and (gb is None or torch.equal(gb, gb2))


def test_linear_rows_head_shapes_use_rows_kernel(dev):
    """LinearRows' backward on a skinny map matches autograd of x W^T + b."""
    from mmpde_amd import ops

    g = torch.Generator().manual_seed(3)
    x = torch.randn(20000, 48, generator=g)
    w = torch.randn(8, 48, generator=g) / 7
    b = torch.randn(8, generator=g)
    dy = torch.randn(20000, 8, generator=g)
    ref = [t.double().requires_grad_() for t in (x, w, b)]
    (torch.addmm(ref[2], ref[0], ref[1].t()) * dy.double()).sum().backward()
    got = [t.to(dev).requires_grad_() for t in (x, w, b)]
    y = ops.LinearRows.apply(*got)
    (y * dy.to(dev)).sum().backward()
    for name, t, r in zip("xwb", got, ref):
        _close(t.grad, r.grad, 2e-5, f"LinearRows d{name}")


def test_frozen_head_backward_returns_input_grad(dev):
    """A frozen output head (output_mlp without gradients) while the rest of the
    GNN trains: LinearRows' backward returns dL/dh alone (no weight or bias
    gradient is formed for the skinny head windows)."""
    from mmpde_amd import ops
    from mmpde_amd.synth import build_models

    _, model, _, _, _, _ = build_models("cy", moving_mesh=False)
    model.to(dev)
    for prm in model.output_mlp.parameters():
        prm.requires_grad_(False)
    g = torch.Generator().manual_seed(5)
    h = torch.randn(6000, 128, generator=g)
    hd = h.to(dev).requires_grad_()
    model._head_train(hd).sum().backward()
    assert all(prm.grad is None for prm in model.output_mlp.parameters())
    hr = h.double().requires_grad_()
    o = model.output_mlp
    d = hr[:, None]
    for i, idx in enumerate((0, 2, 4)):
        c = o[idx]
        d = torch.nn.functional.conv1d(d, c.weight.double().cpu(), c.bias.double().cpu(), stride=c.stride)
        if idx != 4:
            d = torch.relu(d)
    d.squeeze(1).sum().backward()
    # two ReLUs on the way: an fp32 pre-activation within rounding of 0 may take
    # the other side than in float64 and move that node's row, so the bar is a
    # relative L2 error (as tests/test_gpu_train.py's)
    rel = ((hd.grad.double().cpu() - hr.grad).norm() / hr.grad.norm()).item()
    print(f"frozen head dL/dh rel-L2 {rel:.2e}")
    assert rel <= 1e-4
    # a bias-only gradient (weight frozen) on the skinny path too
    x = torch.randn(20000, 48, generator=g).to(dev)
    w = (torch.randn(8, 48, generator=g) / 7).to(dev)
    b = torch.randn(8, generator=g).to(dev).requires_grad_()
    ops.LinearRows.apply(x, w, b).sum().backward()
    _close(b.grad, torch.full((8,), 20000.0, dtype=torch.float64), 1e-6, "bias-only db")


def test_edge_graph_checks_caller_tables(dev):
    """EdgeGraph built by a caller from a table with a source outside [0, n):
    the reverse adjacency (built by the first backward) raises instead of
    dropping that edge's gradient."""
    from mmpde_amd.gnn_2d import EdgeGraph

    nbr = torch.randint(0, 50, (50, 4), dtype=torch.int32)
    nbr[7, 2] = 50
    with pytest.raises(ValueError):
        EdgeGraph(nbr.to(dev)).reverse()
    nbr[7, 2] = 3
    EdgeGraph(nbr.to(dev)).reverse()


@pytest.mark.parametrize("n,C,res,affine", [
    (40336, 128, True, True),           # GNN layer norm(h + upd) at cy B=16
    (5042, 128, False, True),           # embedding BatchNorm1d, B=2
    (777, 12, True, False),             # odd row count, C4 not dividing 256, no affine
])
def test_batch_norm_rows_vs_torch_fp64(dev, n, C, res, affine):
    from mmpde_amd import ops

    g = torch.Generator().manual_seed(n)
    x = 2.0 + torch.randn(n, C, generator=g)     # mean offset: a cancellation test
    r = 0.5 * torch.randn(n, C, generator=g) if res else None
    dy = torch.randn(n, C, generator=g)
    bn_ref = torch.nn.BatchNorm1d(C, affine=affine).double()
    bn = torch.nn.BatchNorm1d(C, affine=affine)
    if affine:
        with torch.no_grad():
            w = 1.0 + 0.1 * torch.randn(C, generator=g)
            b = 0.1 * torch.randn(C, generator=g)
            bn_ref.weight.copy_(w)
            bn_ref.bias.copy_(b)
            bn.weight.copy_(w)
            bn.bias.copy_(b)
    bn = bn.to(dev).train()
    bn_ref.train()
    xr = x.double().requires_grad_()
    rr = r.double().requires_grad_() if res else None
    yr = bn_ref(xr + rr if res else xr)
    (yr * dy.double()).sum().backward()

    xg = x.to(dev).requires_grad_()
    rg = r.to(dev).requires_grad_() if res else None
    y = ops.batch_norm_rows(bn, xg, rg)
    (y * dy.to(dev)).sum().backward()
    torch.cuda.synchronize()
    _close(y, yr, 1e-5, "bn y")
    _close(bn.running_mean, bn_ref.running_mean, 1e-5, "running_mean")
    _close(bn.running_var, bn_ref.running_var, 1e-5, "running_var")
    assert int(bn.num_batches_tracked) == int(bn_ref.num_batches_tracked) == 1
    _close(xg.grad, xr.grad, 2e-5, "bn dx")
    if res:
        _close(rg.grad, rr.grad, 2e-5, "bn dres")
    if affine:
        _close(bn.weight.grad, bn_ref.weight.grad, 2e-5, "bn dweight")
        _close(bn.bias.grad, bn_ref.bias.grad, 2e-5, "bn dbias")
    # deterministic
    g0 = xg.grad.clone()
    xg.grad = None
    if res:
        rg.grad = None
    y2 = ops.batch_norm_rows(bn, xg, rg)
    (y2 * dy.to(dev)).sum().backward()
    assert torch.equal(y2, y) and torch.equal(xg.grad, g0)


def test_batch_norm_rows_eval_uses_running_stats(dev):
    from mmpde_amd import ops

    bn = torch.nn.BatchNorm1d(128).to(dev)
    with torch.no_grad():
        bn.running_mean.uniform_(-1, 1)
        bn.running_var.uniform_(0.5, 2)
    bn.eval()
    x, r = torch.randn(300, 128, device=dev), torch.randn(300, 128, device=dev)
    assert torch.equal(ops.batch_norm_rows(bn, x, r), bn(x + r))


@pytest.mark.parametrize("n,k,ragged,hub", [(57, 7, False, False), (57, 7, True, False),
                                             (40336, 35, False, False), (5000, 30, True, True)])
def test_reverse_adjacency_device_equals_host(dev, n, k, ragged, hub):
    """mmpde_reverse_adjacency against the host argsort construction: the same
    groups in the same (stable, target) order; hubs (one source of every
    fifth slot) exercise long groups."""
    from mmpde_amd.ops import reverse_adjacency

    g = torch.Generator().manual_seed(n + k)
    nbr = torch.randint(0, n, (n, k), generator=g, dtype=torch.int32)
    if hub:
        nbr.view(-1)[::5] = 3
    deg = None
    if ragged:
        deg = torch.randint(0, k + 1, (n,), generator=g, dtype=torch.int32)
        nbr[torch.arange(k)[None, :] >= deg[:, None]] = -1
    off_h, edge_h = reverse_adjacency(nbr, deg)
    off_d, edge_d = reverse_adjacency(nbr.to(dev), deg.to(dev) if deg is not None else None)
    assert torch.equal(off_d.cpu(), off_h)
    assert torch.equal(edge_d[:int(off_h[-1])].cpu(), edge_h)
    with pytest.raises(ValueError):
        bad = nbr.clone()
        bad[0, 0] = n
        reverse_adjacency(bad.to(dev), None)


@pytest.mark.parametrize("edge_gemm", ["f32", "f16x3"])
@pytest.mark.parametrize("ragged", [False, True])
def test_edge_backward_sorted_equals_gather_path(dev, edge_gemm, ragged):
    """mmpde_gnn_edge_backward_sorted + mmpde_gnn_edge_source_sum_sorted (per-edge
    gradients stored source-major, contiguous per-source sums) against
    mmpde_gnn_edge_backward_ex + mmpde_gnn_edge_source_sum (target-major rows,
    gathered sums): the same sums in the same order, so every output is
    bitwise equal."""
    import math

    from mmpde_amd import _lib as L
    from mmpde_amd.ops import reverse_adjacency

    g = torch.Generator().manual_seed(11 + ragged)
    n, k = 3001, 35
    a = (0.5 * torch.randn(n, 128, generator=g)).to(dev)
    b = (0.5 * torch.randn(n, 128, generator=g)).to(dev)
    w2 = (torch.randn(128, 128, generator=g) / math.sqrt(128)).to(dev)
    b2 = (0.1 * torch.randn(128, generator=g)).to(dev)
    gm = torch.randn(n, 128, generator=g).to(dev)
    nbr = torch.randint(0, n, (n, k), generator=g, dtype=torch.int32)
    deg = None
    if ragged:
        deg = torch.randint(0, k + 1, (n,), generator=g, dtype=torch.int32)
        nbr[torch.arange(k)[None, :] >= deg[:, None]] = -1
        deg = deg.to(dev)
    nbr = nbr.to(dev)
    lib, st = L.lib(), L.stream(dev)
    mode = L.EDGE_GEMM[edge_gemm]
    outs = []
    for sorted_ in (False, True):
        ga, gb = torch.empty_like(a), torch.empty_like(b)
        ge = torch.empty((n * k, 128), dtype=torch.float32, device=dev)
        part = torch.empty((lib.mmpde_gnn_edge_backward_partials(None),), dtype=torch.float32, device=dev)
        gw2 = torch.empty((128, 128), dtype=torch.float32, device=dev)
        gb2 = torch.empty((128,), dtype=torch.float32, device=dev)
        off, edge, pos = reverse_adjacency(nbr, deg, check=True, slot_pos=True)
        if sorted_:
            L.check(lib.mmpde_gnn_edge_backward_sorted(L.ptr(a), L.ptr(b), L.ptr(nbr), L.ptr(deg), n, k, L.ptr(w2),
                                                       L.ptr(b2), L.ptr(gm), L.ptr(pos), None, L.ptr(ga), L.ptr(ge),
                                                       L.ptr(part), L.ptr(gw2), L.ptr(gb2), mode, st), "sorted")
            L.check(lib.mmpde_gnn_edge_source_sum_sorted(L.ptr(ge), L.ptr(off), n, L.ptr(gb), st), "sum")
        else:
            L.check(lib.mmpde_gnn_edge_backward_ex(L.ptr(a), L.ptr(b), L.ptr(nbr), L.ptr(deg), n, k, L.ptr(w2),
                                                   L.ptr(b2), L.ptr(gm), L.ptr(ga), L.ptr(ge), L.ptr(part),
                                                   L.ptr(gw2), L.ptr(gb2), mode, st), "ex")
            L.check(lib.mmpde_gnn_edge_source_sum(L.ptr(ge), L.ptr(off), L.ptr(edge), n, L.ptr(gb), st), "sum")
        outs.append((ga, gb, gw2, gb2))
    torch.cuda.synchronize()
    for x, y in zip(*outs):
        assert torch.equal(x, y)


@pytest.mark.parametrize("n", [5, 1000, 40336])
def test_head_train_vs_fp64(dev, n):
    """ops.HeadTrain (the Conv1d head, gnn_2d.py:108-114, forward and backward
    on mmpde_head_train_*) against float64 autograd of the same nn.Sequential:
    y and dL/dh within 2e-5 of max|ref|, the six weight / bias gradients
    (sums over n nodes) within 5e-5; a second backward gives the same bits."""
    from mmpde_amd import ops

    torch.manual_seed(n)
    mlp = torch.nn.Sequential(torch.nn.Conv1d(1, 4, 16, stride=3), torch.nn.ReLU(),
                              torch.nn.Conv1d(4, 8, 12, stride=3), torch.nn.ReLU(),
                              torch.nn.Conv1d(8, 1, 8, stride=2))
    h = torch.randn(n, 128)
    gy = torch.randn(n, 1)
    ref = mlp.double()
    hr = h.double().requires_grad_(True)
    yr = ref(hr[:, None]).squeeze(1)
    yr.backward(gy.double())
    mlp_d = mlp.float().to(dev)
    assert ops.head_train_fits(mlp_d, h.to(dev))

    def run():
        hd = h.to(dev).requires_grad_(True)
        for p in mlp_d.parameters():
            p.grad = None
        y = ops.HeadTrain.apply(hd, mlp_d[0].weight, mlp_d[0].bias, mlp_d[2].weight, mlp_d[2].bias,
                                mlp_d[4].weight, mlp_d[4].bias)
        y.backward(gy.to(dev))
        torch.cuda.synchronize()
        return y, hd.grad, [p.grad.clone() for p in mlp_d.parameters()]

    y, gh, gp = run()
    _close(y, yr, 2e-5, f"head y n={n}")
    _close(gh, hr.grad, 2e-5, f"head dL/dh n={n}")
    for name, g, r in zip(("w1", "b1", "w2", "b2", "w3", "b3"), gp, [p.grad for p in ref.parameters()]):
        _close(g, r, 5e-5, f"head d{name} n={n}")
    y2, gh2, gp2 = run()
    assert torch.equal(y, y2) and torch.equal(gh, gh2) and all(torch.equal(a, b) for a, b in zip(gp, gp2))
