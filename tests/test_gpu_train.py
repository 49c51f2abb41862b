"""Training backward: gradients of the HIP training path
against torch.autograd through the float64 oracle.

Reference iteration (train_helper_2d.py:107-128, models in train() mode,
mmpde.py:71-73,86):

    graph     = create_graph(itp, data, labels, steps, device, mesh_model)
    graph_uni = create_graph(itp, data, labels, steps, device, None)
    pred = interpolate_pred(itp, model_b(graph), graph, data, device) + model(graph_uni)
    loss = MSELoss(pred, labels); loss.backward()

The DMM mesh model is frozen (eval(), not in the AdamW groups of
mmpde.py:269-271), so the mesh is a constant of the parameter gradients and
both sides use the same moved mesh (the engine's, injected into the oracle).

Bars, written per check: the edge-stage kernels 2e-5 of max|ref| (fp32
arithmetic against float64, fixed seeds); every parameter gradient of model,
model_b and ItpNet max(1e-4, 2 x torch-fp32's) relative L2 and 1e-3 of
max|ref| element-wise (see _grad_close; a bias feeding a train-mode BatchNorm
has an exactly-zero gradient: its absolute bar is 1e-4 of the sibling weight's
max|ref|); the loss 1e-5 relative; BatchNorm running buffers after the step
1e-5 of max|ref|.  The same oracle run in float32 is printed beside each
gradient as the fp32 floor of that quantity.

Both oracle runs (float64 reference, float32 floor) are conditioned on the HIP
forward's own activation pattern (mmpde_amd.gnn_2d.RELU_RECORD ->
refcpu.RELU_PATTERN): the embedding ReLU and, per GNN layer, the z1 = a_i + b_j,
z2 (message_net_2's relu_mask bits), update_net_1 and update_net_2 ReLUs.  A
pre-activation within rounding of a kink (the Burgers case holds one at 8e-9
of its row's max in model_b's layer-2 update_net_2) then takes the same side
in all three evaluations, so the bars compare gradients of one function.
"""
import copy
import math

import pytest
import torch

from oracle import refcpu

pytestmark = pytest.mark.gpu


def _err(got, ref, what):
    got = got.detach().double().cpu().reshape(-1)
    ref = ref.detach().double().cpu().reshape(-1)
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    err = (got - ref).abs().max().item() if ref.numel() else 0.0
    scale = ref.abs().max().item() if ref.numel() else 0.0
    print(f"{what}: max|err| {err:.3e} max|ref| {scale:.3e} rel {err / max(scale, 1e-300):.2e}")
    return err, scale


def _close(got, ref, rtol, what, atol=0.0):
    err, scale = _err(got, ref, what)
    assert err <= rtol * scale + atol, (what, err, rtol * scale + atol)


def _rel_norm(got, ref):
    got = got.detach().double().cpu().reshape(-1)
    ref = ref.detach().double().cpu().reshape(-1)
    return ((got - ref).norm() / ref.norm().clamp(min=1e-300)).item()


def _grad_close(got, ref, floor32, what, atol=0.0):
    """Parameter gradients sum ~1e5 per-edge terms with heavy cancellation: the
    bar is a relative L2 error of max(1e-4, 2 x the fp32 oracle's own) --
    model_b's inputs come through fp32 interpolation on both fp32 sides, which
    sets a floor near 1e-4 for burgers -- and 1e-3 of max|ref| (+atol)
    element-wise.  Both oracle runs share the HIP forward's activation pattern
    (module doc)."""
    err, scale = _err(got, ref, what)
    rn, floor = _rel_norm(got, ref), _rel_norm(floor32, ref)
    print(f"    rel-L2 {rn:.2e} (fp32 oracle {floor:.2e})")
    assert rn <= max(1e-4, 2 * floor) or (atol and err <= atol), (what, rn, floor)
    assert err <= 1e-3 * scale + atol, (what, err, 1e-3 * scale + atol)


# --------------------------------------------------------------------------- edge stage
def _edge_mean_ref(a, b, w2, b2, nbr, deg):
    """gnn_2d.py:59-63 message_net_2 + aggr='mean' over the factored first layer
    (z1 = a_i + b_j), float64, padding slots (e >= deg) masked."""
    n, k = nbr.shape
    live = (torch.arange(k)[None, :] < deg[:, None]).to(a.dtype)
    z1 = a[:, None, :] + b[nbr.clamp(min=0).long()]
    m = torch.relu(torch.relu(z1) @ w2.t() + b2) * live[..., None]
    return m.sum(1) / deg.clamp(min=1).to(a.dtype)[:, None]


@pytest.mark.parametrize("edge_gemm", ["f32", "f16x3"])
@pytest.mark.parametrize("ragged", [False, True])
def test_edge_mean_forward_backward_vs_autograd(dev, ragged, edge_gemm):
    from mmpde_amd.gnn_2d import EdgeGraph, EdgeMean

    g = torch.Generator().manual_seed(5 + ragged)
    n, k = 203, 9                         # a partial last 16-row tile
    a = 0.5 * torch.randn(n, 128, generator=g)
    b = 0.5 * torch.randn(n, 128, generator=g)
    w2 = torch.randn(128, 128, generator=g) / math.sqrt(128)
    b2 = 0.1 * torch.randn(128, generator=g)
    nbr = torch.randint(0, n, (n, k), generator=g, dtype=torch.int32)
    if ragged:
        deg = torch.randint(0, k + 1, (n,), generator=g, dtype=torch.int32)
        deg[:3] = 0                       # isolated targets: mean 0, no gradient
        nbr[torch.arange(k)[None, :] >= deg[:, None]] = -1
    else:
        deg = torch.full((n,), k, dtype=torch.int32)
    gout = torch.randn(n, 128, generator=g)

    ref_in = [t.double().requires_grad_() for t in (a, b, w2, b2)]
    ref = _edge_mean_ref(*ref_in, nbr, deg)
    (ref * gout.double()).sum().backward()

    graph = EdgeGraph(nbr.to(dev), deg.to(dev) if ragged else None)
    got_in = [t.to(dev).requires_grad_() for t in (a, b, w2, b2)]
    out = EdgeMean.apply(*got_in, graph, edge_gemm)
    (out * gout.to(dev)).sum().backward()
    torch.cuda.synchronize()
    tag = ("ragged " if ragged else "fixed ") + edge_gemm
    _close(out, ref, 2e-5, f"{tag} mean")
    for name, t, r in zip(("a", "b", "W2", "b2"), got_in, ref_in):
        _close(t.grad, r.grad, 2e-5, f"{tag} d/d{name}")
    # deterministic: a second backward gives the same bits
    grads = [t.grad.clone() for t in got_in]
    for t in got_in:
        t.grad = None
    EdgeMean.apply(*got_in, graph, edge_gemm).mul(gout.to(dev)).sum().backward()
    for t, g0 in zip(got_in, grads):
        assert torch.equal(t.grad, g0)


# --------------------------------------------------------------------------- whole step
def _sds(dtype=torch.float64, **mods):
    """State dicts in `dtype`; parameters are autograd leaves, buffers plain copies."""
    out = {}
    for key, m in mods.items():
        params = {n for n, _ in m.named_parameters()}
        d = {}
        for n, t in m.state_dict().items():
            t = t.detach().cpu().clone()
            if t.is_floating_point():
                t = t.to(dtype)
                if n in params:
                    t.requires_grad_(True)
            d[n] = t
        out[key] = d
    return out


def _setup(kind, B, seed=0):
    from mmpde_amd.synth import build_models, burgers_grid_points, fields

    pde, model, model_b, itp, dmm, gc = build_models(kind, seed=seed)
    if kind == "cy":
        u = fields(pde.ori_grid, B, 30, seed=seed + 1)
        opde = refcpu.PDEConst("cy", pde.grid_size, ori_grid=pde.ori_grid.double())
    else:
        u = fields(burgers_grid_points(), B, 31, seed=seed + 1).reshape(B, 31, 48, 48)
        opde = refcpu.PDEConst("burgers", pde.grid_size)
    return pde, opde, model, model_b, itp, dmm, gc, u


@pytest.mark.parametrize("edge_gemm", ["f32", "f16x3"])
@pytest.mark.parametrize("kind", ["cy", "burgers"])
def test_training_step_gradients_vs_oracle(dev, kind, edge_gemm):
    torch.set_num_threads(min(16, torch.get_num_threads()))
    B = 2
    pde, opde, model, model_b, itp, dmm, gc, u = _setup(kind, B)
    steps = [4, 11]
    sds = _sds(model=model, model_b=model_b, itp=itp)
    sds32 = _sds(torch.float32, model=model, model_b=model_b, itp=itp)   # the fp32 floor
    for m in (model, model_b, itp, dmm):
        m.to(dev)
    model.edge_gemm = model_b.edge_gemm = edge_gemm   # the edge backward's GEMM arithmetic
    model.train()
    model_b.train()
    itp.train()
    dmm.eval()                            # frozen mesh model (mmpde.py:201)

    data, labels = gc.create_data(u, steps)
    graph = gc.create_graph(itp, data, labels, steps, dev, dmm)
    graph_uni = gc.create_graph(itp, data, labels, steps, dev, None)
    from mmpde_amd import gnn_2d
    gnn_2d.RELU_RECORD = []
    try:
        out_b = model_b(graph)
        rec_b = gnn_2d.RELU_RECORD
        gnn_2d.RELU_RECORD = []
        out_u = model(graph_uni)
        rec_u = gnn_2d.RELU_RECORD
    finally:
        gnn_2d.RELU_RECORD = None
    pred = gc.interpolate_pred(itp, out_b, graph, data, dev) + out_u
    loss = torch.nn.MSELoss()(pred, labels.to(dev).reshape(-1, 1))
    loss.backward()
    torch.cuda.synchronize()

    mesh = graph.pos[:, 1:3].detach().cpu().double()
    opde32 = copy.copy(opde)
    if opde.ori_grid is not None:
        opde32.ori_grid = opde.ori_grid.float()
    # the HIP forward's activation pattern, per (model, site): both oracle runs
    # below evaluate the same function on it
    pats = {}
    for key, rec, g in (("model_b", rec_b, graph), ("model", rec_u, graph_uni)):
        n = g.x.shape[0]
        nbr = g.edge_index[0].reshape(n, -1).cpu()
        assert torch.equal(g.edge_index[1].cpu(), torch.arange(n).repeat_interleave(nbr.shape[1]))
        assert [r[0] for r in rec] == ["emb"] + ["layer"] * 6, [r[0] for r in rec]
        pats[(key, "embedding_mlp", "emb")] = rec[0][1].cpu()
        for i, (_, a, b, v, upd, words) in enumerate(rec[1:]):
            p = f"gnn_layers.{i}"
            a, b = a.detach().cpu(), b.detach().cpu()
            pats[(key, p, "z1")] = ((a[:, None, :] + b[nbr]) > 0).reshape(-1, 128)
            w = words.cpu().to(torch.int64) & 0xFFFFFFFF                         # [E, 4]
            c = torch.arange(128)
            pats[(key, p, "z2")] = ((w[:, c // 32] >> (c % 32)) & 1).bool()
            pats[(key, p, "v")] = v.cpu()
            pats[(key, p, "upd")] = upd.cpu()
    sd_key = {}

    def pattern(sd, prefix, site):
        return pats.get((sd_key.get(id(sd)), prefix, site))

    sd_key.update({id(sds[k]): k for k in ("model", "model_b")})
    sd_key.update({id(sds32[k]): k for k in ("model", "model_b")})
    refcpu.RELU_PATTERN = pattern
    try:
        rloss, aux = refcpu.mmpde_train_loss(opde, sds, data.double(), labels.double(), steps,
                                             mesh_override=mesh)
        rloss.backward()
        loss32, _ = refcpu.mmpde_train_loss(opde32, sds32, data, labels, steps, mesh_override=mesh.float())
        loss32.backward()
    finally:
        refcpu.RELU_PATTERN = None
    assert torch.equal(graph.edge_index.cpu(), aux["graph"].edge_index)
    _close(pred, aux["pred"], 2e-5, f"{kind} train-mode pred")
    assert abs(loss.item() - rloss.item()) <= 1e-5 * rloss.item(), (loss.item(), rloss.item())

    checked = 0
    for key, mod in (("model", model), ("model_b", model_b), ("itp", itp)):
        for name, p in mod.named_parameters():
            r = sds[key][name].grad
            if r is None:                 # layers3 (never used) / unused modes
                assert p.grad is None or not p.grad.abs().max().item()
                continue
            assert p.grad is not None, f"{key}.{name} got no gradient"
            atol = 0.0
            if name.endswith(".bias"):
                atol = 1e-4 * sds[key][name[:-5] + ".weight"].grad.abs().max().item()
            _grad_close(p.grad, r, sds32[key][name].grad, f"{kind} grad {key}.{name}", atol=atol)
            checked += 1
        for name, buf in mod.named_buffers():
            if name.endswith(("running_mean", "running_var")):
                _close(buf, sds[key][name], 1e-5, f"{kind} {key}.{name} after step")
    assert checked == 2 * 74 + (14 if kind == "cy" else 20)   # every trained parameter


# --------------------------------------------------------------------------- loops
def _loop_run(dev, seed):
    import random

    from mmpde_amd.train import training_itp, training_loop_branch

    pde, opde, model, model_b, itp, dmm, gc, u = _setup("cy", 4, seed=2)
    for m in (model, model_b, itp, dmm):
        m.to(dev)
    model.train()
    model_b.train()
    itp.train()
    dmm.eval()
    opt = torch.optim.AdamW([{"params": model.parameters()}, {"params": model_b.parameters()},
                             {"params": itp.parameters()}], lr=1e-4)   # mmpde.py:269-271
    ds = torch.utils.data.TensorDataset(u, u)
    loader = torch.utils.data.DataLoader(ds, batch_size=2, shuffle=False)
    crit = torch.nn.MSELoss()
    random.seed(seed)
    li = training_itp(itp, dmm, [0], 128 * 2, opt, None, loader, gc, crit, dev)
    lb = training_loop_branch(model, model_b, itp, dmm, [0, 1], 2, opt, None, loader, gc, crit,
                              dev)
    lb2 = training_loop_branch(model, model_b, itp, dmm, [0, 1], 2, opt, None, loader, gc, crit,
                               dev)
    params = {f"{k}.{n}": p.detach().cpu().clone()
              for k, m in (("model", model), ("model_b", model_b), ("itp", itp))
              for n, p in m.named_parameters()}
    return li.cpu(), torch.cat((lb, lb2)).cpu(), params


def test_training_loops_deterministic_and_learning(dev):
    """training_itp + two epochs of training_loop_branch (train_helper_2d.py:9-134)
    with AdamW: finite, the GNN loss falls, and a second run from the same seed
    reproduces every loss and every parameter bit for bit.  The HIP kernels are
    deterministic by construction (no atomics, fixed reduction orders); the
    library ops around them (MIOpen / hipBLASLt backward) are made so with
    torch.use_deterministic_algorithms -- without it the losses still repeat
    but the parameters drift in the last bits."""
    torch.use_deterministic_algorithms(True, warn_only=True)
    try:
        li, lb, p = _loop_run(dev, 0)
        li2, lb2, p2 = _loop_run(dev, 0)
    finally:
        torch.use_deterministic_algorithms(False)
    print("itp losses", li.tolist(), "branch losses", lb.tolist())
    assert torch.isfinite(li).all() and torch.isfinite(lb).all()
    assert all(torch.isfinite(t).all() for t in p.values())
    assert lb[2:].mean() < lb[:2].mean()
    differ = [n for n in p if not torch.equal(p[n], p2[n])]
    print("parameters differing between the runs:", differ)
    assert torch.equal(li, li2) and torch.equal(lb, lb2) and not differ
