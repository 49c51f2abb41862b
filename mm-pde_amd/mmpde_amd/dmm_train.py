"""DMM training: the Monge-Ampere mesh-mover fit of the reference
(mesh/dmm_utils.py:29-267 sampling / monitor / interpolation, :391-1095
train_MA_res's Adam and LBFGS phases, :1149-1284 evaluate_tri / evaluate),
SURVEY.md §8(f) row 4.  The random-feature branch (torchmin BFGS,
dmm_utils.py:290-388 and the rf path of mesh/dmm.py) needs pytorch-minimize,
which is not available, and is not built.

What runs where:
* the DMM forward in train() mode: differentiable device torch ops
  (dmm_model.DMM._forward_train), so grad(phi) and its second derivatives
  come from autograd exactly as in the reference;
* the softmax kernel smoother -- the reference's ``interpolate`` /
  ``interpolate_tri``, which materialise [queries, points] tensors with the
  value field repeated per query -- on the HIP kernel mmpde_softmax_interp,
  with its position VJP (mmpde_softmax_interp_grad) behind ``SoftmaxInterp``;
  the monitor's uniform-grid derivatives of interpolate_tri (the reference's
  autograd.grad with grad_outputs = 1) are that VJP directly;
* sampling follows the reference's numpy RNG calls one for one (np.random
  uniform / choice), so a seeded run draws the same points.

``train_MA_res`` keeps the reference's signature, optimisers (Adam with weight
decay + MultiStepLR [100, 150]; LBFGS with tolerances -1 + MultiStepLR
[75, 125]), loss weights, logging lists and checkpoint dict.
"""
from __future__ import annotations

import os
from datetime import datetime

import numpy as np
import torch
from torch import nn

from . import _lib as L


# --------------------------------------------------------------------------- kernels
class SoftmaxInterp(torch.autograd.Function):
    """out[q] = sum_j vals[s_v(q), j] softmax_j(-scale |pts[s_p(q), j] - qry[q]|)
    (mmpde_softmax_interp); differentiable in qry only (the sampled positions
    x + grad(phi) in the loss)."""

    @staticmethod
    def forward(ctx, pts, vals, qry, scale):
        L.require_device(pts, vals, qry)
        pts = L.f32c(pts).reshape(-1, pts.shape[-2], 2)
        vals = L.f32c(vals).reshape(-1, pts.shape[1])
        qry = L.f32c(qry).reshape(-1, 2)
        out = torch.empty((qry.shape[0],), dtype=torch.float32, device=qry.device)
        L.check(L.lib().mmpde_softmax_interp(L.ptr(pts), pts.shape[1], pts.shape[0], L.ptr(vals),
                                             vals.shape[0], L.ptr(qry), qry.shape[0], float(scale),
                                             L.ptr(out), L.stream(qry.device)), "mmpde_softmax_interp")
        ctx.save_for_backward(pts, vals, qry)
        ctx.scale = float(scale)
        return out

    @staticmethod
    def backward(ctx, g):
        pts, vals, qry = ctx.saved_tensors
        gq = torch.empty_like(qry)
        L.check(L.lib().mmpde_softmax_interp_grad(L.ptr(pts), pts.shape[1], pts.shape[0], L.ptr(vals),
                                                  vals.shape[0], L.ptr(qry), qry.shape[0], ctx.scale,
                                                  L.ptr(L.f32c(g)), L.ptr(gq), L.stream(qry.device)),
                "mmpde_softmax_interp_grad")
        return None, None, gq, None


def softmax_interp_grad_at(pts, vals, qry, scale):
    """d out / d qry of SoftmaxInterp for grad_out = 1: [n_q, 2]."""
    pts = L.f32c(pts).reshape(-1, pts.shape[-2], 2)
    vals = L.f32c(vals).reshape(-1, pts.shape[1])
    qry = L.f32c(qry).reshape(-1, 2)
    ones = torch.ones((qry.shape[0],), dtype=torch.float32, device=qry.device)
    gq = torch.empty_like(qry)
    L.check(L.lib().mmpde_softmax_interp_grad(L.ptr(pts), pts.shape[1], pts.shape[0], L.ptr(vals),
                                              vals.shape[0], L.ptr(qry), qry.shape[0], float(scale),
                                              L.ptr(ones), L.ptr(gq), L.stream(qry.device)),
            "mmpde_softmax_interp_grad")
    return gq


_LATTICES = {}


def unit_lattice(n: int, device) -> torch.Tensor:
    """np.meshgrid(linspace(0, 1, n), linspace(0, 1, n)) flattened 'xy' [n^2, 2]
    (the grid of dmm_utils.py:241-243; point i n + j = (x_j, y_i))."""
    key = (n, str(device))
    g = _LATTICES.get(key)
    if g is None:
        a = np.linspace(0, 1, n)
        g = torch.tensor(np.array(np.meshgrid(a, a)), dtype=torch.float).reshape(2, -1).t()
        g = g.contiguous().to(device)
        _LATTICES[key] = g
    return g


def interpolate(u: torch.Tensor, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """dmm_utils.py:233-249 for u [S, n, n] on the unit lattice and queries
    x, y [Q, 1], S dividing Q (query q reads field q // (Q / S); the
    reference passes the field repeated once per query, S = Q).  -> [Q, 1]."""
    n = u.shape[-1]
    q = torch.cat((x.reshape(-1, 1), y.reshape(-1, 1)), -1)
    return SoftmaxInterp.apply(unit_lattice(n, u.device), u.reshape(-1, n * n), q, float(n))[:, None]


def interpolate_tri(u: torch.Tensor, pts: torch.Tensor, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """dmm_utils.py:251-267 for values u [S, n] at mesh points pts [n, 2] (or
    [S', n, 2]) and queries x, y [Q, 1]: softmax weights of -sqrt(n) |p - q|.
    -> [Q, 1]."""
    n = u.shape[-1]
    q = torch.cat((x.reshape(-1, 1), y.reshape(-1, 1)), -1)
    return SoftmaxInterp.apply(pts.reshape(-1, n, 2), u.reshape(-1, n), q, float(np.sqrt(n)))[:, None]


# --------------------------------------------------------------------------- monitor
def monitor(alpha, ux, uy):
    """dmm_utils.py:209-210."""
    return 1 + (torch.abs(ux) ** 2 + torch.abs(uy) ** 2) ** (1 / 2) / (0.01 * alpha)


def diff_x(u):
    """dmm_utils.py:215-219 (forward difference along dim -2, last row repeated)."""
    d = torch.zeros_like(u)
    d[:, :-1, :] = torch.diff(u, dim=-2)
    d[:, -1, :] = d[:, -2, :]
    return d


def diff_y(u):
    """dmm_utils.py:221-225."""
    d = torch.zeros_like(u)
    d[:, :, :-1] = torch.diff(u, dim=-1)
    d[:, :, -1] = d[:, :, -2]
    return d


def _alpha_m_rhs(ux, uy):
    """alpha, m = monitor(alpha, ux, uy), RHS of fields ux, uy [b, n, n]."""
    n = ux.shape[-1]
    alpha = torch.sum((torch.abs(ux) ** 2 + torch.abs(uy) ** 2) ** (1 / 2), dim=(-2, -1)) / (n - 1) ** 2
    m = monitor(alpha[:, None, None].expand(-1, n, n), ux, uy)
    return alpha, m, torch.sum(m, dim=(-2, -1)) / (n - 1) ** 2


# --------------------------------------------------------------------------- sampling
def sample_train_data(u, nx, nu, device):
    """dmm_utils.py:29-54 (array data u [T, s, s]): nu random fields, their
    monitor, and nx points per field drawn with probability ~ m at 40 nx
    uniform candidates.  Returns u, ux, uy, alpha, m, RHS, x [nu nx, 2].
    nu must be a multiple of 4 (the reference interpolates in 4 chunks and
    fails otherwise)."""
    if nu % 4:
        raise ValueError("batch_size_u must be a multiple of 4 (dmm_utils.py:41-46)")
    cand = torch.tensor(np.random.uniform(0, 1, (nu, 40 * nx, 2)), dtype=torch.float).to(device)
    idx = np.random.choice(a=u.shape[0], size=nu, replace=True)
    u = u[idx].to(device)
    s = u.shape[-1]
    ux = diff_x(u) * (s - 1)
    uy = diff_y(u) * (s - 1)
    alpha, m, rhs = _alpha_m_rhs(ux, uy)
    p = interpolate(m, cand[..., 0].reshape(-1, 1), cand[..., 1].reshape(-1, 1))
    p = p.reshape(nu, -1).cpu().numpy()
    chosen = torch.zeros(nu, nx, 2).to(device)
    for i in range(nu):
        pi = p[i] / np.sum(p[i])
        chosen[i] = cand[i, np.random.choice(a=cand.shape[1], size=nx, replace=False, p=pi)]
    return u, ux, uy, alpha, m, rhs, chosen.reshape(-1, 2)


def _edges(nx, device):
    """The four sides' nx // 4 linspace points: x = 0, x = 1, y = 0, y = 1
    (dmm_utils.py:73-92)."""
    t = np.linspace(0, 1, int(nx / 4))
    sides = ([[0, v] for v in t], [[1, v] for v in t], [[v, 0] for v in t], [[v, 1] for v in t])
    return [torch.tensor(b, dtype=torch.float).to(device) for b in sides]


def sample_train_data_bound(u, nx, nu, device):
    """dmm_utils.py:56-103: boundary points of the four sides (repeated for nu
    fields each), 4 nu random fields and their monitors."""
    idx = np.random.choice(a=u.shape[0], size=4 * nu, replace=True)
    u = u[idx].to(device)
    s = u.shape[-1]
    _, m, _ = _alpha_m_rhs(diff_x(u) * (s - 1), diff_y(u) * (s - 1))
    bounds = [b.repeat(nu, 1, 1).reshape(-1, 2) for b in _edges(nx, device)]
    us = [u[k * nu:(k + 1) * nu] for k in range(4)]
    ms = [m[k * nu:(k + 1) * nu] for k in range(4)]
    return (*bounds, *us, *ms)


def sample_train_data_tri(all_u, nx, nu, device):
    """dmm_utils.py:106-167 (mesh data all_u [T, N, >=3] with columns x, y, u):
    the fields' derivatives on the n x n unit lattice (n = sqrt(N)) as the
    position gradient of interpolate_tri (the reference's autograd.grad with
    grad_outputs = 1), alpha, monitor, RHS, then nx points per field drawn ~ m
    interpolated at 40 nx uniform candidates.  nu must be a multiple of 10 (the
    reference's sub_nu chunks, dmm_utils.py:124-158)."""
    if nu % 10:
        raise ValueError("batch_size_u must be a multiple of 10 (dmm_utils.py:124-158)")
    u = all_u[:, :, 2].to(device)
    cand = torch.tensor(np.random.uniform(0, 1, (nu, 40 * nx, 2)), dtype=torch.float).to(device)
    idx = np.random.choice(a=u.shape[0], size=nu, replace=True)
    u = u[idx].to(device)
    mesh = all_u[idx, :, :2].to(device).float()                      # [nu, N, 2]
    N = u.shape[-1]
    n = int(np.sqrt(N))
    lat = unit_lattice(n, device)                                   # [n^2, 2]
    q = lat[None].expand(nu, -1, -1).reshape(-1, 2)
    g = softmax_interp_grad_at(mesh, u, q, float(np.sqrt(N))).reshape(nu, n, n, 2)
    uni_ux, uni_uy = g[..., 0], g[..., 1]
    alpha, uni_m, rhs = _alpha_m_rhs(uni_ux, uni_uy)
    cx, cy = cand[..., 0].reshape(-1, 1), cand[..., 1].reshape(-1, 1)
    ux_c = interpolate(uni_ux, cx, cy).reshape(nu, -1)
    uy_c = interpolate(uni_uy, cx, cy).reshape(nu, -1)
    p = monitor(alpha[:, None].expand(-1, cand.shape[1]), ux_c, uy_c).cpu().numpy()
    chosen = torch.zeros(nu, nx, 2).to(device)
    for i in range(nu):
        pi = p[i] / np.sum(p[i])
        chosen[i] = cand[i, np.random.choice(a=cand.shape[1], size=nx, replace=False, p=pi)]
    return u, uni_ux, uni_uy, alpha, uni_m, rhs, chosen.reshape(-1, 2)


def sample_train_data_bound_tri(u, nx, nu, device):
    """dmm_utils.py:169-206."""
    idx = np.random.choice(a=u.shape[0], size=4 * nu, replace=True)
    u = u[idx, :, 2].to(device)
    bounds = [b.repeat(nu, 1, 1).reshape(-1, 2) for b in _edges(nx, device)]
    return (*bounds, *[u[k * nu:(k + 1) * nu] for k in range(4)])


# --------------------------------------------------------------------------- loss
def _grad(out, x):
    return torch.autograd.grad(out, x, grad_outputs=torch.ones_like(out), retain_graph=True,
                               create_graph=True, allow_unused=True)[0]


def boundary_loss(model, bounds, bound_us):
    """Soft boundary condition (dmm_utils.py:441-503): d phi / dx = 0 on x = 0, 1
    and d phi / dy = 0 on y = 0, 1, mean of the four MSEs."""
    mse = nn.MSELoss()
    parts = []
    for side, (b, bu) in enumerate(zip(bounds, bound_us)):
        if len(b) == 0:
            parts.append(torch.zeros(1, device=b.device))
            continue
        c1, c2 = b[:, 0].view(-1, 1), b[:, 1].view(-1, 1)
        c1.requires_grad = True
        c2.requires_grad = True
        out = model(bu, torch.cat((c1, c2), dim=1))
        d = _grad(out, c1 if side < 2 else c2)
        parts.append(mse(d, torch.zeros_like(d)))
    return sum(parts) / 4


def ma_losses(model, u, ux, uy, alpha, rhs, x, nx, bound_constraint="soft", init_mesh=False):
    """The interior terms of dmm_utils.py:507-552: phi at the sampled points (hard
    constraint: the boundary-shaped ansatz), grad(phi), and either the identity
    fit (init_mesh) or the Monge-Ampere residual of the moved points
    m(x + grad phi) det(I + Hess phi) / RHS - 1 with the convexity penalty.
    Returns (loss_in, loss_convex or None, LHS or None)."""
    mse = nn.MSELoss()
    x1 = x[:, 0].view(x.shape[0], 1)
    x2 = x[:, 1].view(x.shape[0], 1)
    x1.requires_grad = True
    x2.requires_grad = True
    xx = torch.cat((x1, x2), dim=1)
    if bound_constraint == "soft":
        out = model(u, xx)
    else:
        out = (x1 ** 2) * (x2 ** 2) * ((x1 - 1) ** 2) * ((x2 - 1) ** 2) * model(u, xx) \
            + 0.5 * x1 ** 2 + 0.5 * x2 ** 2
    phix, phiy = _grad(out, x1), _grad(out, x2)
    if init_mesh:
        return (mse(x1 + phix, x1) + mse(x2 + phiy, x2)) / 2, None, None
    phixy, phixx = _grad(phix, x2), _grad(phix, x1)
    phiyx, phiyy = _grad(phiy, x1), _grad(phiy, x2)
    # ux, uy of each field at its moved points (field f for points f nx .. f nx + nx - 1)
    uxm = interpolate(ux, x1 + phix, x2 + phiy)
    uym = interpolate(uy, x1 + phix, x2 + phiy)
    u_xi_x = uxm * (1 + phixx) + uym * phiyx
    u_xi_y = uxm * phixy + uym * (1 + phiyy)
    m_xi = monitor(alpha[:, None].expand(-1, nx).reshape(-1, 1), u_xi_x, u_xi_y)
    lhs = m_xi * ((1 + phixx) * (1 + phiyy) - phixy * phiyx)
    loss_in = mse(lhs / rhs[:, None].expand(-1, nx).reshape(-1, 1), torch.ones_like(lhs))
    zero = torch.tensor(0).type_as(phixx)
    loss_convex = torch.mean(torch.min(zero, 1 + phixx) ** 2 + torch.min(zero, 1 + phiyy) ** 2)
    return loss_in, loss_convex, lhs


def _sample(args, all_u, bx, bu, device):
    if args.experiment == "burgers":
        u, ux, uy, alpha, _, rhs, x = sample_train_data(all_u, bx, bu, device)
        bounds = sample_train_data_bound(all_u, bx, bu, device)[:8]
    elif args.experiment == "cy":
        u, ux, uy, alpha, _, rhs, x = sample_train_data_tri(all_u, bx, bu, device)
        bounds = sample_train_data_bound_tri(all_u, bx, bu, device)
    else:
        raise ValueError(args.experiment)
    return u, ux, uy, alpha, rhs, x, bounds[:4], bounds[4:8]


def objective(model, args, sample, nx, init_mesh, device):
    """One draw's total loss (dmm_utils.py:441-552): (loss, loss_in, loss_bound,
    loss_convex, LHS, RHS)."""
    u, ux, uy, alpha, rhs, x, bounds, bound_us = sample
    if args.bound_constraint == "soft":
        loss_bound = boundary_loss(model, bounds, bound_us)
    else:
        loss_bound = torch.tensor(0).to(device)
    loss_in, loss_convex, lhs = ma_losses(model, u, ux, uy, alpha, rhs, x, nx, args.bound_constraint,
                                          init_mesh)
    loss = args.loss_weight1 * loss_bound + args.loss_weight0 * loss_in
    if not init_mesh and args.loss_convex:
        loss = loss + args.loss_weight2 * loss_convex
    return loss, loss_in, loss_bound, loss_convex, lhs, rhs


# --------------------------------------------------------------------------- training
def train_MA_res(ori_u, all_u, test_u, args, model, init_mesh, n_epoch_adam, n_epoch_lbfgs, device,
                 save_dir=None, evaluate_every=1, reference_save_path=False):  # noqa: N802 - reference name
    """dmm_utils.py:391-1095 without the random-feature branch: n_epoch_adam
    epochs of Adam then n_epoch_lbfgs of LBFGS, each epoch max(1, train_sample_grid
    T / (bx bu)) draws of fresh samples; per epoch the equation residual of the
    last logged draw, the scheduler step, evaluate[_tri] on the train and test
    fields, and the checkpoint dict torch.save'd to save_dir (default
    args.experiment, as the reference; False: not saved).  Returns the
    reference's 15-tuple (dmm_utils.py:1094-1095): model, loss_in, loss_bound,
    loss_convex, test_equ_loss / max / min / mid, train_std, train_minmax,
    test_std, test_minmax, itp_list1, itp_list2 (empty: filled only by the
    random-feature branch), logs_txt.

    Checkpoint file: 'dmm_{experiment}_epoch{N}.pt' in save_dir, one per epoch;
    reference_save_path=True writes the reference's name instead,
    '{experiment}/{datetime}_{rf}_bound{loss_bound_rf}_..._{gamma_adam}'
    (dmm_utils.py:768-770), so scripts that look checkpoints up by that name
    find them.  The dict holds the reference's keys plus test_equ_loss and logs.

    Deliberate difference: with init_mesh=True the reference's LBFGS closure
    (dmm_utils.py:659-662) never calls backward -- LBFGS then steps on zeroed
    gradients -- and its logging (:691-696) reads loss_convex and LHS, which
    that branch never assigns (a NameError on the first logged draw).  Here the
    init_mesh LBFGS phase runs backward like every other phase and logs 0 for
    the convexity loss and None for LHS (tests/test_gpu_dmm_train.py
    ::test_init_mesh_lbfgs_phase_trains)."""
    model.train()
    opt_adam = torch.optim.Adam(model.parameters(), lr=args.lr_adam, betas=(0.9, 0.999), eps=1e-8,
                                weight_decay=args.weight_decay)
    sch_adam = torch.optim.lr_scheduler.MultiStepLR(opt_adam, milestones=[100, 150], gamma=args.gamma_adam)
    opt_lbfgs = torch.optim.LBFGS(model.parameters(), lr=args.lr_lbfgs, tolerance_grad=-1, tolerance_change=-1)
    sch_lbfgs = torch.optim.lr_scheduler.MultiStepLR(opt_lbfgs, milestones=[75, 125], gamma=args.gamma_lbfgs)
    log = {k: [] for k in ("loss_in", "loss_bound", "loss_convex", "LHS", "RHS", "test_equ_loss",
                           "test_equ_max", "test_equ_min", "test_equ_mid", "train_std", "train_minmax",
                           "test_std", "test_minmax", "train_mean", "test_mean", "logs_txt")}
    log["logs_txt"].append(str(args))
    counters = [0, 0]   # draws of the Adam / LBFGS phases (logged every 200th)

    def record(phase, loss_in, loss_bound, loss_convex, lhs, rhs):
        if counters[phase] % 200 == 0:
            log["loss_in"].append(loss_in.item())
            log["loss_convex"].append(loss_convex.item() if loss_convex is not None else 0.0)
            log["loss_bound"].append(loss_bound.item())
            log["LHS"].append(lhs.detach() if lhs is not None else None)
            log["RHS"].append(rhs)
        counters[phase] += 1

    for epoch in range(1, n_epoch_adam + n_epoch_lbfgs + 1):
        start = datetime.now()
        adam = epoch < n_epoch_adam + 1
        bx = args.batch_size_x_adam if adam else args.batch_size_x_lbfgs
        bu = args.batch_size_u_adam if adam else args.batch_size_u_lbfgs
        draws = max(1, int(args.train_sample_grid * all_u.shape[0] / (bx * bu)))
        for _ in range(draws):
            if adam:
                sample = _sample(args, all_u, bx, bu, device)
                opt_adam.zero_grad()
                loss, li, lb, lc, lhs, rhs = objective(model, args, sample, bx, init_mesh, device)
                loss.backward()
                record(0, li, lb, lc, lhs, rhs)
                opt_adam.step()
            else:
                def closure():
                    sample = _sample(args, all_u, bx, bu, device)
                    opt_lbfgs.zero_grad()
                    loss, li, lb, lc, lhs, rhs = objective(model, args, sample, bx, init_mesh, device)
                    loss.backward()
                    record(1, li, lb, lc, lhs, rhs)
                    return loss
                opt_lbfgs.step(closure)
        if log["LHS"] and log["LHS"][-1] is not None:
            # as dmm_utils.py:689: LHS [P, 1] / RHS [nu] broadcasts to the [P, nu]
            # table of every (point, field) pair (a reference quirk, kept)
            equ = log["LHS"][-1] / log["RHS"][-1] - torch.tensor(1).to(device)
            log["test_equ_loss"].append(torch.mean(torch.abs(equ)).item())
            log["test_equ_max"].append(torch.max(equ).item())
            log["test_equ_min"].append(torch.min(equ).item())
            log["test_equ_mid"].append(torch.median(equ).item())
        (sch_adam if adam else sch_lbfgs).step()
        line = "Epoch: {} | Loss in: {} | Loss bound: {} | Loss convex: {}".format(
            epoch, log["loss_in"][-1], log["loss_bound"][-1], log["loss_convex"][-1])
        if log["test_equ_loss"]:
            line += " | Test equ loss: {:1.4f}".format(log["test_equ_loss"][-1])
        log["logs_txt"].append(f"{datetime.now() - start} " + line)
        if evaluate_every and epoch % evaluate_every == 0:
            if args.experiment == "burgers":
                tr = evaluate(model, all_u, device, epoch)
                te = evaluate(model, test_u, device, epoch)
            else:
                tr = evaluate_tri(model, all_u[:, :, 2], all_u[0, :, :2], device, epoch)
                te = evaluate_tri(model, test_u[:, :, 2], all_u[0, :, :2], device, epoch)
            for k, v in zip(("train_mean", "train_std", "train_minmax"), tr):
                log[k].append(v)
            for k, v in zip(("test_mean", "test_std", "test_minmax"), te):
                log[k].append(v)
            log["logs_txt"].append(
                "Train mean: {:1.6f} | Train std: {:1.6f} | Train minmax: {:1.6f} | Test mean: {:1.6f}"
                " | Test std: {:1.6f} | Test minmax: {:1.6f}".format(*tr, *te))
        ckpt = {"model_state_dict": model.state_dict(), "loss_in": log["loss_in"],
                "loss_bound": log["loss_bound"], "loss_convex": log["loss_convex"], "args": args,
                "train_std": log["train_std"], "train_minmax": log["train_minmax"],
                "test_std": log["test_std"], "test_minmax": log["test_minmax"],
                "test_equ_loss": log["test_equ_loss"], "logs": log["logs_txt"]}
        if save_dir is not False:
            d = save_dir if save_dir is not None else args.experiment
            os.makedirs(d, exist_ok=True)
            if reference_save_path:
                name = "{}_{}_bound{}_{}_{}_{}_{}_{}_{}_{}_{}_{}_{}_{}_{}".format(
                    datetime.now(), args.rf, args.loss_bound_rf, args.epochs_rf, args.max_iter, args.sub_u,
                    args.epochs_lbfgs, args.batch_size_u_adam, args.batch_size_x_adam, args.loss_weight1,
                    args.train_sample_grid, args.branch_layers, args.lr_adam, args.trunk_layers,
                    args.gamma_adam)
            else:
                name = f"dmm_{args.experiment}_epoch{epoch}.pt"
            torch.save(ckpt, os.path.join(d, name))
    return (model, log["loss_in"], log["loss_bound"], log["loss_convex"], log["test_equ_loss"],
            log["test_equ_max"], log["test_equ_min"], log["test_equ_mid"], log["train_std"],
            log["train_minmax"], log["test_std"], log["test_minmax"], [], [], log["logs_txt"])


# --------------------------------------------------------------------------- evaluation
def _moved(model, u, xi):
    """xi + grad(phi) of one trajectory: autograd in train() mode (as the
    reference, whose training loop evaluates the model in its training mode),
    the analytic VJP (DMM.mesh) in eval()."""
    if not model.training:
        return model.mesh(u, xi)
    x1, x2 = xi[:, [0]].clone(), xi[:, [1]].clone()
    x1.requires_grad = True
    x2.requires_grad = True
    phi = model(u, torch.cat((x1, x2), dim=-1))
    return torch.cat((_grad(phi, x1) + x1, _grad(phi, x2) + x2), -1).detach()


def evaluate_tri(model, u, grid, device, epoch=None):
    """dmm_utils.py:1162-1232: on up to 150 random fields, the monitor at each
    moved triangle's centroid times its area (Delaunay triangles of the fixed
    mesh), averaged: (mean, std, max - min) over triangles, mean over fields."""
    from scipy.spatial import Delaunay

    u = u.to(device)
    grid = grid.to(device).float()
    N = u.shape[-1]
    n = int(np.sqrt(N))
    tris = torch.from_numpy(Delaunay(grid.detach().cpu().numpy()).simplices.astype(np.int64)).to(device)
    lat = unit_lattice(n, device)
    stats = []
    for t in np.random.choice(u.shape[0], min(150, u.shape[0]), replace=False):
        x = _moved(model, u[[t]], grid)
        v = x[tris]                                                    # [T, 3, 2]
        area = 0.5 * torch.abs(v[:, 0, 0] * (v[:, 1, 1] - v[:, 2, 1]) + v[:, 1, 0] * (v[:, 2, 1] - v[:, 0, 1])
                               + v[:, 2, 0] * (v[:, 0, 1] - v[:, 1, 1]))
        cen = v.mean(1)
        g = softmax_interp_grad_at(grid, u[[t]], lat, float(np.sqrt(N))).reshape(1, n, n, 2)
        _, m, _ = _alpha_m_rhs(g[..., 0], g[..., 1])
        mc = interpolate_tri(m.reshape(1, -1), lat, cen[:, :1], cen[:, 1:]).reshape(-1)
        mg = mc * area
        stats.append((torch.mean(mg).item(), torch.std(mg).item(), (torch.max(mg) - torch.min(mg)).item()))
    return tuple(float(np.mean([s[i] for s in stats])) for i in range(3))


def evaluate(model, u, device, epoch=None):
    """dmm_utils.py:1235-1284 (array data u [T, s, s]): the monitor at each moved
    quadrilateral's centre times its area (product of the diagonals / 2)."""
    s = u.shape[-1]
    xi = unit_lattice(s, device)
    u = u.to(device)
    _, m, _ = _alpha_m_rhs(diff_x(u) * (s - 1), diff_y(u) * (s - 1))
    stats = []
    for t in np.random.choice(u.shape[0], u.shape[0], replace=False):
        x = _moved(model, u[[t]], xi)
        x1, x2 = x[:, 0].reshape(s, s), x[:, 1].reshape(s, s)
        bl1, bl2 = x1[:-1, :-1], x2[:-1, :-1]
        br1, br2 = x1[1:, :-1], x2[1:, :-1]
        tl1, tl2 = x1[:-1, 1:], x2[:-1, 1:]
        tr1, tr2 = x1[1:, 1:], x2[1:, 1:]
        d1 = ((bl1 - tr1) ** 2 + (bl2 - tr2) ** 2) ** 0.5
        d2 = ((br1 - tl1) ** 2 + (br2 - tl2) ** 2) ** 0.5
        area = d1 * d2 / 2
        c1 = (bl1 + br1 + tl1 + tr1) / 4
        c2 = (bl2 + br2 + tl2 + tr2) / 4
        mc = interpolate(m[[t]], c1.reshape(-1, 1), c2.reshape(-1, 1)).reshape(s - 1, s - 1)
        mg = mc * area
        stats.append((torch.mean(mg).item(), torch.std(mg).item(), (torch.max(mg) - torch.min(mg)).item()))
    return tuple(float(np.mean([st[i] for st in stats])) for i in range(3))
