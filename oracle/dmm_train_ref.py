"""oracle/dmm_train_ref.py -- TEST INFRASTRUCTURE ONLY.  CPU restatement of the
DMM training pieces of the reference (mesh/dmm_utils.py), used by
tests/test_gpu_dmm_train.py as the checker of mmpde_amd.dmm_train.  Only tests
import it.  Written from the reference's source text (running the reference
was refused), with the reference's own tensor formulas:
explicit [queries, points] distance / softmax tensors for the two
interpolations, autograd.grad(create_graph=True) for the derivatives of phi,
numpy's global RNG for sampling in the reference's call order.  The DMM
forward is refcpu.dmm_forward(train=True) on a state dict whose tensors may
require grad.  Parity pinned by torch (same ops); the numpy RNG by numpy.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from . import refcpu


def lattice(n, dtype=torch.float64):
    """meshgrid(linspace(0,1,n), linspace(0,1,n)) 'xy', flattened [n^2, 2]
    (dmm_utils.py:241-243), rounded to fp32 as the reference's
    torch.tensor(..., dtype=torch.float)."""
    a = np.linspace(0, 1, n)
    return torch.tensor(np.array(np.meshgrid(a, a)), dtype=torch.float).to(dtype).reshape(2, -1).t()


def interpolate(u, x, y):
    """dmm_utils.py:233-249: u [b, n, n] (one field per query), x, y [b, 1]."""
    n = u.shape[-1]
    g = lattice(n, u.dtype)
    d = -torch.norm(g[None].expand(x.shape[0], -1, -1) - torch.cat((x, y), -1)[:, None, :], dim=-1) * n
    w = torch.softmax(d, dim=-1)
    return torch.sum(u.reshape(-1, n * n) * w, dim=-1)[:, None]


def interpolate_tri(u, ori_x, ori_y, x, y):
    """dmm_utils.py:251-267: u [b, n], ori_x/ori_y [b, n, 1], x/y [b, n, 1]."""
    n = u.shape[-1]
    d = -torch.norm(torch.cat((ori_x, ori_y), -1) - torch.cat((x, y), -1), dim=-1) * np.sqrt(n)
    return torch.sum(u * torch.softmax(d, dim=-1), dim=-1)[:, None]


def monitor(alpha, ux, uy):
    return 1 + (torch.abs(ux) ** 2 + torch.abs(uy) ** 2) ** (1 / 2) / (0.01 * alpha)


def diff_x(u):
    d = torch.zeros_like(u)
    d[:, :-1, :] = torch.diff(u, dim=-2)
    d[:, -1, :] = d[:, -2, :]
    return d


def diff_y(u):
    d = torch.zeros_like(u)
    d[:, :, :-1] = torch.diff(u, dim=-1)
    d[:, :, -1] = d[:, :, -2]
    return d


def alpha_m_rhs(ux, uy):
    n = ux.shape[-1]
    alpha = torch.sum((torch.abs(ux) ** 2 + torch.abs(uy) ** 2) ** (1 / 2), dim=(-2, -1)) / (n - 1) ** 2
    m = monitor(alpha[:, None, None].repeat(1, n, n), ux, uy)
    return alpha, m, torch.sum(m, dim=(-2, -1)) / (n - 1) ** 2


def _grad(out, x):
    return torch.autograd.grad(out, x, grad_outputs=torch.ones_like(out), retain_graph=True,
                               create_graph=True, allow_unused=True)[0]


def tri_lattice_derivatives(u, mesh):
    """sample_train_data_tri's uni_ux, uni_uy (dmm_utils.py:128-139): the
    derivative of interpolate_tri(u, mesh, .) at the lattice points, by autograd.
    u [b, N], mesh [b, N, 2] -> ([b, n, n], [b, n, n])."""
    b, N = u.shape
    n = int(np.sqrt(N))
    g = lattice(n, u.dtype)
    gx, gy = [], []
    for f in range(b):          # one field at a time (the reference chunks by nu / 10)
        x1 = g[:, :1].clone().requires_grad_(True)
        x2 = g[:, 1:].clone().requires_grad_(True)
        u_ = interpolate_tri(u[f][None].repeat(n * n, 1), mesh[f, None, :, :1].repeat(n * n, 1, 1),
                             mesh[f, None, :, 1:].repeat(n * n, 1, 1),
                             x1[:, None, :].repeat(1, N, 1), x2[:, None, :].repeat(1, N, 1))
        gx.append(_grad(u_, x1).reshape(n, n).detach())
        gy.append(_grad(u_, x2).reshape(n, n).detach())
    return torch.stack(gx), torch.stack(gy)


def phi_fn(sd, mode, ori_grid=None, edge_index=None):
    """phi(u, X) of the DMM in train() mode (refcpu.dmm_forward(train=True))."""
    def f(u, X):
        return refcpu.dmm_forward(sd, mode, u, X, ori_grid=ori_grid, grid_edge_index=edge_index,
                                  train=True)
    return f


def boundary_loss(phi, bounds, bound_us):
    parts = []
    for side, (b, bu) in enumerate(zip(bounds, bound_us)):
        c1 = b[:, 0].reshape(-1, 1).clone().requires_grad_(True)
        c2 = b[:, 1].reshape(-1, 1).clone().requires_grad_(True)
        d = _grad(phi(bu, torch.cat((c1, c2), 1)), c1 if side < 2 else c2)
        parts.append(F.mse_loss(d, torch.zeros_like(d)))
    return sum(parts) / 4


def interior_losses(phi, u, ux, uy, alpha, rhs, x, nx):
    """dmm_utils.py:507-546 with the reference's repeats of the fields per point."""
    x1 = x[:, :1].clone().requires_grad_(True)
    x2 = x[:, 1:].clone().requires_grad_(True)
    out = phi(u, torch.cat((x1, x2), 1))
    px, py = _grad(out, x1), _grad(out, x2)
    pxy, pxx = _grad(px, x2), _grad(px, x1)
    pyx, pyy = _grad(py, x1), _grad(py, x2)
    s = ux.shape[-1]
    rep = ux[:, None].repeat(1, nx, 1, 1).reshape(-1, s, s)
    uxm = interpolate(rep, x1 + px, x2 + py)
    uym = interpolate(uy[:, None].repeat(1, nx, 1, 1).reshape(-1, s, s), x1 + px, x2 + py)
    a = uxm * (1 + pxx) + uym * pyx
    b = uxm * pxy + uym * (1 + pyy)
    m_xi = monitor(alpha[:, None].repeat(1, nx).reshape(-1, 1), a, b)
    lhs = m_xi * ((1 + pxx) * (1 + pyy) - pxy * pyx)
    loss_in = F.mse_loss(lhs / rhs[:, None].repeat(1, nx).reshape(-1, 1), torch.ones_like(lhs))
    z = torch.tensor(0).type_as(pxx)
    loss_convex = torch.mean(torch.min(z, 1 + pxx) ** 2 + torch.min(z, 1 + pyy) ** 2)
    return loss_in, loss_convex, lhs


def total_loss(phi, sample, nx, w0=1.0, w1=1000.0, w2=1.0):
    u, ux, uy, alpha, rhs, x, bounds, bound_us = sample
    lb = boundary_loss(phi, bounds, bound_us)
    li, lc, lhs = interior_losses(phi, u, ux, uy, alpha, rhs, x, nx)
    return w1 * lb + w0 * li + w2 * lc, li, lb, lc


def _choose(cand, p, nx):
    nu, K = p.shape
    x = torch.zeros(nu, nx, 2, dtype=torch.float64)
    for i in range(nu):
        x[i] = cand[i, np.random.choice(a=K, size=nx, replace=False, p=p[i] / np.sum(p[i]))]
    return x.reshape(-1, 2)


def _sides(nx):
    t = np.linspace(0, 1, int(nx / 4))
    return [torch.tensor(v, dtype=torch.float).double() for v in
            ([[0, a] for a in t], [[1, a] for a in t], [[a, 0] for a in t], [[a, 1] for a in t])]


def sample_arr(all_u, nx, nu):
    """sample_train_data + sample_train_data_bound (dmm_utils.py:29-103), array
    data all_u [T, s, s], numpy RNG calls in the reference's order; fp64."""
    cand = torch.tensor(np.random.uniform(0, 1, (nu, 40 * nx, 2)), dtype=torch.float).double()
    idx = np.random.choice(a=all_u.shape[0], size=nu, replace=True)
    u = all_u[idx].double()
    s = u.shape[-1]
    ux, uy = diff_x(u) * (s - 1), diff_y(u) * (s - 1)
    alpha, m, rhs = alpha_m_rhs(ux, uy)
    K = cand.shape[1]
    p = interpolate(m[:, None].repeat(1, K, 1, 1).reshape(-1, s, s), cand[..., :1].reshape(-1, 1),
                    cand[..., 1:].reshape(-1, 1)).reshape(nu, K).float().numpy()
    x = _choose(cand, p, nx)
    bidx = np.random.choice(a=all_u.shape[0], size=4 * nu, replace=True)
    bu = all_u[bidx].double()
    bounds = [sd.repeat(nu, 1, 1).reshape(-1, 2) for sd in _sides(nx)]
    return (u, ux, uy, alpha, rhs, x, bounds, [bu[k * nu:(k + 1) * nu] for k in range(4)])


def sample_tri(all_u, nx, nu):
    """sample_train_data_tri + sample_train_data_bound_tri (dmm_utils.py:106-206)
    with the reference's numpy RNG calls in order; fp64."""
    u = all_u[:, :, 2].double()
    cand = torch.tensor(np.random.uniform(0, 1, (nu, 40 * nx, 2)), dtype=torch.float).double()
    idx = np.random.choice(a=u.shape[0], size=nu, replace=True)
    u = u[idx]
    mesh = all_u[idx, :, :2].double()
    uni_ux, uni_uy = tri_lattice_derivatives(u, mesh)
    alpha, _, rhs = alpha_m_rhs(uni_ux, uni_uy)
    n = uni_ux.shape[-1]
    K = cand.shape[1]
    cx, cy = cand[..., :1].reshape(-1, 1), cand[..., 1:].reshape(-1, 1)
    ux_c = interpolate(uni_ux[:, None].repeat(1, K, 1, 1).reshape(-1, n, n), cx, cy).reshape(nu, K)
    uy_c = interpolate(uni_uy[:, None].repeat(1, K, 1, 1).reshape(-1, n, n), cx, cy).reshape(nu, K)
    p = monitor(alpha[:, None].repeat(1, K), ux_c, uy_c).float().numpy()
    x = _choose(cand, p, nx)
    bidx = np.random.choice(a=all_u.shape[0], size=4 * nu, replace=True)
    bu = all_u[bidx, :, 2].double()
    bounds = [sd.repeat(nu, 1, 1).reshape(-1, 2) for sd in _sides(nx)]
    return (u, uni_ux, uni_uy, alpha, rhs, x, bounds, [bu[k * nu:(k + 1) * nu] for k in range(4)])


def evaluate_tri_one(phi, u1, grid, tris):
    """One field of evaluate_tri (dmm_utils.py:1181-1228): (mean, std, max-min) of
    monitor-at-centroid x area over the moved Delaunay triangles."""
    N = u1.shape[-1]
    n = int(np.sqrt(N))
    x1 = grid[:, :1].clone().requires_grad_(True)
    x2 = grid[:, 1:].clone().requires_grad_(True)
    out = phi(u1, torch.cat((x1, x2), 1))
    pts = torch.cat((_grad(out, x1) + x1, _grad(out, x2) + x2), 1).detach()
    v = pts[tris]
    area = 0.5 * torch.abs(v[:, 0, 0] * (v[:, 1, 1] - v[:, 2, 1]) + v[:, 1, 0] * (v[:, 2, 1] - v[:, 0, 1])
                           + v[:, 2, 0] * (v[:, 0, 1] - v[:, 1, 1]))
    cen = v.mean(1)
    ux, uy = tri_lattice_derivatives(u1, grid[None])
    _, m, _ = alpha_m_rhs(ux, uy)
    g = lattice(n, u1.dtype)
    T = cen.shape[0]
    mc = interpolate_tri(m.reshape(1, -1).repeat(T, 1), g[None, :, :1].repeat(T, 1, 1),
                         g[None, :, 1:].repeat(T, 1, 1), cen[:, None, :1].repeat(1, n * n, 1),
                         cen[:, None, 1:].repeat(1, n * n, 1)).reshape(-1)
    mg = mc * area
    return torch.mean(mg).item(), torch.std(mg).item(), (torch.max(mg) - torch.min(mg)).item()


def evaluate_one(phi, u1, s):
    """One field of evaluate (dmm_utils.py:1235-1284), array data u1 [1, s, s]:
    (mean, std, max-min) of monitor-at-centre x diagonal-product area over the
    moved quadrilaterals of the s x s 'xy' lattice."""
    g = lattice(s, u1.dtype)
    x1 = g[:, :1].clone().requires_grad_(True)
    x2 = g[:, 1:].clone().requires_grad_(True)
    out = phi(u1, torch.cat((x1, x2), 1))
    X1 = (_grad(out, x1) + x1).reshape(s, s).detach()
    X2 = (_grad(out, x2) + x2).reshape(s, s).detach()
    _, m, _ = alpha_m_rhs(diff_x(u1) * (s - 1), diff_y(u1) * (s - 1))
    bl, br, tl, tr = (slice(None, -1), slice(None, -1)), (slice(1, None), slice(None, -1)), \
        (slice(None, -1), slice(1, None)), (slice(1, None), slice(1, None))
    d1 = ((X1[bl] - X1[tr]) ** 2 + (X2[bl] - X2[tr]) ** 2) ** 0.5
    d2 = ((X1[br] - X1[tl]) ** 2 + (X2[br] - X2[tl]) ** 2) ** 0.5
    c1 = (X1[bl] + X1[br] + X1[tl] + X1[tr]) / 4
    c2 = (X2[bl] + X2[br] + X2[tl] + X2[tr]) / 4
    Q = (s - 1) ** 2
    mc = interpolate(m.repeat(Q, 1, 1), c1.reshape(-1, 1), c2.reshape(-1, 1)).reshape(s - 1, s - 1)
    mg = mc * d1 * d2 / 2
    return torch.mean(mg).item(), torch.std(mg).item(), (torch.max(mg) - torch.min(mg)).item()
