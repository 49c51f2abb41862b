"""Probe: one rollout step captured as a HIP graph vs eager launches (timing only)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mm-pde_amd"))
from mmpde_amd.rollout import MMPDERollout  # noqa: E402
from mmpde_amd.synth import build_models, fields  # noqa: E402

dev = torch.device("cuda:0")
pde, model, model_b, itp, dmm, gc = build_models("cy", moving_mesh=True)
for m in (model, model_b, itp, dmm):
    m.to(dev)
for m in (model, model_b):
    m.edge_gemm = "f16x3"
B = 16
u_all = fields(pde.ori_grid, B, 30)
eng = MMPDERollout("cy", model, model_b, itp, dmm, gc, B, dev)
u0 = u_all[:, 0].to(dev).contiguous()
K = 40
with torch.no_grad():
    u = u0
    for i in range(3):
        u = eng.step(u, 1 + i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    u = u0
    for i in range(K):
        u = eng.step(u, 5)
    torch.cuda.synchronize()
    te = (time.perf_counter() - t0) / K
    ue = u.clone()

    us = u0.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            us.copy_(eng.step(us, 5))
    torch.cuda.current_stream().wait_stream(s)
    us.copy_(u0)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        us.copy_(eng.step(us, 5))
    us.copy_(u0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        g.replay()
    torch.cuda.synchronize()
    tg = (time.perf_counter() - t0) / K
    d = ((us - ue).abs().max() / ue.abs().max()).item()
print(f"eager {1e3 * te:.3f} ms/step  graph {1e3 * tg:.3f} ms/step  max rel diff {d:.3e}")
