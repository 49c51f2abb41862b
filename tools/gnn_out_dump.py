"""Dump one GNN forward (cy, B=16, f16x3 and f32) to a file, to compare two
library builds bit for bit (profiling aid).
    python tools/gnn_out_dump.py OUT.pt"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mm-pde_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import torch  # noqa: E402

from mmpde_amd.rollout import _Nodes  # noqa: E402
from mmpde_amd.synth import build_models  # noqa: E402
from oracle import refcpu  # noqa: E402

dev = torch.device("cuda:0")
pde, model, _, _, _, gc = build_models("cy", moving_mesh=False, seed=0)
B = 16
pts = pde.ori_grid
n = B * pts.shape[0]
torch.manual_seed(7)
pos = torch.cat((torch.full((n, 1), float(gc.time_grid()[5])), pts.repeat(B, 1)), 1)
u = torch.randn(n, 1)
_, nbr, _ = refcpu.knn_graph(pts.repeat(B, 1), 35, B)
model.to(dev)
outs = {}
for mode in ("f16x3", "f32"):
    model.edge_gemm = mode
    outs[mode] = model(_Nodes(u.to(dev), pos.to(dev), nbr.int().to(dev), seg_n=pts.shape[0])).cpu()
torch.save(outs, sys.argv[1])
print("saved", {k: float(v.abs().sum()) for k, v in outs.items()})
