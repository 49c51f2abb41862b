"""Moved-mesh kNN graph: full search vs candidate table (profiling aid).
Cylinder-sized synthetic mesh, B trajectories moved by a displacement of the
given size; prints both times and the share of queries the table answered.
    python tools/knn_cand_time.py [B] [disp]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mm-pde_amd"))
import torch  # noqa: E402

from mmpde_amd import _lib as L, ops  # noqa: E402
from mmpde_amd.synth import cy_synth_mesh  # noqa: E402


def timed(fn, reps=50):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return 1e3 * a.elapsed_time(b) / reps


B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
disp = float(sys.argv[2]) if len(sys.argv) > 2 else 0.004
dev = torch.device("cuda:0")
xi = cy_synth_mesh().to(dev)
N = xi.shape[0]
gen = torch.Generator(device=dev).manual_seed(3)
pos = (xi.repeat(B, 1) + disp * torch.randn((B * N, 2), generator=gen, device=dev)).contiguous()
cand = ops.knn_candidates(xi)
need = L.lib().mmpde_knn_graph_cand_scratch_bytes(B, N)
scr = torch.zeros((need,), dtype=torch.uint8, device=dev)
t_full = timed(lambda: ops.knn_graph_nbr(pos, B, 35))
t_cand = timed(lambda: ops.knn_graph_moved(pos, xi, cand, B, 35, scr))
same = torch.equal(ops.knn_graph_nbr(pos, B, 35), ops.knn_graph_moved(pos, xi, cand, B, 35, scr))
done = scr[need - B * N:].float().mean().item()
print(f"B={B} N={N} disp={disp}: full {t_full:.1f} us, candidates {t_cand:.1f} us, "
      f"answered by table {100 * done:.1f}%, equal {same}")
qry = xi.repeat(B, 1).contiguous()
t_fq = timed(lambda: ops.knn_query(pos, qry, B, 30))
t_cq = timed(lambda: ops.knn_query_moved(pos, qry, xi, cand, B, 30, scr))
same = torch.equal(ops.knn_query(pos, qry, B, 30), ops.knn_query_moved(pos, qry, xi, cand, B, 30, scr))
done = scr[need - B * N:].float().mean().item()
print(f"  query k=30: full {t_fq:.1f} us, candidates {t_cq:.1f} us, answered by table "
      f"{100 * done:.1f}%, equal {same}")

# the bench's own moved meshes: share of queries the table answers over a rollout
from mmpde_amd.rollout import MMPDERollout  # noqa: E402
from mmpde_amd.synth import build_models, fields  # noqa: E402

pde, model, model_b, itp, dmm, gc = build_models("cy", moving_mesh=True)
for m in (model, model_b, itp, dmm):
    m.to(dev)
eng = MMPDERollout("cy", model, model_b, itp, dmm, gc, B, dev, moving_mesh=True)
u = fields(pde.ori_grid, B, 30)[:, 0].to(dev).contiguous()
shares, dmax = [], []
with torch.no_grad():
    for i in range(10):
        u = eng.step(u, 1 + i)
        torch.cuda.synchronize()
        s = eng.knn_scratch
        shares.append(s[s.numel() - B * N:].float().mean().item())
        dmax.append(s[:4 * B].view(torch.float32).max().item())
print("bench rollout: table share per step", [round(x, 4) for x in shares],
      "max displacement", [round(x, 4) for x in dmax])
