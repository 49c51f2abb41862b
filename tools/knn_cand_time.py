"""Moved-mesh kNN: full search vs candidate table (profiling aid).
Cylinder-sized synthetic mesh, B trajectories moved by random displacements
of the given size (and a case with one node of every trajectory moved far);
prints both times and the share of queries the table answered, then the share
over the bench's own rollout (cy and burgers).
    python tools/knn_cand_time.py [B] [disp ...]"""
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
disps = [float(x) for x in sys.argv[2:]] or [0.004, 0.02]
dev = torch.device("cuda:0")
xi = cy_synth_mesh().to(dev)
N = xi.shape[0]
cand = ops.knn_candidates(xi)
thr_g = ops.knn_skip_threshold(xi, cand, 36, moved_queries=True)
thr_q = ops.knn_skip_threshold(xi, cand, 30)
print(f"skip thresholds: graph {thr_g:.4f}, query {thr_q:.4f}")
need = L.lib().mmpde_knn_graph_cand_scratch_bytes(B, N)
scr = torch.zeros((need,), dtype=torch.uint8, device=dev)
qry = xi.repeat(B, 1).contiguous()
for disp in disps:
    for far in (False, True):
        gen = torch.Generator(device=dev).manual_seed(3)
        if far:   # tiny displacements everywhere, one node per trajectory moved by `disp`
            pos = (xi.repeat(B, 1) + 1e-4 * torch.randn((B * N, 2), generator=gen, device=dev))
            pos = pos.reshape(B, N, 2)
            pos[:, N // 3] += disp
            pos = pos.reshape(-1, 2).contiguous()
        else:
            pos = (xi.repeat(B, 1) + disp * torch.randn((B * N, 2), generator=gen, device=dev)).contiguous()
        what = f"one node moved {disp}" if far else f"random disp {disp}"
        cells = ops.knn_moved_cells(pos, xi, B)
        t_cells = timed(lambda: ops.knn_moved_cells(pos, xi, B, out=cells))
        t_full = timed(lambda: ops.knn_graph_nbr(pos, B, 35))
        t_cand = timed(lambda: ops.knn_graph_moved(pos, xi, cand, B, 35, scr, cells=cells))
        same = torch.equal(ops.knn_graph_nbr(pos, B, 35),
                           ops.knn_graph_moved(pos, xi, cand, B, 35, scr, cells=cells))
        cells = ops.knn_moved_cells(pos, xi, B)
        ops.knn_graph_moved(pos, xi, cand, B, 35, scr, cells=cells)
        done = ops.knn_table_share(cells, B, N)[:, 0].mean().item()
        t_skip = timed(lambda: ops.knn_graph_moved(pos, xi, cand, B, 35, scr, cells=cells,
                                                   skip_above=thr_g))
        print(f"B={B} N={N} {what}: graph full {t_full:.1f} us, candidates {t_cand:.1f} us "
              f"(+ cells {t_cells:.1f} us, shared with the query), answered by table "
              f"{100 * done:.1f}%, equal {same}; with the skip threshold {t_skip:.1f} us")
        t_fq = timed(lambda: ops.knn_query(pos, qry, B, 30))
        t_cq = timed(lambda: ops.knn_query_moved(pos, qry, xi, cand, B, 30, scr, cells=cells))
        same = torch.equal(ops.knn_query(pos, qry, B, 30),
                           ops.knn_query_moved(pos, qry, xi, cand, B, 30, scr, cells=cells))
        cells = ops.knn_moved_cells(pos, xi, B)
        ops.knn_query_moved(pos, qry, xi, cand, B, 30, scr, cells=cells)
        done = ops.knn_table_share(cells, B, N)[:, 1].mean().item()
        t_qskip = timed(lambda: ops.knn_query_moved(pos, qry, xi, cand, B, 30, scr, cells=cells,
                                                    skip_above=thr_q))
        print(f"  query k=30: full {t_fq:.1f} us, candidates {t_cq:.1f} us, answered by table "
              f"{100 * done:.1f}%, equal {same}; with the skip threshold {t_qskip:.1f} us")
        # the rollout's policy (ops.KnnTablePolicy): per role, table or full
        # search from the share read back at an earlier call, probes included
        pol = ops.KnnTablePolicy(dev, B, N, ("graph", "query"))

        def policy_step():
            ug, uq = pol.use_table("graph"), pol.use_table("query")
            c = ops.knn_moved_cells(pos, xi, B, out=cells) if (ug or uq) else None
            if ug:
                ops.knn_graph_moved(pos, xi, cand, B, 35, scr, cells=c, skip_above=thr_g)
                pol.after_table("graph", c, 0)
            else:
                ops.knn_graph_nbr(pos, B, 35)
            if uq:
                ops.knn_query_moved(pos, qry, xi, cand, B, 30, scr, cells=c, skip_above=thr_q)
                pol.after_table("query", c, 1)
            else:
                ops.knn_query(pos, qry, B, 30)
        for _ in range(8):   # the first read-backs resolve (the host runs ahead of the GPU)
            policy_step()
        torch.cuda.synchronize()
        t_pol = timed(policy_step, reps=128)
        modes = {r: pol.mode(r) for r in pol.state}
        print(f"  policy (graph + query + cells, probes every {pol.PROBE_EVERY}): {t_pol:.1f} us per call "
              f"against full {t_full + t_fq:.1f} / table {t_cand + t_cq + t_cells:.1f}; modes {modes}")

# the bench's own moved meshes: share of queries the tables answer over a rollout
from mmpde_amd.rollout import MMPDERollout  # noqa: E402
from mmpde_amd.synth import build_models, burgers_grid_points, fields  # noqa: E402

for kind, bk in (("cy", B), ("burgers", 2 * B)):
    pde, model, model_b, itp, dmm, gc = build_models(kind, moving_mesh=True)
    for m in (model, model_b, itp, dmm):
        m.to(dev)
    eng = MMPDERollout(kind, model, model_b, itp, dmm, gc, bk, dev, moving_mesh=True)
    if kind == "cy":
        u = fields(pde.ori_grid, bk, 30)[:, 0].to(dev).contiguous()
    else:
        u = fields(burgers_grid_points(), bk, 31).reshape(bk, 31, 48, 48)[:, 0].to(dev).contiguous()
    shares, dmax = [], []
    with torch.no_grad():
        for i in range(10):
            u = eng.step(u, 1 + i)
            shares.append(eng.knn_table_share())
            dmax.append((eng.mesh.reshape(bk, -1, 2) - eng.xi).norm(dim=-1).max().item())
        modes = eng.knn_modes()
    print(f"{kind} bench rollout (B={bk}): table share (graph, query[, mode-1 query]) per step",
          [tuple(None if a is None else round(a, 4) for a in sh) for sh in shares],
          "max displacement", [round(x, 4) for x in dmax], "policy after 10 steps", modes)
