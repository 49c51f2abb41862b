"""The rollout's table / full-search policy for the moved-mesh kNN searches
(ops.KnnTablePolicy; reference data_creator_2d.py:66-78 and :260 on the DMM's
moved mesh).  Whatever the policy picks, every call's indices equal the full
search's bit for bit; small displacements keep the candidate table, large
ones (the table answers few lookups) move the search to the full scan after
the first read-back, with single-call probes after that.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("disp,want", [(0.004, "table"), (0.02, "full")])
def test_policy_mode_and_bit_exact(dev, disp, want):
    from mmpde_amd import ops
    from mmpde_amd.synth import cy_synth_mesh

    B = 4
    xi = cy_synth_mesh().to(dev)
    N = xi.shape[0]
    g = torch.Generator(device=dev).manual_seed(3)
    pos = (xi.repeat(B, 1) + disp * torch.randn((B * N, 2), generator=g, device=dev)).contiguous()
    qry = xi.repeat(B, 1).contiguous()
    cand = ops.knn_candidates(xi)
    full_g = ops.knn_graph_nbr(pos, B, 35)
    full_q = ops.knn_query(pos, qry, B, 30)
    pol = ops.KnnTablePolicy(dev, B, N, ("graph", "query"))
    pol.PROBE_EVERY = 5
    cells = torch.empty((ops.L.lib().mmpde_knn_moved_cells_bytes(B) // 4,), device=dev)
    used = {"graph": [], "query": []}
    for _ in range(24):
        ug, uq = pol.use_table("graph"), pol.use_table("query")
        used["graph"].append(ug)
        used["query"].append(uq)
        c = ops.knn_moved_cells(pos, xi, B, out=cells) if (ug or uq) else None
        if ug:
            nbr = ops.knn_graph_moved(pos, xi, cand, B, 35, cells=c)
            pol.after_table("graph", c, 0)
        else:
            nbr = ops.knn_graph_nbr(pos, B, 35)
        if uq:
            idx = ops.knn_query_moved(pos, qry, xi, cand, B, 30, cells=c)
            pol.after_table("query", c, 1)
        else:
            idx = ops.knn_query(pos, qry, B, 30)
        assert torch.equal(nbr, full_g) and torch.equal(idx, full_q)
        torch.cuda.synchronize()      # read-backs resolve at the next call
    if want == "table":
        assert pol.mode("graph") == pol.mode("query") == "table"
        assert all(used["graph"]) and all(used["query"])
    else:
        assert pol.mode("graph") in ("full", "probe")
        # after the first read-back: full search, with single-call probes
        assert 0 < sum(used["graph"][2:]) <= 6
