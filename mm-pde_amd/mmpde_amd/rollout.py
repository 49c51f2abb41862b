"""Autoregressive MM-PDE rollout engine (the benchmarked hot path).

One step is the forward of train_helper_2d.py:174-185 (test_timestep_losses),
composed directly on the C-ABI with every buffer preallocated:

    pred = interpolate_pred(itp, model_b(graph_moved), graph_moved, data) + model(graph_uni)

cylinder (DMM graph mode):
    mesh   = DMM.mesh(u, grid)                      # x = xi + d(phi)/d(xi)
    nbr_m  = knn_graph(mesh, k=35)                  # moved-mesh graph (every step)
    out_b  = model_b(u, (t, mesh), nbr_m)
    idx    = knn_query(src=mesh, qry=grid, k=30)    # sklearn replacement
    pred   = itp_interp(mesh, out_b, grid, idx, '2') + res_cut(u) + model(u, (t, grid), nbr_u)
Burgers (DMM array mode) additionally interpolates u onto the moved mesh first
(ItpNet mode '1'); the reference's interpolation of the *labels* onto the
moved mesh (data_creator_2d.py:208-209) feeds only graph.y, which no step
reads, so the rollout (which has no labels) does not compute it.

The fixed-grid GNN runs on a side stream beside the moving-mesh chain.

Rollout: the prediction becomes the next step's input (u <- pred, t index + 1),
which the reference itself never does (it only evaluates one-step losses,
SURVEY.md §3); ``step`` is that one-step forward.  What depends only on the
fixed grid and the weights is built once at construction: the fixed-grid graph
(``nbr_u``) and the DMM head's grid side (trunk(xi), Q, J; ``dmm_cache``).
Changing weights after construction needs a new engine.
"""
from __future__ import annotations

import torch

from . import _lib as L
from . import ops


# default of MMPDERollout.priorities (set_priorities)
PRIORITIES = False


class MMPDERollout:
    def __init__(self, kind, model, model_b, itp, dmm, graph_creator, batches: int, device,
                 moving_mesh: bool = True):
        self.kind = kind
        self.model, self.model_b, self.itp, self.dmm = model, model_b, itp, dmm
        self.gc = graph_creator
        self.B = batches
        self.device = torch.device(device)
        self.moving_mesh = moving_mesh
        self.trace_hook = None   # callable() -> _lib.GnnTrace | None, one per GNN forward
        self._knn_used = {}      # kNN searches that used the candidate table in the last step
        # run the fixed-grid model beside the moving-mesh chain (False: one stream,
        # e.g. to time single kernels without a concurrent neighbour)
        self.overlap = True
        # stream priorities (set_priorities): the moving-mesh chain and the
        # kNN-30 query at high priority, the fixed-grid model at low priority
        self.priorities = PRIORITIES
        gc = graph_creator
        self.grid = gc.uniform_grid(self.device).contiguous()           # [N, 2]
        self.N = N = self.grid.shape[0]
        self.n = n = batches * N
        self.grid_rep = self.grid.repeat(batches, 1).contiguous()        # [B*N, 2]
        self.nbr_u = gc.fixed_graph_nbr(self.grid, batches)
        self.t = gc.time_grid()
        f32 = dict(dtype=torch.float32, device=self.device)
        self.out_u = torch.empty((n, 1), **f32)
        self.out_b = torch.empty((n, 1), **f32)
        self.ws_gnn = torch.empty((L.lib().mmpde_gnn_workspace_bytes(n) // 4,), **f32)
        if moving_mesh:
            hd = dmm.device_params()[1]
            self.ws_dmm = torch.empty(
                (L.lib().mmpde_dmm_workspace_bytes(batches, N, hd.latent, hd.hidden) // 4,), **f32)
            self.mesh = torch.empty((n, 2), **f32)
            if kind == "burgers":
                s = int(round(N ** 0.5))
                self.s = s
                self.xi = gc.xi_grid_xy(s, s, self.device)
            else:
                self.xi = self.grid
            for mode in ("1", "2") if kind == "burgers" else ("2",):
                itp.packed(mode)
            # the DMM head's grid side depends on xi and the weights only
            self.dmm_cache = dmm.head_cache(self.xi, workspace=self.ws_dmm)
            # the moved-mesh graph from the 128 nearest of each xi point, the
            # kNN-30 query of the fixed grid from the 128 nearest xi points of
            # each grid point (exact: csrc/knn.hip knn_cand_kernel, full search
            # where its bound fails).  Burgers' grid is in 'ij' order and xi in
            # 'xy' order, so the query table is built for the grid's own order.
            self.knn_cand = ops.knn_candidates(self.xi)
            self.knn_cand_q = (self.knn_cand if self.grid is self.xi
                               else ops.knn_candidates(self.xi, ref=self.grid))
            # trajectories whose typical displacement exceeds these go straight
            # to the full search (about half the lookups would fail; read once)
            self.knn_skip = ops.knn_skip_threshold(self.xi, self.knn_cand, gc.n + 1, moved_queries=True)
            self.knn_skip_q = ops.knn_skip_threshold(self.xi, self.knn_cand_q, 30, ref=self.grid)
            nb = max(L.lib().mmpde_knn_graph_cand_scratch_bytes(batches, N), 1)
            self.knn_scratch = torch.empty((nb,), dtype=torch.uint8, device=self.device)
            # the kNN-30 query runs on side2 beside the graph: its own scratch
            self.knn_scratch_q = torch.empty((nb,), dtype=torch.uint8, device=self.device)
            # queries of the kNN-30 searches whose sorted fp64 distances hold an
            # exact tie (sklearn's order unpinned there): cumulative, read by
            # knn_query_ties()
            self.knn_ties = torch.zeros((1,), dtype=torch.int32, device=self.device)
            # per-step displacement record shared by both (ops.knn_moved_cells)
            self.knn_cells = torch.empty((L.lib().mmpde_knn_moved_cells_bytes(batches) // 4,),
                                         dtype=torch.float32, device=self.device)
            if kind == "burgers":
                # mode '1': kNN-30 of the moved mesh (near xi, 'xy' order) onto the
                # fixed grid: a table of the 128 grid points nearest each xi point,
                # and a displacement record of the unmoved grid (all zero)
                # (rebuilt every step, which also zeroes its miss counters)
                self.knn_cand_1 = ops.knn_candidates(self.grid, ref=self.xi)
                self.knn_skip_1 = ops.knn_skip_threshold(self.grid, self.knn_cand_1, 30, ref=self.xi,
                                                         moved_queries=True)
                self.knn_cells_1 = torch.empty_like(self.knn_cells)
                self.knn_scratch_1 = torch.empty((nb,), dtype=torch.uint8, device=self.device)
            # table vs full search per role, from the share the table answered at
            # an earlier step (ops.KnnTablePolicy: the cost model, no sync)
            self.knn_policy = ops.KnnTablePolicy(
                self.device, batches, N, ("graph", "query") + (("query1",) if kind == "burgers" else ()))
            # the fixed-grid model depends on u only: it runs on a side stream,
            # with its own workspace, beside the moving-mesh chain
            self.ws_gnn_u = torch.empty_like(self.ws_gnn)
            # the kNN-30 query onto the fixed grid and res_cut need only the mesh
            # and u: a second side stream runs them beside the moved-mesh graph
            # and model_b
            self.set_priorities(self.priorities)

        # hipGraph replay of the step (enable_graph): static input / time /
        # output buffers, one graph per stage, replayed on the stage's stream
        self._graphs = None
        self._g_u = self._g_t = self._g_out = None

    def set_priorities(self, on: bool) -> None:
        """on: the moving-mesh chain (DMM, kNN graph, model_b) runs on a
        high-priority stream and the kNN-30 query / res_cut on another, the
        fixed-grid model(u) on a low-priority one, so that the chain's small
        kernels take the SIMDs the fixed-grid GNN's kernels free before that
        GNN's next launch does (the chain gates model_b).  off: default
        priorities, the chain on the caller's stream.  Which stream runs a
        kernel does not change its result."""
        if not self.moving_mesh:
            return
        self.priorities = bool(on)
        hi, lo = (-8, 8) if on else (0, 0)   # torch clamps to the device's range
        self.side = torch.cuda.Stream(self.device, priority=lo)
        self.side2 = torch.cuda.Stream(self.device, priority=hi)
        self.main_hi = torch.cuda.Stream(self.device, priority=hi) if on else None
        self._graphs = None

    def _trace(self):
        return self.trace_hook() if self.trace_hook is not None else None

    def _nodes(self, u, xy, nbr, step_idx):
        """The GNN's node inputs with (x, y) positions and one t for every node
        (mmpde_gnn_scales.pos_xy): no (t, x, y) array is filled per step.  Graph
        capture passes the device slot holding t."""
        if isinstance(step_idx, torch.Tensor):
            return _Nodes(u, xy, nbr, self.N, t_slot=step_idx)
        return _Nodes(u, xy, nbr, self.N, t=float(self.t[step_idx]))

    # ------------------------------------------------------------ the stages
    # The moving-mesh step is five stages on three streams (every kernel is one
    # of the C-ABI's; each stage runs on the caller's current stream):
    #   side   model(u) on the fixed grid                       needs u
    #   main1  DMM mesh, per-trajectory displacement record     needs u
    #   side2  kNN-30 query onto the fixed grid, res_cut(u)     needs main1
    #   main2  moved-mesh kNN-35 graph (Burgers: u onto the moved mesh), model_b
    #   final  interpolation + res_cut + model(u) in one kernel  needs all
    def _st_side(self, u_flat, step_idx):
        nodes_u = self._nodes(u_flat, self.grid_rep, self.nbr_u, step_idx)
        self.model(nodes_u, out=self.out_u, workspace=self.ws_gnn_u, trace=self._trace())

    def _st_main1(self, u):
        B = self.B
        self.dmm.mesh(u, self.xi, out=self.mesh, workspace=self.ws_dmm, head_cache=self.dmm_cache)
        pol = self.knn_policy
        self._use_g, self._use_q = pol.use_table("graph"), pol.use_table("query")
        self._knn_used = {"graph": self._use_g, "query": self._use_q}
        self._cells = ops.knn_moved_cells(self.mesh, self.xi, B, out=self.knn_cells) \
            if self.knn_cand is not None and (self._use_g or self._use_q) else None

    def _st_side2(self, u):
        B, N = self.B, self.N
        pol, cells, mesh = self.knn_policy, self._cells, self.mesh
        if self._use_q:
            idx2 = ops.knn_query_moved(mesh, self.grid_rep, self.xi, self.knn_cand_q, B, 30,
                                       self.knn_scratch_q, ref=self.grid, cells=cells,
                                       skip_above=self.knn_skip_q, ties=self.knn_ties)
            if cells is not None:
                pol.after_table("query", cells, 1)
        else:
            idx2 = ops.knn_query(mesh, self.grid_rep, B, 30, ties=self.knn_ties)
        self.idx2 = idx2
        if self.kind == "burgers":
            self._res = self.itp.res_cut(u.reshape(B, 1, self.s, self.s)).reshape(-1)
        else:
            self._res = self.itp.res_cut(u.reshape(B, N)).reshape(-1)

    def _st_main2(self, u_flat, step_idx):
        B = self.B
        pol, cells, mesh = self.knn_policy, self._cells, self.mesh
        if self._use_g:
            nbr_m = ops.knn_graph_moved(mesh, self.xi, self.knn_cand, B, self.gc.n, self.knn_scratch,
                                        cells=cells, skip_above=self.knn_skip)
            if cells is not None:
                pol.after_table("graph", cells, 0)
        else:
            nbr_m = ops.knn_graph_nbr(mesh, B, self.gc.n)
        self.nbr_m = nbr_m
        if self.kind == "burgers":
            self._knn_used["query1"] = pol.use_table("query1")
            if self._knn_used["query1"]:
                cells1 = ops.knn_moved_cells(self.grid_rep, self.grid, B, out=self.knn_cells_1)
                idx1 = ops.knn_query_moved(self.grid_rep, mesh, self.grid, self.knn_cand_1, B, 30,
                                           self.knn_scratch_1, ref=self.xi, cells=cells1,
                                           skip_above=self.knn_skip_1, ties=self.knn_ties)
                if self.knn_cand_1 is not None:
                    pol.after_table("query1", cells1, 1)
            else:
                idx1 = ops.knn_query(self.grid_rep, mesh, B, 30, ties=self.knn_ties)
            self.idx1 = idx1
            u_m = ops.itp_interp(self.grid_rep, u_flat, mesh, idx1, B, self.itp.packed("1"))
        else:
            u_m = u_flat
        nodes_m = self._nodes(u_m, mesh, nbr_m, step_idx)
        self.model_b(nodes_m, out=self.out_b, workspace=self.ws_gnn, trace=self._trace())

    def _st_final(self):
        # interpolate_pred(...) + model(graph_uniform) (train_helper_2d.py:178-185):
        # (interp + res_cut) + out_u in the interpolation kernel's epilogue
        return ops.itp_interp(self.mesh, self.out_b, self.grid_rep, self.idx2, self.B, self.itp.packed("2"),
                              addend=self._res, addend2=self.out_u.reshape(-1))

    # ------------------------------------------------------------ hipGraph
    def enable_graph(self, u_like: torch.Tensor, serial: bool = False) -> None:
        """Capture the step for replay: one hipGraph per stage (see the stage
        list above), each captured on the stream it replays on, with its own
        memory pool (two stages that replay concurrently never share scratch).
        `graph_step` replays them with the eager step's cross-stream waits, so
        the side streams' stages still run beside the main chain (a single
        graph of the whole step replays its branches one after the other).
        The step must have run eagerly once before (weight images packed, DMM
        head cache built).  Inputs are copied into static buffers; the time
        value is read from a one-element device slot, so the graphs serve every
        step index.  serial: every stage captured and replayed on one stream (the
        measurement baseline of the side streams' overlap)."""
        if self.trace_hook is not None:
            raise ValueError("graph replay records no per-kernel events; clear trace_hook")
        self._g_u = torch.empty_like(u_like).contiguous()
        self._g_u.copy_(u_like)
        self._g_t = torch.zeros((1,), dtype=torch.float32, device=self.device)
        u, t = self._g_u, self._g_t
        u_flat = u.reshape(-1)
        torch.cuda.synchronize(self.device)
        cap = torch.cuda.Stream(self.device)
        graphs = {}

        def capture(name, stream, fn):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=stream):
                out = fn()
            torch.cuda.synchronize(self.device)
            graphs[name] = g
            return out

        if not self.moving_mesh:
            self._g_out = capture("main", cap, lambda: self.model(
                self._nodes(u_flat, self.grid_rep, self.nbr_u, t), out=self.out_u,
                workspace=self.ws_gnn).reshape(u.shape))
        else:
            capture("side", cap if serial else self.side, lambda: self._st_side(u_flat, t))
            capture("main1", cap, lambda: self._st_main1(u))
            capture("side2", cap if serial else self.side2, lambda: self._st_side2(u))
            capture("main2", cap, lambda: self._st_main2(u_flat, t))
            self._g_out = capture("final", cap, self._st_final).reshape(u.shape)
        self._graphs = graphs
        self._graph_serial = serial

    def graph_step(self, u: torch.Tensor, step_idx: int) -> torch.Tensor:
        """`step` by replaying the captured graphs.  Returns the static output
        buffer (overwritten by the next replay; clone to keep it)."""
        if self._graphs is None:
            raise RuntimeError("enable_graph() first")
        if u.data_ptr() != self._g_u.data_ptr():
            self._g_u.copy_(u.reshape(self._g_u.shape))
        self._g_t.fill_(float(self.t[step_idx]))
        g = self._graphs
        if not self.moving_mesh:
            g["main"].replay()
            return self._g_out
        if self._graph_serial:
            for name in ("side", "main1", "side2", "main2", "final"):
                g[name].replay()
            return self._g_out
        cur = torch.cuda.current_stream(self.device)
        self.side.wait_stream(cur)
        with torch.cuda.stream(self.side):
            g["side"].replay()
        g["main1"].replay()
        self.side2.wait_stream(cur)
        with torch.cuda.stream(self.side2):
            g["side2"].replay()
        g["main2"].replay()
        cur.wait_stream(self.side)
        cur.wait_stream(self.side2)
        g["final"].replay()
        return self._g_out

    def step(self, u: torch.Tensor, step_idx) -> torch.Tensor:
        """u: [B, N] (cylinder) or [B, s, s] (Burgers) on the device -> pred, same shape.
        step_idx: time index (int), or during graph capture the device slot holding t."""
        u = u.contiguous()
        u_flat = u.reshape(-1)
        if not self.moving_mesh:
            return self.model(self._nodes(u_flat, self.grid_rep, self.nbr_u, step_idx), out=self.out_u,
                              workspace=self.ws_gnn, trace=self._trace()).reshape(u.shape)
        cur = torch.cuda.current_stream(self.device)
        side = self.side if self.overlap else cur
        main = self.main_hi if self.overlap and self.main_hi is not None else cur
        if main is not cur:   # the chain first: its first kernel is queued before model(u)'s
            main.wait_stream(cur)
            u.record_stream(main)
        side.wait_stream(cur)
        if main is not cur:
            with torch.cuda.stream(main):
                self._st_main1(u)
        with torch.cuda.stream(side):
            u.record_stream(side)
            self._st_side(u_flat, step_idx)
        if main is cur:
            self._st_main1(u)
        side2 = self.side2 if self.overlap else cur
        side2.wait_stream(main)
        with torch.cuda.stream(side2):
            u.record_stream(side2)
            self._st_side2(u)
            self.idx2.record_stream(cur)
            self._res.record_stream(cur)
        with torch.cuda.stream(main):
            self._st_main2(u_flat, step_idx)
        if main is not cur:
            cur.wait_stream(main)
        cur.wait_stream(side)
        cur.wait_stream(side2)
        return self._st_final().reshape(u.shape)

    def knn_table_share(self):
        """(graph, query[, burgers mode-'1' query]): the share of the last step's
        moved-mesh kNN lookups the candidate tables answered (the rest went to
        the full search); None for a search the policy ran without the table
        that step (ops.KnnTablePolicy).  Diagnostics: synchronises the device."""
        if not self.moving_mesh or self.knn_cand is None:
            return None
        torch.cuda.synchronize(self.device)
        used = self._knn_used
        s = ops.knn_table_share(self.knn_cells, self.B, self.N).mean(0).tolist()
        s = [s[0] if used.get("graph") else None, s[1] if used.get("query") else None]
        if self.kind == "burgers":
            s.append(ops.knn_table_share(self.knn_cells_1, self.B, self.N)[:, 1].mean().item()
                     if used.get("query1") else None)
        return tuple(s)

    def knn_modes(self):
        """Per kNN search of the step: 'table', 'full' or 'probe' (ops.KnnTablePolicy)."""
        if not self.moving_mesh:
            return {}
        return {r: self.knn_policy.mode(r) for r in self.knn_policy.state}

    def knn_query_ties(self) -> int:
        """Queries of the kNN-30 searches (reference data_creator_2d.py:75-76)
        since construction whose sorted fp64 distances held an exact tie inside
        the first 30 or at rank 30: the only inputs on which sklearn's order (its
        KD-tree traversal) may differ from the engine's (distance, index) order,
        i.e. where parity with the reference is unpinned.  Synchronises."""
        if not self.moving_mesh:
            return 0
        torch.cuda.synchronize(self.device)
        return int(self.knn_ties.item())

    def rollout(self, u0: torch.Tensor, start_step: int, n_steps: int):
        """Feed each prediction back as the next input; returns the final state."""
        u = u0
        for s in range(start_step, start_step + n_steps):
            u = self.step(u, s)
        return u


class _Nodes:
    """The graph fields the solver reads (x, pos, nbr, seg_n = nodes per
    trajectory); pos [n, 2] = (x, y) with t (host float) or t_slot (device
    scalar) for every node, or the reference's [n, 3] (t, x, y)."""
    __slots__ = ("x", "pos", "nbr", "edge_index", "seg_n", "t", "t_slot")

    def __init__(self, x, pos, nbr, seg_n=None, t=None, t_slot=None):
        self.x = x.reshape(-1, 1)
        self.pos = pos
        self.nbr = nbr
        self.edge_index = None
        self.seg_n = seg_n
        self.t = t
        self.t_slot = t_slot
