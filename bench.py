#!/usr/bin/env python
"""MM-PDE rollout benchmark (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cy-mmpde]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)

A *step* is one full MM-PDE forward step over the rank's trajectories (DMM
moved mesh, moved-mesh kNN-35 graph, model_b, kNN-30 + ItpNet interpolation +
res_cut, model on the fixed-grid graph, sum), fed back autoregressively.
Default workload = BASELINE configs[3]: cylinder MM-PDE, 16 trajectories of
the 2521-node mesh per GPU (weak scaling: trajectories shard across ranks, no
data-path collective).  --global-trajectories G fixes the job instead
(configs[4]'s strong-scaling half: G = 64 split over the ranks, "scaling":
"strong").  value = node-updates/s of the whole job
= trajectories_total * 2521 * K / max-over-ranks(time of the K timed steps).

Also reported (rank 0):
* roofline: the dominant kernel (GNN edge stage, 12 launches per step) timed
  live with hipEvents recorded on its own stream around every launch, in a
  second timed pass of the same K steps run on ONE stream (the pass that sets
  `value` runs the fixed-grid model on a side stream beside the moving-mesh
  chain, where two edge kernels can share the GPU, and records no events);
  achieved = algorithmic FLOP per launch / mean launch time.
* cpu_baseline (N = 1 only): the CPU oracle (op-for-op restatement of the
  reference, oracle/refcpu.py) timed on a bounded sample on this host.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mm-pde_amd"))

import torch  # noqa: E402

METRIC = "MM-PDE rollout node-updates/sec, cylinder 2521-node mesh, 1/2/4/8 GPUs"
F32_MFMA_PEAK_TFLOPS = 157.3          # MI355X_MICROARCH.md: dense fp32 matrix peak
F16_MFMA_PEAK_TFLOPS = 2516.6         # 256 CU x 4 SIMD x 1024 FLOP/clk x 2.4 GHz (~2.5 PF dense)
HBM_PEAK_GBS = 8000.0
# counter records regenerated on the current kernels (tools/gpu_pmc.sh with
# PMC_NAME=edge_pmc_r06; tools/gpu_configs.sh with STEP_HBM=...: tools/gpu_records.sh pmc:NAME)
EDGE_PMC_RECORD = "edge_pmc_r06.json"
STEP_HBM_RECORD = "r06_cy_gnn_step_hbm.json"
CONFIGS = {
    # name: (kind, moving_mesh, default trajectories per GPU, BASELINE.json config,
    #        Burgers grid side: 48 = the MM-PDE --base_resolution, 96 = PDEs.py's default)
    "cy-mmpde": ("cy", True, 16, "configs[3]: Cylinder MM-PDE, batch=16", None),
    "cy-gnn": ("cy", False, 8, "configs[2]: Cylinder GNN, batch=8", None),
    "burgers-mmpde": ("burgers", True, 32, "configs[1]: Burgers' MM-PDE, batch=32", 48),
    "burgers-gnn": ("burgers", False, 1, "configs[0]: Burgers' GNN, default resolution 96x96, batch=1", 96),
}


def set_burgers_side(pde, s):
    """The Burgers grid (31, s, s) on a synth.build_models PDE (built at 48x48)."""
    pde.grid_size = pde.movingmesh_grid_size = pde.ori_grid_size = [31, s, s]


class HipEvents:
    """hipEvent pool through libamdhip64 (the events are recorded by the C-ABI on
    the stream the edge kernel is launched on)."""

    def __init__(self, count):
        self.h = ctypes.CDLL("libamdhip64.so")
        self.h.hipEventCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
        self.h.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p,
                                               ctypes.c_void_p]
        self.h.hipEventDestroy.argtypes = [ctypes.c_void_p]
        self.ev = []
        for _ in range(count):
            e = ctypes.c_void_p()
            if self.h.hipEventCreate(ctypes.byref(e)) != 0:
                raise RuntimeError("hipEventCreate failed")
            self.ev.append(e.value)

    def elapsed_ms(self, a, b):
        ms = ctypes.c_float()
        if self.h.hipEventElapsedTime(ctypes.byref(ms), a, b) != 0:
            raise RuntimeError("hipEventElapsedTime failed")
        return ms.value

    def close(self):
        for e in self.ev:
            self.h.hipEventDestroy(e)


class EdgeTracer:
    """Hands out one GnnExec (n_layers edge-begin / edge-end / node-end events)
    per GNN forward."""

    def __init__(self, n_forwards, n_layers=6):
        from mmpde_amd import _lib

        self.L = n_layers
        self.pool = HipEvents(3 * n_forwards * n_layers)
        self.used = 0
        self.traces = []
        self._lib = _lib
        self.active = False

    def __call__(self):
        if not self.active:
            return None
        i = self.used
        self.used += 1
        L = self.L
        base = 3 * L * i
        arr = [(ctypes.c_void_p * L)(*self.pool.ev[base + q * L:base + (q + 1) * L]) for q in range(3)]
        cast = [ctypes.cast(a, ctypes.POINTER(ctypes.c_void_p)) for a in arr]
        t = self._lib.GnnExec(cast[0], cast[1], 0, None, cast[2])
        self.traces.append((t, arr))
        return t

    def launch_times_ms(self):
        """[(layer index, edge-stage ms, node-stage ms)] for every traced layer."""
        out = []
        for _, (beg, mid, end) in self.traces:
            for l in range(self.L):
                out.append((l, self.pool.elapsed_ms(beg[l], mid[l]), self.pool.elapsed_ms(mid[l], end[l])))
        return out


def cpu_baseline(kind, moving_mesh, seconds, side=48):
    """The CPU oracle (op-for-op restatement of the reference forward, unfused,
    brute-force kNN) on a bounded sample: 2 trajectories, repeated one-step
    forwards until `seconds` of work (>= 1 step)."""
    sys.path.insert(0, ROOT)
    from mmpde_amd.synth import build_models, burgers_grid_points, fields
    from oracle import refcpu

    cores = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    torch.set_num_threads(cores)
    B = 2
    pde, model, model_b, itp, dmm, gc = build_models(kind, moving_mesh=moving_mesh)
    if kind == "cy":
        grid = pde.ori_grid
        u = fields(grid, B, 30)
        opde = refcpu.PDEConst("cy", [30, grid.shape[0]], ori_grid=grid)
        n_nodes = grid.shape[0]
    else:
        u = fields(burgers_grid_points(side), B, 31).reshape(B, 31, side, side)
        opde = refcpu.PDEConst("burgers", [31, side, side])
        n_nodes = side * side
    sds = {k: {n: t.detach() for n, t in m.state_dict().items()}
           for k, m in (("model", model), ("model_b", model_b), ("itp", itp), ("dmm", dmm))
           if m is not None}
    steps, t0 = 0, time.perf_counter()
    data = u[:, 0:1]
    while True:
        s = 1 + steps % 29
        pred, _ = refcpu.mmpde_step(opde, sds, data, data, [s] * B, moving_mesh=moving_mesh)
        data = pred.reshape(data.shape)
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": B * n_nodes * steps / el, "unit": "node-updates/s", "cores": cores,
            "kind": "port",
            "sample": f"oracle/refcpu.py, {B} trajectories x {steps} autoregressive steps "
                      f"({el:.1f} s, torch CPU fp32, {cores} threads)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="cy-mmpde", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=None,
                    help="trajectories per GPU (weak scaling: the job grows with --gpus)")
    ap.add_argument("--global-trajectories", type=int, default=None,
                    help="a FIXED number of trajectories for the whole job, sharded "
                         "contiguously across the ranks (strong scaling, BASELINE "
                         "configs[4]: 64 over 1/2/4/8 GPUs)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--edge-gemm", default="f16x3", choices=["f32", "f16x3"],
                    help="message_net_2 arithmetic (include/mmpde_hip.h MMPDE_EDGE_GEMM_*)")
    ap.add_argument("--no-f32-exact", action="store_true",
                    help="skip the second, exact-fp32-MFMA timed run reported as f32_exact")
    ap.add_argument("--graph", nargs="?", const="streams", default=None, choices=["streams", "serial"],
                    help="replay hipGraph captures of the step instead of launching it eagerly: "
                         "'streams' (default) one graph per stage replayed on the stage's own "
                         "stream (MMPDERollout.enable_graph); 'serial' every stage on one stream "
                         "(the diagnostic baseline of the stream overlap)")
    ap.add_argument("--dist-backend", default=None, choices=["nccl", "gloo"],
                    help="process-group backend under torchrun (default nccl = RCCL; gloo "
                         "lets several ranks share one GPU, for rehearsing the multi-rank path)")
    ap.add_argument("--priorities", choices=["on", "off"], default=None,
                    help="stream priorities of the step (MMPDERollout.set_priorities): the "
                         "moving-mesh chain high, the fixed-grid model low (default: the engine's)")
    ap.add_argument("--serial", action="store_true",
                    help="one stream in every pass (per-kernel profiles without concurrent "
                         "kernels sharing the GPU)")
    args = ap.parse_args()

    from mmpde_amd import dist as D
    from mmpde_amd.rollout import MMPDERollout
    from mmpde_amd.synth import build_models, burgers_grid_points, fields

    rank, local, world = D.init(args.dist_backend)
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    device = D.local_device(local)
    torch.cuda.set_device(device)
    kind, moving, b_default, cfg_name, side = CONFIGS[args.config]
    strong = args.global_trajectories is not None
    if strong:
        if args.batch is not None:
            raise SystemExit("--batch (per GPU) and --global-trajectories (whole job) exclude each other")
        total = args.global_trajectories
        if total < world:
            raise SystemExit("--global-trajectories must give every rank at least one trajectory")
        cfg_name = ("configs[4]: Cylinder MM-PDE batched rollout, trajectories sharded across GPUs"
                    if kind == "cy" and moving else cfg_name)
    else:
        total = (args.batch or b_default) * world
    lo, hi = D.shard_range(total, rank, world)
    B = hi - lo

    pde, model, model_b, itp, dmm, gc = build_models(kind, moving_mesh=moving)
    if kind == "burgers" and side != 48:
        if moving:
            raise SystemExit("the synthetic MM-PDE models are built for the 48x48 grid")
        set_burgers_side(pde, side)
    for m in (model, model_b, itp, dmm):
        if m is not None:
            m.to(device)
    for m in (model, model_b):
        if m is not None:
            m.edge_gemm = args.edge_gemm
    if kind == "cy":
        pts, t_len = pde.ori_grid, 30
        u_all = fields(pts, total, t_len)[lo:hi]
    else:
        pts, t_len = burgers_grid_points(side), 31
        u_all = fields(pts, total, t_len).reshape(total, t_len, side, side)[lo:hi]
    n_nodes = pts.shape[0]
    eng = MMPDERollout(kind, model, model_b, itp, dmm, gc, hi - lo, device, moving_mesh=moving)
    if args.priorities is not None:
        eng.set_priorities(args.priorities == "on")
    n_gnn = 2 if moving else 1
    tracer = EdgeTracer(n_forwards=n_gnn * args.steps)
    eng.trace_hook = tracer
    u0 = u_all[:, 0].to(device).contiguous()
    n_t = t_len - 1

    host_s = {}

    def timed_run(mode, trace):
        """W warmup + K timed autoregressive steps from u0; returns (max-over-ranks
        seconds, final state).  trace: record the edge-kernel events, one stream.
        host_s[(mode, trace)]: seconds the host spent inside the K step calls (issuing
        launches; equal to the wall time when the pass is host-bound)."""
        for m in (model, model_b):
            if m is not None:
                m.edge_gemm = mode
        eng.overlap = not (trace or args.serial)
        graph = args.graph and not trace
        u = u0
        with torch.no_grad():
            for i in range(args.warmup):
                u = eng.step(u, 1 + i % n_t)
            if graph:  # capture after the eager warmup (weights packed, caches built)
                hook, eng.trace_hook = eng.trace_hook, None
                eng.enable_graph(u, serial=args.graph == "serial")
                eng.trace_hook = hook
                u = u.clone()
            run = eng.graph_step if graph else eng.step
            torch.cuda.synchronize(device)
            D.barrier(device)
            tracer.active = trace
            t0 = time.perf_counter()
            for i in range(args.steps):
                u = run(u, 1 + (args.warmup + i) % n_t)
            host_s[(mode, trace)] = time.perf_counter() - t0
            torch.cuda.synchronize(device)
            D.barrier(device)
            t1 = time.perf_counter()
            tracer.active = False
        return D.max_over_ranks(t1 - t0, device), u.clone()

    elapsed, u = timed_run(args.edge_gemm, False)
    elapsed_traced, _ = timed_run(args.edge_gemm, True)
    finite = bool(torch.isfinite(u).all())
    exact = None
    if not args.no_f32_exact and args.edge_gemm != "f32":
        el32, u32 = timed_run("f32", False)
        rel = ((u - u32).abs().max() / u32.abs().max().clamp_min(1e-30)).item()
        exact = {"value": total * n_nodes * args.steps / el32,
                 "ms_per_step": 1e3 * el32 / args.steps,
                 "final_state_max_rel_diff_vs_main": rel}
    launches = tracer.launch_times_ms()
    ties = eng.knn_query_ties() if moving else 0
    tracer.pool.close()

    if rank != 0:
        return
    n_local = (hi - lo) * n_nodes
    k = gc.n
    # Dominant kernel = the edge stage (message_net_2 over every edge + mean),
    # 12 launches per step.  Algorithmic FLOP per launch:
    # n nodes x k edges x 2 x 128 x 128.
    edge_f = n_local * k * 2 * 128 * 128
    tot_ms = sum(e for _, e, _ in launches)
    node_ms = sum(nd for _, _, nd in launches)
    nl = max(len(launches), 1)
    launch_ms = tot_ms / nl
    achieved = edge_f * len(launches) / max(tot_ms * 1e-3, 1e-12) / 1e12
    # Peak of the arithmetic the kernel runs: f32 -> dense fp32 MFMA peak;
    # f16x3 -> each fp32 product is three fp16 MFMA products, so the
    # fp32-equivalent peak is the dense fp16 MFMA peak / 3.
    peak = F32_MFMA_PEAK_TFLOPS if args.edge_gemm == "f32" else F16_MFMA_PEAK_TFLOPS / 3
    traffic = None
    pmc = os.path.join(ROOT, "profiles", EDGE_PMC_RECORD)   # tools/gpu_pmc.sh on this round's kernels
    if os.path.exists(pmc):
        with open(pmc) as f:
            rec = json.load(f)
        if rec.get("workload") == args.config and rec.get("nodes") == n_local:
            traffic = rec.get("modes", {}).get(args.edge_gemm, {}).get("hbm_bytes_per_launch")
    line = {
        "metric": METRIC if kind == "cy" else METRIC.replace("cylinder 2521-node mesh",
                                                             f"Burgers {side}x{side} grid"),
        "value": total * n_nodes * args.steps / elapsed,
        "unit": "node-updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "f32" if args.edge_gemm == "f32" else
                 ("f32 (every GNN GEMM fp32-emulated by the fp16x3 split with fp32 accumulate: "
                  "edge message_net_2, node update_net_1/_2 and message_net_1 projections, "
                  "embedding; DMM, ItpNet, res_cut, kNN and heads exact fp32)"),
        "data": "synthetic: seeded cy-synth 2521-node mesh / 48x48 grid, seeded sin-cos+noise "
                "fields, seeded default-init weights (no dataset or checkpoint offline)",
        "config": {"workload": args.config, "baseline_config": cfg_name,
                   "trajectories_per_gpu": B if not strong else total / world,
                   "global_trajectories": total,
                   "nodes_per_trajectory": n_nodes, "neighbors": gc.n, "time_window": 1,
                   "parallelism": f"trajectory-shard x{world} (no data-path collective)",
                   "dist_backend": (torch.distributed.get_backend() if torch.distributed.is_initialized()
                                    else None),
                   "shard": "contiguous trajectory blocks, dist.shard_range; rank 0 holds "
                            f"{hi - lo}",
                   "rollout": "autoregressive (pred -> next input)",
                   "launch": ("hipGraph replay of the step, one graph per stage on its own stream"
                              if args.graph == "streams" else
                              "hipGraph replay of the step, every stage on one stream" if args.graph else
                              "eager, three HIP streams"),
                   "stream_priorities": bool(getattr(eng, "priorities", False))},
        "roofline": {"kernel": ("gnn_edge_wave_kernel" if args.edge_gemm == "f16x3" else "gnn_edge_kernel")
                               + " (message_net_2 over every edge + mean aggregation, one launch "
                               "per GNN layer, 12 per step)",
                     "bound": "mfma", "achieved": achieved, "peak": peak,
                     "unit": "TFLOP/s", "frac": achieved / peak,
                     "traffic": traffic, "launch_ms": launch_ms, "launches": len(launches),
                     "flop_per_launch": edge_f,
                     "traced_pass_ms_per_step": 1e3 * elapsed_traced / args.steps,
                     "traced_pass_host_ms_per_step": 1e3 * host_s[(args.edge_gemm, True)] / args.steps,
                     "algorithmic_bytes_per_launch": n_local * (128 * 4 * 2 + k * 4 + 128 * 4),
                     "edge_gemm": args.edge_gemm,
                     "peak_basis": "dense fp32 MFMA" if args.edge_gemm == "f32" else
                                   "dense fp16 MFMA / 3 (three fp16 products per fp32 product)"},
        "node_stage_ms": node_ms / nl,
        "host_issue_ms_per_step": 1e3 * host_s[(args.edge_gemm, False)] / args.steps,
        "finite": finite,
    }
    if moving:
        # kNN-30 queries with an exact fp64 distance tie (sklearn's order
        # unpinned there), over every step this process ran
        line["knn_query_ties"] = ties
    if not moving:
        # configs[2] is quoted against the scatter-add / HBM roofline: SURVEY.md
        # §8(d)'s fused minimum of ~18.7 KB of HBM traffic per GNN node-update
        # (per layer read + write h, the 2 KB of message_net_1 node halves, 35
        # neighbour ids), against rocprofv3 FETCH/WRITE of the whole step
        step_s = elapsed / args.steps
        alg = n_local * 18.7e3
        hbm = {"survey_fused_min_bytes_per_node_update": 18.7e3,
               "algorithmic_bytes_per_step": alg, "achieved": alg / step_s / 1e9,
               "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": alg / step_s / 1e9 / HBM_PEAK_GBS,
               "measured_bytes_per_step": None}
        rec_path = os.path.join(ROOT, "profiles", STEP_HBM_RECORD)
        if os.path.exists(rec_path):
            with open(rec_path) as f:
                rec = json.load(f)
            if rec.get("workload") == args.config and rec.get("nodes") == n_local:
                hbm["measured_bytes_per_step"] = rec["hbm_bytes_per_step"]
                hbm["measured_GBs"] = rec["hbm_bytes_per_step"] / step_s / 1e9
        line["hbm"] = hbm
    if exact is not None:
        line["f32_exact"] = exact
    if world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(kind, moving, args.cpu_seconds, side or 48)
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
