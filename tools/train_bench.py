"""Training-iteration timing (not the headline metric).

One iteration of train_helper_2d.py:95-131 (training_loop_branch's body) on
synthetic cylinder data at BASELINE configs[3]'s shape (B trajectories of the
2521-node mesh, k = 35, DMM frozen): create_graph x 2, model_b / model
forward in train() mode, interpolate_pred, MSE, backward, AdamW step.  Prints
one JSON line with ms per iteration and node-updates/s (B*N nodes of both
GNNs' forward + backward per iteration).  The edge-stage backward kernel is
timed with HIP events around a standalone EdgeMean backward of one layer.

    python tools/train_bench.py [--batch 16] [--iters 10] [--warmup 3] [--edge-gemm f32|f16x3]

--edge-gemm sets both GNNs' edge_gemm: the edge-stage backward's three GEMMs
in exact fp32 or in the fp16x3 split (mmpde_gnn_edge_backward_ex).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mm-pde_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--edge-gemm", default="f32", choices=["f32", "f16x3"])
    ap.add_argument("--op-profile", default=None,
                    help="write torch.profiler's per-op counts of 3 iterations here, then exit")
    ap.add_argument("--host-profile", default=None,
                    help="write a cProfile summary (tottime order) of the timed iterations here")
    args = ap.parse_args()
    from mmpde_amd.gnn_2d import EdgeGraph, EdgeMean
    from mmpde_amd.synth import build_models, fields

    dev = torch.device("cuda:0")
    B = args.batch
    pde, model, model_b, itp, dmm, gc = build_models("cy", seed=0)
    u = fields(pde.ori_grid, B, 30, seed=1)
    for m in (model, model_b, itp, dmm):
        m.to(dev)
    model.edge_gemm = model_b.edge_gemm = args.edge_gemm
    model.train()
    model_b.train()
    itp.train()
    dmm.eval()
    opt = torch.optim.AdamW([{"params": model.parameters()}, {"params": model_b.parameters()},
                             {"params": itp.parameters()}], lr=1e-4)
    crit = torch.nn.MSELoss()
    steps = [(3 + 7 * b) % 27 + 1 for b in range(B)]
    data, labels = gc.create_data(u, steps)
    data, labels = data.to(dev), labels.to(dev)

    def it():
        opt.zero_grad()
        graph = gc.create_graph(itp, data, labels, steps, dev, dmm)
        graph_uni = gc.create_graph(itp, data, labels, steps, dev, None)
        pred = gc.interpolate_pred(itp, model_b(graph), graph, data, dev) + model(graph_uni)
        loss = crit(pred, labels.reshape(-1, 1))
        loss.backward()
        opt.step()
        return loss

    for _ in range(args.warmup):
        it()
    torch.cuda.synchronize()
    if args.op_profile:
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CPU]) as prof:
            for _ in range(3):
                it()
            torch.cuda.synchronize()
        with open(args.op_profile, "w") as f:
            f.write(prof.key_averages().table(sort_by="count", row_limit=60))
        return
    prof = None
    if args.host_profile:
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    t0 = time.perf_counter()
    issue = 0.0
    for _ in range(args.iters):
        t1 = time.perf_counter()
        loss = it()
        issue += time.perf_counter() - t1
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / args.iters
    if prof is not None:
        import pstats
        prof.disable()
        with open(args.host_profile, "w") as f:
            pstats.Stats(prof, stream=f).sort_stats("tottime").print_stats(45)
        prof.dump_stats(args.host_profile + ".prof")

    # one layer's edge backward alone (HIP events on the current stream)
    n = B * 2521
    g = torch.Generator(device="cpu").manual_seed(0)
    a = torch.randn(n, 128, generator=g).to(dev).requires_grad_()
    b = torch.randn(n, 128, generator=g).to(dev).requires_grad_()
    lay = model.gnn_layers[0].message_net_2[0]
    from mmpde_amd.ops import knn_graph_nbr
    graph = EdgeGraph(knn_graph_nbr(gc.uniform_grid(dev).repeat(B, 1), B, 35))
    gout = torch.randn(n, 128, device=dev)
    for _ in range(3):
        EdgeMean.apply(a, b, lay.weight, lay.bias, graph, args.edge_gemm).backward(gout)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 10
    out = EdgeMean.apply(a, b, lay.weight, lay.bias, graph, args.edge_gemm)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        torch.autograd.grad(out, (a, b, lay.weight, lay.bias), gout, retain_graph=True)
    e1.record()
    torch.cuda.synchronize()
    bwd_us = e0.elapsed_time(e1) * 1e3 / reps
    edges = n * 35
    # algorithmic: the two GEMMs of a linear layer's backward (gm1 = gz2 W2 and
    # the dW2 outer products); message_net_2's ReLU pattern comes from the
    # forward's bits (relu_mask), so z2 is not recomputed and not counted
    flops = 2 * 2 * edges * 128 * 128
    print(json.dumps({
        "what": "MM-PDE training iteration (train_helper_2d.py:95-131), cy synthetic",
        "batch": B, "nodes": n, "edge_gemm": args.edge_gemm, "ms_per_iter": round(ms, 3),
        "host_issue_ms_per_iter": round(issue * 1e3 / args.iters, 3),
        "train_node_updates_per_s": round(2 * 6 * n / (ms * 1e-3)),
        "loss": float(loss),
        "edge_backward_layer_us": round(bwd_us, 1),
        "edge_backward_tflops": round(flops / (bwd_us * 1e-6) / 1e12, 2),
        "edge_backward_peak_tflops": 157.3 if args.edge_gemm == "f32" else round(2516.6 / 3, 1),
    }))


if __name__ == "__main__":
    main()
