"""Training-path GEMM shapes at cy B=16 (n = 40336 rows): torch / hipBLASLt
times of the node-side GEMMs of one GNN layer in train mode (gnn_2d.py
GNN_Layer_FS_2D.train_forward) -- forward y = x W^T, backward dX = dY W and
dW = dY^T x -- and dW by alternatives (profiling aid).
    python tools/gemm_shapes.py [n]"""
import sys

import torch

n = int(sys.argv[1]) if len(sys.argv) > 1 else 40336
dev = torch.device("cuda:0")


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return 1e3 * a.elapsed_time(b) / reps


g = torch.Generator(device=dev).manual_seed(0)
for K in (132, 131, 257, 128):
    x = torch.randn(n, K, device=dev, generator=g)
    w = torch.randn(128, K, device=dev, generator=g) * 0.05
    dy = torch.randn(n, 128, device=dev, generator=g)
    t_f = timed(lambda: x @ w.t())
    t_dx = timed(lambda: dy @ w)
    t_dw = timed(lambda: dy.t() @ x)
    res = [f"K={K}: fwd {t_f:.1f} us, dX {t_dx:.1f}, dW {t_dw:.1f}"]
    for C in (8, 16, 40, 79):
        R = -(-n // C)
        pad = C * R - n
        xp = torch.nn.functional.pad(x, (0, 0, 0, pad)).reshape(C, R, K)
        dyp = torch.nn.functional.pad(dy, (0, 0, 0, pad)).reshape(C, R, 128)
        t_b = timed(lambda: torch.bmm(dyp.transpose(1, 2), xp).sum(0))
        res.append(f"dW bmm C={C} {t_b:.1f}")
    xt = x.t().contiguous()
    res.append(f"dW with x^T given {timed(lambda: (xt @ dy).t()):.1f}")
    print("; ".join(res), flush=True)
