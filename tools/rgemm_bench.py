"""Row-GEMM timing (csrc/rgemm.hip via ops.LinearRows) against torch's library
GEMM at the train-mode GNN shapes (cy B=16: n = 40336 rows): forward
y = x W^T + b, input gradient dX = dY W, weight gradient dW = dY^T X (+ db).
HIP events on the current stream around 20 back-to-back calls.

    python tools/rgemm_bench.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mm-pde_amd")]

import torch  # noqa: E402


def timed(fn, reps=20):
    """Microseconds per call of `reps` back-to-back calls (the host's issue time
    overlaps the device work when the kernels are the longer part)."""
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    from mmpde_amd import rows
    dev = torch.device("cuda:0")
    out = []
    for n, k, nout in ((40336, 128, 128), (40336, 256, 128), (40336, 128, 256), (40336, 62, 128),
                       (40336, 128, 64), (40336, 64, 30)):
        x = torch.randn(n, k, device=dev)
        w = torch.randn(nout, k, device=dev)
        b = torch.randn(nout, device=dev)
        dy = torch.randn(n, nout, device=dev)
        dw = torch.empty(nout, k, device=dev)
        db = torch.empty(nout, device=dev)
        r = {"n": n, "k": k, "nout": nout,
             "fwd_us": timed(lambda: rows.linear_fwd(x, w, b)),
             "fwd_torch_us": timed(lambda: torch.addmm(b, x, w.t())),
             "dx_us": timed(lambda: rows.linear_bwd_input(dy, w)),
             "dx_torch_us": timed(lambda: dy @ w),
             "dw_us": timed(lambda: rows.linear_bwd_weight(dy, x, dw, db)),
             "dw_torch_us": timed(lambda: (dy.t() @ x, dy.sum(0)))}
        flop = 2 * n * k * nout
        r["fwd_tflops"] = flop / r["fwd_us"] / 1e6
        out.append(r)
        print(json.dumps({q: (round(v, 2) if isinstance(v, float) else v) for q, v in r.items()}), flush=True)


if __name__ == "__main__":
    main()
