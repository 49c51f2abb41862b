"""A/B of the linear chain (one launch) against per-layer skinny launches at
the rollout's shapes (cy B=16): res_cut 2521-2048-512-2048-2521 and the DMM
output MLP + P (2521-512-256-64-512), HIP-event time per call on one stream,
then the bench step with both settings.  Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mm-pde_amd")]

import torch  # noqa: E402


def timed(fn, reps=200):
    for _ in range(10):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    from mmpde_amd import ops
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    out = {}
    for name, dims, acts in (("res_cut", [2521, 2048, 512, 2048, 2521], [1, 1, 1, 0]),
                             ("dmm_mlp", [2521, 512, 256, 64, 512], [1, 1, 0, 0])):
        layers = [((torch.randn(b, a, generator=g) / a ** 0.5).to(dev), torch.randn(b, generator=g).to(dev), act)
                  for a, b, act in zip(dims, dims[1:], acts)]
        x = torch.randn(16, dims[0], generator=g).to(dev)

        def sep():
            h = x
            for w, b, act in layers:
                h = ops.linear_skinny(h, w, b, act)
            return h
        out[name] = {"chain_us": round(timed(lambda: ops.linear_chain(x, layers)), 2),
                     "per_layer_us": round(timed(sep), 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
