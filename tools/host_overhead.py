"""Host (Python + launch) time of one rollout step against its GPU time
(profiling aid): if issuing a step takes about as long as the GPU takes to run
it, the host, not the kernels, sets the step time.
    python tools/host_overhead.py [B] [steps]"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mm-pde_amd"))
import torch  # noqa: E402

from mmpde_amd.rollout import MMPDERollout  # noqa: E402
from mmpde_amd.synth import build_models, fields  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
dev = torch.device("cuda:0")
pde, model, model_b, itp, dmm, gc = build_models("cy", moving_mesh=True)
for m in (model, model_b, itp, dmm):
    m.to(dev)
for m in (model, model_b):
    m.edge_gemm = "f16x3"
eng = MMPDERollout("cy", model, model_b, itp, dmm, gc, B, dev)
u0 = fields(pde.ori_grid, B, 30)[:, 0].to(dev).contiguous()
with torch.no_grad():
    for serial in (False, True):
        eng.overlap = not serial
        u = u0
        for i in range(5):
            u = eng.step(u, 1 + i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(K):
            u = eng.step(u, 1 + i % 29)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"{'serial' if serial else 'three streams'}: issue {1e3 * (t1 - t0) / K:.3f} ms/step, "
              f"wall {1e3 * (t2 - t0) / K:.3f} ms/step")
    eng.overlap = True
    # where the host time goes
    pr = cProfile.Profile()
    pr.enable()
    for i in range(K):
        u = eng.step(u, 1 + i % 29)
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("cumulative").print_stats(25)
    pstats.Stats(pr).sort_stats("tottime").print_stats(20)
