"""bench.py's multi-rank path (BASELINE configs[4]) run once
on the one-GPU box: two ranks under torch.distributed.run with the gloo
backend (RCCL needs one GPU per rank), both on cuda:0.  Checks the JSON line
the driver reads at N = 2: n_gpus, scaling, the contiguous per-rank shards
(dist.shard_range), a finite rollout and a positive whole-job value.  The
8-GPU RCCL run itself is the driver's."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("mode", ["strong", "weak"])
def test_bench_two_ranks_gloo(mode):
    if torch.cuda.device_count() < 1:      # counts devices without initialising HIP here
        pytest.skip("no ROCm device")
    extra = ["--global-trajectories", "10"] if mode == "strong" else ["--batch", "3"]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--dist-backend", "gloo", "--no-cpu-baseline", "--no-f32-exact"] + extra
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]            # rank 0 prints one line
    rec = json.loads(lines[0])
    print(json.dumps({k: rec[k] for k in ("value", "ms_per_step", "n_gpus", "scaling")}))
    cfg = rec["config"]
    assert rec["n_gpus"] == 2 and cfg["dist_backend"] == "gloo"
    assert rec["finite"] is True and rec["value"] > 0
    if mode == "strong":
        # 10 trajectories over 2 ranks: 5 + 5
        assert rec["scaling"] == "strong" and cfg["global_trajectories"] == 10
        assert cfg["trajectories_per_gpu"] == 5 and "rank 0 holds 5" in cfg["shard"]
        total = 10
    else:
        assert rec["scaling"] == "weak" and cfg["global_trajectories"] == 6
        assert cfg["trajectories_per_gpu"] == 3 and "rank 0 holds 3" in cfg["shard"]
        total = 6
    # value = whole-job node-updates / max-over-ranks time of the K timed steps
    assert abs(rec["value"] - total * 2521 * 3 / (rec["ms_per_step"] * 3e-3)) <= 1e-6 * rec["value"]
