"""N>1 path on CPU: world_size-2 gloo ranks shard trajectories and all-gather losses."""
import os
import socket

import torch
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, q):
    import sys
    sys.path[:0] = [os.path.join(ROOT, "mm-pde_amd")]
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from mmpde_amd import dist as D

    D.init(backend="gloo")
    lo, hi = D.shard_range(total, rank, world)
    g = torch.Generator().manual_seed(0)
    pred = torch.randn(total, 50, generator=g)
    lab = torch.randn(total, 50, generator=g)
    local = D.per_trajectory_mse(pred[lo:hi], lab[lo:hi], hi - lo)
    allv = D.all_gather_losses(local, total)
    m = D.max_over_ranks(float(rank))
    D.barrier()
    q.put((rank, allv, m))
    torch.distributed.destroy_process_group()


def test_shard_range_covers_exactly():
    from mmpde_amd.dist import shard_range

    for total in (1, 7, 16, 64):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))


def test_gloo_world2_gather():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port, total, world = _free_port(), 7, 2
    ps = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    g = torch.Generator().manual_seed(0)
    pred = torch.randn(total, 50, generator=g)
    lab = torch.randn(total, 50, generator=g)
    exp = ((pred - lab) ** 2).mean(1)
    for rank, allv, m in res:
        assert torch.allclose(allv, exp)
        assert m == world - 1
