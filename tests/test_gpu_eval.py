"""Teacher-forced evaluation (reference test_timestep_losses,
train_helper_2d.py:137-200) on the engine, single process against the oracle,
and trajectory-sharded over two ranks (gloo collectives on CPU tensors, both
ranks on cuda:0) against the single-process run.

Bars: losses 1e-4 relative to the oracle (an MSE of fp32 predictions that
agree to ~1e-6 relative); sharded vs single process: bit for bit in both edge
GEMM modes (every kernel computes a trajectory's rows independently of the
others: the f16x3 split scale is taken per trajectory, and the edge kernel's
summation units and the skinny linears' K splits depend on the trajectory and
the layer shapes alone, never on how many trajectories share a launch), for
shards of 16, 8 and 12 trajectories per rank -- configs[4]'s strong-scaling
shards of 64 trajectories over 4 and 8 GPUs are 16 and 8 per rank.
The RCCL path of dist.py (backend "nccl") runs in a one-rank process group on
the box's one GPU: the collectives the bench and the sharded evaluation call.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from conftest import ROOT
from oracle import refcpu

pytestmark = pytest.mark.gpu


def _sds(**mods):
    return {k: {n: t.detach().cpu() for n, t in m.state_dict().items()} for k, m in mods.items()}


def _inputs(kind, total):
    from mmpde_amd.synth import build_models, burgers_grid_points, fields

    pde, model, model_b, itp, dmm, gc = build_models(kind)
    if kind == "cy":
        u = fields(pde.ori_grid, total, 30)
        opde = refcpu.PDEConst("cy", pde.grid_size, ori_grid=pde.ori_grid)
    else:
        u = fields(burgers_grid_points(), total, 31).reshape(total, 31, 48, 48)
        opde = refcpu.PDEConst("burgers", pde.grid_size)
    return pde, opde, (model, model_b, itp, dmm, gc), u


@pytest.mark.parametrize("kind", ["cy", "burgers"])
def test_timestep_losses_vs_oracle(dev, kind):
    from mmpde_amd import evaluate as EV
    from mmpde_amd.rollout import MMPDERollout

    B = 3
    pde, opde, (model, model_b, itp, dmm, gc), u = _inputs(kind, B)
    sds = _sds(model=model, model_b=model_b, itp=itp, dmm=dmm)
    for m in (model, model_b, itp, dmm):
        m.to(dev)
    assert EV.timestep_steps(1, gc.t_res) == list(range(1, gc.t_res))   # mmpde.py:139
    steps = [1, 12, gc.t_res - 1]
    eng = MMPDERollout(kind, model, model_b, itp, dmm, gc, B, dev)
    res = EV.test_timestep_losses(eng, u.to(dev), B, steps=steps)
    ref_step, ref_traj = refcpu.test_timestep_losses(opde, sds, u, steps)
    got_traj = res["per_trajectory"].cpu()
    print(kind, "per-step", res["per_step"].tolist(), "oracle", ref_step.tolist())
    assert torch.allclose(got_traj, ref_traj, rtol=1e-4, atol=0)
    assert torch.allclose(res["per_step"].cpu(), ref_step, rtol=1e-4, atol=0)
    assert abs(res["mean"].item() - ref_step.mean().item()) <= 1e-4 * ref_step.mean().item()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_worker(rank, world, port, kind, total, mode, steps, n_roll, q):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "mm-pde_amd")]
    os.environ.update(RANK=str(rank), LOCAL_RANK="0", WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        from mmpde_amd import dist as D
        from mmpde_amd import evaluate as EV
        from mmpde_amd.rollout import MMPDERollout

        D.init(backend="gloo")                 # the collectives run on CPU tensors
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        out = _run_shard(kind, total, mode, steps, n_roll, dev, D, EV, MMPDERollout)
        torch.distributed.destroy_process_group()
        q.put((rank, [t.numpy() for t in out], None))   # by value, not shared fds
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, None, repr(e)))


def _run_shard(kind, total, mode, steps, n_roll, dev, D, EV, MMPDERollout):
    import torch.distributed as dist

    rank, _, world = D.env_world()
    lo, hi = D.shard_range(total, rank, world)
    _, _, (model, model_b, itp, dmm, gc), u = _inputs(kind, total)
    for m in (model, model_b, itp, dmm):
        m.to(dev)
    for m in (model, model_b):
        m.edge_gemm = mode
    eng = MMPDERollout(kind, model, model_b, itp, dmm, gc, hi - lo, dev)
    u_loc = u[lo:hi].to(dev)
    res = EV.test_timestep_losses(eng, u_loc, total, steps=steps)
    fin = eng.rollout(u_loc[:, 0].contiguous(), 1, n_roll).cpu()
    if world > 1:                               # gather the final states (verification only)
        parts = [torch.zeros((-(-total // world),) + fin.shape[1:]) for _ in range(world)]
        buf = torch.zeros_like(parts[0])
        buf[:fin.shape[0]] = fin
        dist.all_gather(parts, buf)
        spans = [D.shard_range(total, r, world) for r in range(world)]
        fin = torch.cat([p[:b - a] for p, (a, b) in zip(parts, spans)])
    return res["per_trajectory"].cpu(), res["mean"].cpu(), fin


@pytest.mark.parametrize("total", [32, 16, 24])
@pytest.mark.parametrize("mode", ["f32", "f16x3"])
def test_sharded_eval_matches_single_process(dev, mode, total):
    from mmpde_amd import dist as D
    from mmpde_amd import evaluate as EV
    from mmpde_amd.rollout import MMPDERollout

    # shards of 16, 8 and 12 trajectories against one launch of all of them:
    # the edge kernel's summation units depend on the trajectory alone
    # (csrc/edge_wave.hip, edge_wave_plan)
    kind, world, steps, n_roll = "cy", 2, [1, 7, 20], 4
    single = _run_shard(kind, total, mode, steps, n_roll, dev, D, EV, MMPDERollout)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank_worker,
                      args=(r, world, port, kind, total, mode, steps, n_roll, q))
          for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    bad = []
    for rank, out, err in res:
        assert err is None, (rank, err)
        for name, a, b in zip(("per-trajectory losses", "mean loss", "final state"), out, single):
            a = torch.from_numpy(a)
            assert a.shape == b.shape, (name, a.shape, b.shape)
            rel = ((a - b).abs().max() / b.abs().max()).item()
            print(f"{mode} rank {rank} {name}: max rel diff {rel:.3e}")
            # both modes bit for bit: f16x3 takes its split scale per trajectory
            # (include/mmpde_hip.h mmpde_gnn_exec.seg_n), so a shard's outputs do
            # not depend on the trajectories of the other shard
            if not torch.equal(a, b):
                bad.append((rank, name, rel))
    assert not bad, bad


def _rccl_worker(port, q):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "mm-pde_amd")]
    os.environ.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    try:
        import torch.distributed as dist
        from mmpde_amd import dist as D

        rank, local, world = D.init(backend="nccl", force=True)
        dev = torch.device(f"cuda:{local}")
        assert dist.get_backend() == "nccl"
        losses = torch.arange(5, dtype=torch.float32, device=dev) * 0.25
        got = D.all_gather_losses(losses, 5)
        mx = D.max_over_ranks(1.5, dev)
        D.barrier(dev)
        torch.cuda.synchronize(dev)
        dist.destroy_process_group()
        q.put((got.cpu().numpy(), mx, None))
    except Exception as e:
        q.put((None, None, repr(e)))


def test_rccl_collectives_one_rank(dev):
    """dist.py over RCCL (torch backend "nccl"): init, the loss all-gather, the
    max-over-ranks all-reduce and the device barrier, as the bench and the
    sharded evaluation call them, in a one-rank group on this box's GPU."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    got, mx, err = q.get(timeout=180)
    p.join(timeout=60)
    assert err is None, err
    assert p.exitcode == 0
    assert got.tolist() == [0.0, 0.25, 0.5, 0.75, 1.0] and mx == 1.5
