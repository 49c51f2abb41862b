"""Trajectory sharding across GPUs.

The reference is single-device.  Its kNN graphs are built per trajectory (the
``batch`` vector, data_creator_2d.py:250-260) and BatchNorm runs on running
statistics in eval, so trajectories are fully independent: each rank owns a
contiguous block of trajectories and runs the whole step on it with no
data-path collective.  The only exchange is an all-gather of per-trajectory
losses (teacher-forced evaluation) -- one RCCL call of B_local floats.

One process per GPU; rendezvous from the torchrun environment (RANK,
LOCAL_RANK, WORLD_SIZE, MASTER_ADDR/PORT).  Backend "nccl" is RCCL on ROCm.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def env_world():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def init(backend: str | None = None, force: bool = False):
    """Initialise the process group when launched under torchrun (or, with
    force, for a one-rank world too); returns (rank, local_rank, world).
    backend: "nccl" (RCCL, the default with a GPU) or "gloo" (CPU collectives:
    the CPU tests, and several ranks sharing one GPU, which RCCL refuses)."""
    rank, local, world = env_world()
    if (world > 1 or force) and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return rank, local, world


def local_device(local: int) -> torch.device:
    """The GPU of local rank `local`: one per rank on a full node; ranks beyond
    the visible devices share them round-robin (gloo only: RCCL needs one GPU
    per rank)."""
    return torch.device(f"cuda:{local % max(torch.cuda.device_count(), 1)}")


def _cpu_collectives() -> bool:
    """gloo group: collectives on host tensors."""
    return dist.get_backend() == "gloo"


def shard_range(total: int, rank: int, world: int):
    """Contiguous block [lo, hi) of `total` trajectories owned by `rank`
    (sizes differ by at most one)."""
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def per_trajectory_mse(pred: torch.Tensor, labels: torch.Tensor, batches: int) -> torch.Tensor:
    """MSE of each trajectory (mmpde.py:33-36 applied per trajectory).  Device
    tensors go through mmpde_traj_mse (fixed summation order per trajectory, so
    the value does not depend on how trajectories are sharded); host tensors
    (the gloo tests) use torch."""
    if pred.is_cuda:
        from . import _lib as L

        p = L.f32c(pred).reshape(-1)
        q = L.f32c(labels.to(pred.device)).reshape(-1)
        if p.numel() != q.numel() or p.numel() % batches:
            raise ValueError("pred / labels must hold `batches` equal trajectories")
        out = torch.empty((batches,), dtype=torch.float32, device=pred.device)
        L.check(L.lib().mmpde_traj_mse(L.ptr(p), L.ptr(q), batches, p.numel() // batches,
                                       L.ptr(out), L.stream(pred.device)), "mmpde_traj_mse")
        return out
    d = (pred.reshape(batches, -1) - labels.reshape(batches, -1)).float()
    return (d * d).mean(dim=1)


def _group():
    return dist.is_available() and dist.is_initialized()


def all_gather_losses(local: torch.Tensor, total: int) -> torch.Tensor:
    """Gather per-trajectory losses of every rank in trajectory order (the one
    collective of the sharded step; runs whenever a process group exists)."""
    if not _group():
        return local
    world = dist.get_world_size()
    sizes = [shard_range(total, r, world) for r in range(world)]
    width = max(hi - lo for lo, hi in sizes)
    buf = torch.zeros(width, dtype=local.dtype, device=local.device)
    buf[:local.numel()] = local
    out = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(out, buf)
    return torch.cat([o[:hi - lo] for o, (lo, hi) in zip(out, sizes)])


def max_over_ranks(value: float, device=None) -> float:
    if not _group():
        return value
    t = torch.tensor([value], dtype=torch.float64, device=None if _cpu_collectives() else device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier(device=None):
    if _group():
        if device is not None and device.type == "cuda" and not _cpu_collectives():
            dist.barrier(device_ids=[device.index])
        else:
            dist.barrier()
