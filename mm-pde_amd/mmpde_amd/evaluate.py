"""Teacher-forced evaluation on the engine, sharded over ranks (SURVEY.md §8(d)
"a teacher-forced mode that mirrors test_timestep_losses", §8(e)).

Reference harness: train_helper_2d.py:137-200 (``test_timestep_losses``).  For
every step s in range(tw, t_res - tw + 1) (mmpde.py:139; the ``step % tw``
filter of train_helper_2d.py:167-168 passes every step at tw = 1) and every
test batch, the one-step
forward runs on the TRUE state u[s - tw:s] (teacher forcing, not the rollout's
own prediction), and the loss is MSELoss(pred, labels) (mmpde.py:33-36,
:184-185); it prints and returns the mean over batches, then over steps.

Here each rank owns a contiguous block of trajectories (dist.shard_range) and
runs the one-step forward on its block through ``MMPDERollout.step``; the loss
is kept per trajectory on the device, and the only collective is one
all-gather of those B_local floats per step (dist.all_gather_losses).  Equal
trajectory sizes make the mean of per-trajectory MSEs equal to the batch MSE
of the reference, so the returned means are the reference's numbers for a
test set of B_total trajectories evaluated as one batch.
"""
from __future__ import annotations

import torch

from . import dist as D


def timestep_steps(tw: int, t_res: int):
    """mmpde.py:139 + train_helper_2d.py:167-168: the evaluated step indices."""
    return [s for s in range(tw, t_res - tw + 1) if s == tw or s % tw == 0]


@torch.no_grad()
def test_timestep_losses(engine, u_local: torch.Tensor, total: int, steps=None,
                         gather: bool = True):
    """u_local: this rank's trajectories [B_local, T, N] (cylinder) or
    [B_local, T, s, s] (Burgers) on the engine's device, B_local = engine.B.
    Returns dict with
      per_trajectory [n_steps, total] (all ranks, trajectory order; this rank's
                     block only when gather=False),
      per_step       [n_steps]  mean over trajectories (the reference's
                     ``torch.mean(losses)`` per step),
      mean           scalar     mean over steps (its return value),
      steps          the step indices."""
    tw = engine.gc.tw
    if tw != 1:
        raise NotImplementedError("engine step is time_window 1")
    if u_local.shape[0] != engine.B:
        raise ValueError(f"u_local holds {u_local.shape[0]} trajectories, engine.B = {engine.B}")
    if steps is None:
        steps = timestep_steps(tw, engine.gc.t_res)
    B = engine.B
    rows = []
    for s in steps:
        data = u_local[:, s - tw]                       # [B, N] / [B, s, s]: create_data input
        labels = u_local[:, s:s + tw]
        pred = engine.step(data.contiguous(), s)
        local = D.per_trajectory_mse(pred, labels, B)
        rows.append(D.all_gather_losses(local, total) if gather else local)
    per_traj = torch.stack(rows)
    per_step = per_traj.mean(dim=1)
    return {"per_trajectory": per_traj, "per_step": per_step, "mean": per_step.mean(),
            "steps": list(steps)}
