"""Training loops of train_helper_2d.py on the HIP training path.

``training_itp`` (train_helper_2d.py:9-62) and ``training_loop_branch``
(:65-134) keep the reference signatures, their use of Python's ``random`` for
the unrolling / start-step draws (so a seeded run draws the same steps), and
their loss bookkeeping.  Forward and backward run through the train()-mode
modules: GNN edge stage on the EdgeMean HIP kernels, kNN searches on HIP,
ItpNet / res_cut / node MLPs as device torch ops under autograd (gnn_2d.py,
interpolate.py).  The DMM mesh model stays frozen in eval() as in the
reference (mmpde.py:201; it is not in the AdamW groups of mmpde.py:269-271),
so no gradient is propagated into it: the reference accumulates .grad on the
DMM parameters through the moved coordinates but never steps them.
"""
from __future__ import annotations

import random

import torch


def _draw_steps(graph_creator, unrolling, batch_size):
    """train_helper_2d.py:40-44 / :100-104."""
    unrolled_graphs = random.choice(unrolling)
    steps = [t for t in range(graph_creator.tw,
                              graph_creator.t_res - graph_creator.tw
                              - (graph_creator.tw * unrolled_graphs) + 1)]
    return random.choices(steps, k=batch_size)


def training_itp(itp_model, mesh_model, unrolling, batch_size, optimizer, optimizer2, loader,
                 graph_creator, criterion, device="cpu") -> torch.Tensor:
    """train_helper_2d.py:9-62: ItpNet trained to reproduce the data through the
    moved mesh and back (mode '1' in create_graph, mode '2' + res_cut in
    interpolate_pred).  Returns the per-batch losses / 2."""
    losses = []
    for (_u_base, u_super) in loader:
        optimizer.zero_grad()
        if optimizer2 is not None:
            optimizer2.zero_grad()
        random_steps = _draw_steps(graph_creator, unrolling, batch_size)
        data, labels = graph_creator.create_data(u_super, random_steps)
        graph = graph_creator.create_graph(itp_model, data, labels, random_steps, device,
                                           mesh_model)
        u_uni = graph_creator.interpolate_pred(itp_model, graph.x, graph, data, device)
        data = data.to(device)
        loss = criterion(u_uni, data.reshape(-1, 1))
        loss.backward()
        losses.append(loss.detach() / 2)
        optimizer.step()
        if optimizer2 is not None:
            optimizer2.step()
    return torch.stack(losses)


def training_loop_branch(model, model_b, itp_model, mesh_model, unrolling, batch_size, optimizer,
                         optimizer2, loader, graph_creator, criterion,
                         device="cpu") -> torch.Tensor:
    """train_helper_2d.py:65-134: GNN branch pred = interpolate_pred(itp,
    model_b(graph), graph, data) + model(graph_uni), MSE against the labels;
    CNN branch (BaseCNN) pred = model(data), MSE against labels.squeeze();
    backward, AdamW step."""
    losses = []
    for idx, (_u_base, u_super) in enumerate(loader):
        optimizer.zero_grad()
        if optimizer2 is not None:
            optimizer2.zero_grad()
        random_steps = _draw_steps(graph_creator, unrolling, batch_size)
        data, labels = graph_creator.create_data(u_super, random_steps)
        if f"{model}" != "GNN":
            # the CNN baseline (train_helper_2d.py:116-117,124-125)
            data, labels = data.to(device), labels.to(device)
            pred = model(data)
            loss = criterion(pred, labels.squeeze())
            loss.backward()
            losses.append(loss.detach())
            optimizer.step()
            if optimizer2 is not None and idx % 1 == 0:
                optimizer2.step()
            continue
        graph_uni = graph_creator.create_graph(itp_model, data, labels, random_steps, device, None)
        if mesh_model is not None:
            graph = graph_creator.create_graph(itp_model, data, labels, random_steps, device,
                                               mesh_model)
            pred = graph_creator.interpolate_pred(itp_model, model_b(graph), graph, data,
                                                  device) + model(graph_uni)
        else:
            pred = model(graph_uni)
        labels = labels.to(device)
        loss = criterion(pred, labels.reshape(-1, 1))
        loss.backward()
        losses.append(loss.detach())
        optimizer.step()
        if optimizer2 is not None and idx % 1 == 0:
            optimizer2.step()
    return torch.stack(losses)
