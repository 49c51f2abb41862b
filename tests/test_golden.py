"""The oracle reproduces its committed golden vectors (tests/golden/make_golden.py)."""
import os

import numpy as np
import torch

from conftest import GOLDEN
from oracle import refcpu


def test_gnn_small_regression():
    from mmpde_amd.synth import build_models

    g = np.load(os.path.join(GOLDEN, "gnn_small.npz"))
    torch.manual_seed(3)
    pde, model, _, _, _, _ = build_models("cy", grid=torch.rand(64, 2), moving_mesh=False)
    sd = {k: v.detach() for k, v in model.state_dict().items()}
    ei, _, _ = refcpu.knn_graph(torch.from_numpy(g["pos"][:, 1:3]), 35, 2)
    assert np.array_equal(ei.numpy(), g["edge_index"])
    out = refcpu.mp_pde_solver(sd, refcpu.PDEConst("cy", [30, 64], ori_grid=pde.ori_grid),
                               torch.from_numpy(g["u"]), torch.from_numpy(g["pos"]), ei)
    assert np.array_equal(out.numpy(), g["out"])
