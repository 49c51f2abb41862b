"""Reference checkpoint / dataset readers (mmpde_amd.formats).

The reference's own files (cy_checkpoint, burgers_checkpoint, cylinder_rot_tri,
burgers_192.npy) are not in the tree, so each test writes a file in exactly the
layout the reference writes (mesh/dmm_utils.py:772-782, mmpde.py:293-310) or
reads (mmpde.py:163-171) and checks what the reader returns.  CPU only.
"""
import argparse
import pickle

import numpy as np
import pytest
import torch

from mmpde_amd import formats
from mmpde_amd.synth import build_models


def _equal_sd(a, b):
    sa, sb = a.state_dict(), b.state_dict()
    assert sa.keys() == sb.keys()
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k


def _dmm_args(kind):
    # mesh/dmm.py:18-59 parses these into lists of ints (branch_layers: an int for
    # the burgers ConvNet depth, the list [4, 3] for the cy GNN branch)
    if kind == "cy":
        return argparse.Namespace(experiment="cy", branch_layers=[4, 3], trunk_layers=[16, 512],
                                  out_layers=[1024, 512, 1], lr_adam=2e-4, rf=True)
    return argparse.Namespace(experiment="burgers", branch_layers=7, trunk_layers=[32, 512],
                              out_layers=[1024, 512, 1], lr_adam=2e-4, rf=True)


def _evaluate_stat(seed):
    """What mesh/dmm_utils.py:1228-1232 (evaluate_tri) / :1280-1284 (evaluate)
    return: np.mean over a list of 0-d float32 arrays (torch -> .numpy()), an
    np.float32 scalar."""
    g = torch.Generator().manual_seed(seed)
    per_traj = [torch.std(torch.rand(50, generator=g)).cpu().detach().numpy() for _ in range(4)]
    return np.mean(per_traj)


def _dmm_checkpoint_dict(dmm, kind):
    """The dict mesh/dmm_utils.py:772-782 saves: loss lists of .item() floats
    (:555-557), the argparse args, and per-epoch lists of np.mean scalars
    (:734-737)."""
    return {"model_state_dict": dmm.state_dict(), "loss_in": [0.5, 0.25],
            "loss_bound": [1.0, 0.5], "loss_convex": [0.0, 0.0], "args": _dmm_args(kind),
            "train_std": [_evaluate_stat(1), _evaluate_stat(2)],
            "train_minmax": [_evaluate_stat(3)], "test_std": [_evaluate_stat(4)],
            "test_minmax": [np.float64(_evaluate_stat(5))]}


@pytest.mark.parametrize("kind", ["cy", "burgers"])
def test_dmm_checkpoint_round_trip(tmp_path, kind):
    pde, _, _, _, dmm, _ = build_models(kind, seed=3)
    path = tmp_path / f"{kind}_checkpoint"
    ck = _dmm_checkpoint_dict(dmm, kind)
    assert isinstance(ck["train_std"][0], np.float32)
    torch.save(ck, path)
    back = formats.load_reference_file(path)
    for key in ("train_std", "train_minmax", "test_std", "test_minmax"):
        assert [type(v) for v in back[key]] == [type(v) for v in ck[key]]
        assert back[key] == ck[key]
    if kind == "cy":
        got = formats.load_dmm_checkpoint(path, "cy", grid=pde.ori_grid)
    else:
        got = formats.load_dmm_checkpoint(path, "burgers", s=48)
    assert not got.training
    assert got.mode == dmm.mode
    _equal_sd(got, dmm)


def test_mmpde_checkpoint_round_trip(tmp_path):
    _, model, model_b, itp, dmm, _ = build_models("cy", seed=5)
    args = argparse.Namespace(experiment="cy", model="GNN", moving_mesh=True, neighbors=35,
                              base_resolution=[30, 2521], time_window=1)
    path = tmp_path / "GNN_cy.pt"
    torch.save({"model_state_dict": model.state_dict(), "model_b_state_dict": model_b.state_dict(),
                "mesh_model_state_dict": dmm.state_dict(), "itp_model_state_dict": itp.state_dict(),
                "args": args, "train_losses": [torch.ones(3)], "itp_losses": [torch.zeros(3)],
                "test_timestep_losses": [torch.tensor(0.5)]}, path)
    ck = formats.load_reference_file(path)
    assert ck["args"].neighbors == 35
    _, m2, mb2, it2, d2, _ = build_models("cy", seed=9)
    formats.apply_mmpde_checkpoint(ck, m2, mb2, d2, it2)
    for a, b in ((m2, model), (mb2, model_b), (it2, itp), (d2, dmm)):
        assert not a.training
        _equal_sd(a, b)
    with pytest.raises(KeyError):               # GNN-only checkpoint given a mesh model
        formats.apply_mmpde_checkpoint({"model_state_dict": model.state_dict()}, m2, mb2)


class _NotAllowed:
    def __reduce__(self):
        return (print, ("this must never run",))


def test_loader_refuses_code_in_files(tmp_path):
    path = tmp_path / "evil"
    torch.save({"model_state_dict": {}, "args": _NotAllowed()}, path)
    with pytest.raises(pickle.UnpicklingError):
        formats.load_reference_file(path)


def test_loader_refuses_object_arrays(tmp_path):
    """The numpy allowlist is data only: an object-dtype array (whose elements
    would be arbitrary pickled objects) is still refused."""
    path = tmp_path / "objarr"
    torch.save({"train_std": np.array([1, "x"], dtype=object)}, path)
    with pytest.raises(pickle.UnpicklingError):
        formats.load_reference_file(path)


def _rename_pickled_module(path, old: bytes, new: bytes):
    """Rewrite the GLOBAL opcodes of a torch.save zip's data.pkl (protocol 2: text
    'module\\nname\\n') -- here to produce the numpy 1.x module path
    ('numpy.core.multiarray') that checkpoints written by the reference's
    environment (env.yml pins numpy 1.x) carry."""
    import zipfile

    with zipfile.ZipFile(path) as z:
        items = [(i, z.read(i.filename)) for i in z.infolist()]
    with zipfile.ZipFile(path, "w", zipfile.ZIP_STORED) as z:
        for info, data in items:
            if info.filename.endswith("data.pkl"):
                assert old in data
                data = data.replace(old, new)
            z.writestr(info, data)


def test_numpy1_module_paths(tmp_path):
    path = tmp_path / "cy_checkpoint_np1"
    torch.save({"args": _dmm_args("cy"), "train_std": [_evaluate_stat(7)],
                "test_minmax": [np.float64(0.25)]}, path)
    _rename_pickled_module(path, b"numpy._core.multiarray\n", b"numpy.core.multiarray\n")
    back = formats.load_reference_file(path)
    assert back["train_std"] == [_evaluate_stat(7)]
    assert isinstance(back["train_std"][0], np.float32)
    assert back["test_minmax"] == [0.25]


def test_cylinder_data(tmp_path):
    g = torch.Generator().manual_seed(0)
    data = torch.rand(5, 40, 50, 5, generator=g)
    path = tmp_path / "cylinder_rot_tri"
    torch.save(data, path)
    grid, u_tr, u_te = formats.load_cylinder_data(path, n_train=3)
    assert torch.equal(grid, data[0, 0, :, :2] * 2)
    assert torch.equal(u_tr, data[:3, 10:, :, 2])
    assert torch.equal(u_te, data[3:, 10:, :, 2])
    assert u_tr.shape == (3, 30, 50)


def test_burgers_data(tmp_path):
    arr = np.random.default_rng(1).standard_normal((3, 31, 192, 192)).astype(np.float64)
    path = tmp_path / "burgers_192.npy"
    np.save(path, arr)
    u_tr, u_te = formats.load_burgers_data(path, (31, 48, 48), n_train=2)
    ref = torch.tensor(arr, dtype=torch.float)[:, :, ::4, ::4]
    assert u_tr.dtype == torch.float32 and u_tr.shape == (2, 31, 48, 48)
    assert torch.equal(u_tr, ref[:2]) and torch.equal(u_te, ref[2:])
