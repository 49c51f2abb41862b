"""Reference checkpoint and dataset formats.

* DMM checkpoints written by mesh/dmm_utils.py:772-782 (``cy_checkpoint``,
  ``burgers_checkpoint``): ``{'model_state_dict', 'args', <loss lists>}`` with
  ``args`` the argparse.Namespace of mesh/dmm.py:18-59 (``branch_layers``,
  ``trunk_layers``, ``out_layers`` size the DMM); consumed at mmpde.py:189-201.
* MM-PDE checkpoints written by mmpde.py:293-310: ``{'model_state_dict',
  'model_b_state_dict', 'mesh_model_state_dict', 'itp_model_state_dict', 'args',
  'train_losses', 'itp_losses', 'test_timestep_losses'}`` (the model_b / mesh /
  itp entries only with moving_mesh).
* Datasets: ``mesh/data/cylinder_rot_tri`` (a saved tensor [traj, 40, 2521, 5],
  channels x, y, u, ...; mmpde.py:163-166, mesh/dmm.py:76-81) and
  ``mesh/data/burgers_192.npy`` ([traj, T, 192, 192]; mmpde.py:171).

Every file is read by loaders that execute nothing from it:
``torch.load(weights_only=True)`` with a data-only allowlist, and
``numpy.load(allow_pickle=False)``.  The allowlist is ``argparse.Namespace``
(the ``args`` entry) plus the numpy reconstructors a numpy value pickles to:
the DMM checkpoint's ``train_std`` / ``train_minmax`` / ``test_*`` lists hold
``np.mean(...)`` scalars (mesh/dmm_utils.py:734-737 append the values that
``evaluate`` / ``evaluate_tri`` return, :1232,1284), which pickle as
``numpy.core.multiarray.scalar`` (numpy 1.x files; ``numpy._core`` under numpy
2) + ``numpy.dtype`` + the dtype's class.  Those rebuild a number from its
bytes and call nothing else; object / void / string dtypes are not on the list.
A file that needs any other global is refused (``pickle.UnpicklingError``).
"""
from __future__ import annotations

import argparse

import numpy as np
import torch

from .dmm_model import DMM


def _numpy_data_globals():
    """(callable, pickled name) pairs for numpy scalars / arrays / numeric dtypes,
    under both the numpy 1.x (``numpy.core``) and numpy 2.x (``numpy._core``)
    module paths the reference's checkpoints may name."""
    try:
        from numpy._core import multiarray as ma
    except ImportError:  # numpy 1.x
        from numpy.core import multiarray as ma
    out = [np.dtype, np.ndarray]
    for mod in ("numpy.core.multiarray", "numpy._core.multiarray"):
        out.append((ma.scalar, f"{mod}.scalar"))
        out.append((ma._reconstruct, f"{mod}._reconstruct"))
    numeric = ("Bool", "Int8", "Int16", "Int32", "Int64", "UInt8", "UInt16", "UInt32", "UInt64",
               "Float16", "Float32", "Float64", "LongDouble", "Complex64", "Complex128",
               "LongLong", "ULongLong", "Byte", "UByte", "Short", "UShort", "Int", "UInt",
               "Long", "ULong")
    dts = getattr(np, "dtypes", None)
    if dts is not None:
        seen = set()
        for name in numeric:
            cls = getattr(dts, name + "DType", None)
            if cls is not None and cls not in seen:
                seen.add(cls)
                out.append(cls)
    return out


def load_reference_file(path, map_location="cpu"):
    """torch.load of a reference checkpoint / dataset file without executing code."""
    with torch.serialization.safe_globals([argparse.Namespace] + _numpy_data_globals()):
        return torch.load(path, map_location=map_location, weights_only=True)


def dmm_from_checkpoint(ck, experiment: str, grid: torch.Tensor | None = None,
                        s: int | None = None) -> DMM:
    """mmpde.py:189-201: the DMM the checkpoint's args describe, with its weights,
    in eval mode.  cy: graph mode on ``grid`` ([N, 2], the scaled ori_grid);
    burgers: array mode at resolution ``s``."""
    a = ck["args"]
    trunk = [2] + list(a.trunk_layers)
    if experiment == "cy":
        if grid is None:
            raise ValueError("graph-mode DMM needs the grid (data[0, 0, :, :2] scaled by 2)")
        m = DMM(mode="graph", grid=grid, branch_layer=a.branch_layers, trunk_layer=trunk,
                out_layer=a.out_layers)
    elif experiment == "burgers":
        if s is None:
            raise ValueError("array-mode DMM needs the resolution s")
        m = DMM(s=s, mode="array", branch_layer=a.branch_layers, trunk_layer=trunk,
                out_layer=a.out_layers)
    else:
        raise ValueError(f"experiment {experiment!r}: cy | burgers")
    m.load_state_dict(ck["model_state_dict"])
    return m.eval()


def load_dmm_checkpoint(path, experiment: str, grid: torch.Tensor | None = None,
                        s: int | None = None) -> DMM:
    """``cy_checkpoint`` / ``burgers_checkpoint`` -> eval-mode DMM (mmpde.py:189-201)."""
    return dmm_from_checkpoint(load_reference_file(path), experiment, grid=grid, s=s)


_MMPDE_KEYS = (("model", "model_state_dict"), ("model_b", "model_b_state_dict"),
               ("mesh_model", "mesh_model_state_dict"), ("itp_model", "itp_model_state_dict"))


def apply_mmpde_checkpoint(ck, model, model_b=None, mesh_model=None, itp_model=None):
    """Load an mmpde.py:293-310 checkpoint dict into the given modules (state-dict
    keys are the reference's) and put them in eval mode.  A module passed without
    its entry in the checkpoint, or an entry without its module, raises."""
    mods = {"model": model, "model_b": model_b, "mesh_model": mesh_model, "itp_model": itp_model}
    for name, key in _MMPDE_KEYS:
        m = mods[name]
        if (m is None) != (key not in ck):
            raise KeyError(f"{name}: module {'missing' if m is None else 'given'} but checkpoint "
                           f"{'has' if key in ck else 'lacks'} {key!r}")
        if m is not None:
            m.load_state_dict(ck[key])
            m.eval()
    return model, model_b, mesh_model, itp_model


def load_cylinder_data(path, n_train: int = 80):
    """``cylinder_rot_tri`` -> (ori_grid [N, 2], u_train, u_test), as mmpde.py:163-168:
    coordinates scaled by 2 (a unit square), u = channel 2 from time index 10 on."""
    data = load_reference_file(path)
    if not isinstance(data, torch.Tensor) or data.dim() != 4 or data.shape[-1] < 3:
        raise ValueError("cylinder_rot_tri: expected a tensor [traj, T, N, >=3]")
    data = data.clone()
    data[:, :, :, :2] *= 2
    u = data[:, 10:, :, 2]
    return data[0, 0, :, :2].contiguous(), u[:n_train], u[n_train:]


def load_burgers_data(path, base_resolution=(31, 48, 48), n_train: int = 80):
    """``burgers_192.npy`` -> (u_train, u_test), mmpde.py:171-173: fp32, spatially
    subsampled to base_resolution[1:] by strided slicing."""
    arr = np.load(path, allow_pickle=False)
    if arr.ndim != 4:
        raise ValueError("burgers_192.npy: expected [traj, T, 192, 192]")
    u = torch.tensor(arr, dtype=torch.float)
    u = u[:, :, ::int(arr.shape[2] / base_resolution[1]), ::int(arr.shape[3] / base_resolution[2])]
    return u[:n_train], u[n_train:]
