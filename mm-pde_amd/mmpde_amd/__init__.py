"""mmpde_amd -- MI355X-native MM-PDE forward engine.

Drop-in host mirror of the reference model API (Peiyannn/MM-PDE: gnn_2d.py,
mesh/dmm_model.py, interpolate.py, data_creator_2d.py, PDEs.py) whose compute
runs on hand-written gfx950 HIP kernels in lib/libmmpde_hip.so (C-ABI:
include/mmpde_hip.h).  Importing the package does not touch the GPU; the
library is loaded on first use and every op raises if it is missing.
"""
from .data_creator_2d import GraphCreator_FS_2D
from .dmm_model import DMM, ConvNet, DenseNet
from .gnn_2d import GNN_Layer_FS_2D, MP_PDE_Solver_2D
from .graph import Data
from .interpolate import ItpNet
from .models_cnn import BaseCNN
from .pdes import PDE, burgers, cy
from .rollout import MMPDERollout

__all__ = ["BaseCNN", "GraphCreator_FS_2D", "DMM", "ConvNet", "DenseNet", "GNN_Layer_FS_2D",
           "MP_PDE_Solver_2D", "Data", "ItpNet", "PDE", "burgers", "cy", "MMPDERollout"]
