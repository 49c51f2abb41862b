"""BaseCNN baseline on the HIP conv kernels (drop-in for reference models_cnn.py:8-83).

The reference's CNN baseline (``--model BaseCNN``, mmpde.py:183-184,249-252;
moving_mesh is forced off): eight circular-padded Conv2d layers with ELU and
residual connections on the time window stacked as channels, then
``u[:, -1] + cumsum(dt) * x``.  Module tree, ``state_dict`` keys and the xavier
initialisation order match the reference, so its checkpoints load and a
seeded construction gives the same weights.  The convolutions run on
``mmpde_conv2d_ex`` (circular indices, ELU and the post-activation residual
fused); the output combine is two small elementwise ops.  In train() mode
(the reference's ``training_loop_branch`` non-GNN branch,
train_helper_2d.py:107-125) every convolution is ops.Conv2dSame -- forward on
the same kernel, backward on HIP (input gradient as the convolution of dy with
the flipped kernel, weight / bias gradients by mmpde_conv2d_grad_weight) --
and ELU, the residuals and the output combine are autograd torch ops.
"""
from __future__ import annotations

import torch
from torch import nn

from . import _lib as L
from . import ops


class BaseCNN(nn.Module):
    """Reference models_cnn.py:8-83 (2-D, the variant mmpde.py builds)."""

    def __init__(self, pde, time_window: int = 25, hidden_channels: int = 40,
                 padding_mode: str = "circular"):
        super().__init__()
        self.pde = pde
        self.time_window = time_window
        self.hidden_channels = hidden_channels
        self.padding_mode = padding_mode
        tw, hc = time_window, hidden_channels
        spec = [(tw, hc, 3), (hc, hc, 5), (hc, hc, 5), (hc, hc, 5), (hc, hc, 7), (hc, hc, 7),
                (hc, hc, 7), (hc, tw, 9)]
        for i, (ci, co, ks) in enumerate(spec, 1):
            setattr(self, f"conv{i}", nn.Conv2d(ci, co, ks, padding=ks // 2, padding_mode=padding_mode,
                                                bias=True))
        for i in range(1, 9):
            nn.init.xavier_uniform_(getattr(self, f"conv{i}").weight)

    def __repr__(self):
        return "BaseCNN"

    def forward(self, u: torch.Tensor) -> torch.Tensor:
        """u [B, tw, X, Y] -> squeeze([B, 1, tw, X, Y]) (models_cnn.py:66-83)."""
        L.require_device(u)
        circ = self.padding_mode == "circular"
        if not circ and self.padding_mode != "zeros":
            raise NotImplementedError(f"padding_mode {self.padding_mode!r}")
        if self.training:
            return self._train_forward(u, circ)
        u = L.f32c(u)

        def conv(i, x, act, residual=None):
            c = getattr(self, f"conv{i}")
            ks = c.kernel_size[0]
            return ops.conv2d(x, c.weight, c.bias, 1, ks // 2, act, residual=residual, circular=circ,
                              res_after_act=residual is not None)

        x = conv(1, u, L.ACT_ELU)
        for i in range(2, 8):
            x = conv(i, x, L.ACT_ELU, residual=x)           # x + elu(conv_i(x))
        x = conv(8, x, L.ACT_NONE)
        tw = self.time_window
        dt = torch.cumsum(torch.full((1, tw), float(self.pde.dt), device=u.device), dim=1)[None, :, :, None, None]
        out = u[:, -1][:, None, None].repeat(1, 1, tw, 1, 1) + dt * x[:, None]
        return out.squeeze()

    def _train_forward(self, u: torch.Tensor, circ: bool) -> torch.Tensor:
        """models_cnn.py:66-83, differentiable (ops.Conv2dSame + torch ELU)."""
        import torch.nn.functional as F

        def conv(i, x):
            c = getattr(self, f"conv{i}")
            return ops.Conv2dSame.apply(x, c.weight, c.bias, circ)

        u = u.float()
        x = F.elu(conv(1, u))
        for i in range(2, 8):
            x = x + F.elu(conv(i, x))
        x = conv(8, x)
        tw = self.time_window
        dt = torch.cumsum(torch.ones(1, tw, device=u.device) * float(self.pde.dt), dim=1)[None, :, :, None, None]
        out = u[:, -1][:, None, None].repeat(1, 1, tw, 1, 1) + dt * x[:, None]
        return out.squeeze()
