"""Drop-in ``models.unet`` — unconditional U-Net (reference models/unet.py:101-170)."""
from __future__ import annotations

import torch

from dmx import _lib, spec
from models._native import NativeBacked, build_param_tree


class Unet(NativeBacked):
    _dmx_kind = _lib.DMX_UNET

    def __init__(self, in_ch=3, time_dim=256, remove_deep_conv=False):
        super().__init__()
        if time_dim != 256:
            raise ValueError("dmx implements time_dim=256")
        if in_ch > 4:
            raise ValueError("dmx implements in_ch <= 4")
        self.time_dim = time_dim
        self.remove_deep_conv = remove_deep_conv
        self._dmx_in_ch = in_ch
        build_param_tree(self, spec.unet_spec(in_ch=in_ch, remove_deep_conv=remove_deep_conv))

    def forward(self, x: torch.Tensor, t: torch.Tensor):
        eps, _ = self.native().forward(x, t)
        return eps
