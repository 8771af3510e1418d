"""Drop-in ``models.unet`` — unconditional U-Net (reference models/unet.py:101-170)."""
from __future__ import annotations

import torch

from dmx import _lib
from models._modules import build_unet_body
from models._native import NativeBacked


class Unet(NativeBacked):
    _dmx_kind = _lib.DMX_UNET

    def __init__(self, in_ch=3, time_dim=256, remove_deep_conv=False):
        super().__init__()
        self.time_dim = time_dim
        self.remove_deep_conv = remove_deep_conv
        self._dmx_in_ch = in_ch
        build_unet_body(self, in_ch, remove_deep_conv)

    def _dmx_check_supported(self) -> None:
        if self.time_dim != 256:
            raise RuntimeError(f"time_dim={self.time_dim}: the reference's emb_layer heads take 256 inputs "
                               f"(models/unet.py:63,83); only time_dim=256 has a forward pass")
        if not 1 <= self._dmx_in_ch <= 4:
            raise NotImplementedError(f"dmx implements in_ch in [1, 4] (got {self._dmx_in_ch})")

    def forward(self, x: torch.Tensor, t: torch.Tensor):
        eps, _ = self.native().forward(x, t)
        return eps
