"""Drop-in ``models.unet_cond_geom`` (reference models/unet_cond_geom.py:26-100)."""
from __future__ import annotations

import torch

from dmx import _lib
from models._modules import GeomHead
from models.unet_cond import UnetCond


class UnetCondWithGeomHead(UnetCond):
    """UnetCond + GeomHead; forward returns (eps_pred, geom_pred) like the reference."""

    _dmx_kind = _lib.DMX_UNET_COND_GEOM

    def __init__(self, in_ch=4, time_dim=256, num_classes=3, cfg_drop_prob=0.0, remove_deep_conv=False,
                 geom_dim=12, geom_hidden=256):
        super().__init__(in_ch=in_ch, time_dim=time_dim, num_classes=num_classes, cfg_drop_prob=cfg_drop_prob,
                         remove_deep_conv=remove_deep_conv)
        self.geom_head = GeomHead(in_ch=64, out_dim=geom_dim, hidden=geom_hidden)
        self._geom_dim, self._geom_hidden = geom_dim, geom_hidden

    def _dmx_config(self) -> dict:
        return {"num_classes": self.num_classes, "geom_dim": self._geom_dim, "geom_hidden": self._geom_hidden}

    def forward(self, x: torch.Tensor, t: torch.Tensor, y: torch.Tensor, cond_vals: torch.Tensor = None,
                cond_mask: torch.Tensor = None, cond_drop_prob: float = 0.0):
        use = cond_vals is not None and cond_mask is not None  # unet_cond_geom.py:91 (no dropout here)
        return self._run(x, t, y, cond_vals if use else None, cond_mask if use else None, want_geom=True)
