"""Drop-in ``models.unet_cond`` (reference models/unet_cond.py:102-216).

``UnetCond`` keeps the reference constructor, attributes, module tree, default
initialisation (drawn from the global torch generator in the reference's order) and
state_dict keys; its forward runs the native U-Net of libdmx (conv3x3+GroupNorm+GELU
residual blocks, 4-head self-attention at six resolutions, sinusoidal time + class +
geometric-condition embedding) and returns eps like the reference.
"""
from __future__ import annotations

import torch

from dmx import _lib
from models._modules import AttenionBlock, Down, ResBlock, Up, build_cond_embedding, build_unet_body  # noqa: F401
from models._native import NativeBacked


class UnetCond(NativeBacked):
    """Conditional latent U-Net (reference models/unet_cond.py:102-153)."""

    _dmx_kind = _lib.DMX_UNET_COND

    def __init__(self, in_ch=4, time_dim=256, num_classes=3, cfg_drop_prob=0.1, remove_deep_conv=False):
        super().__init__()
        self.time_dim = time_dim
        self.remove_deep_conv = remove_deep_conv
        self.num_classes = num_classes
        self.cfg_drop_prob = cfg_drop_prob
        self._dmx_in_ch = in_ch
        build_cond_embedding(self, num_classes, time_dim)
        build_unet_body(self, in_ch, remove_deep_conv)

    def _dmx_config(self) -> dict:
        return {"num_classes": self.num_classes}

    def _dmx_check_supported(self) -> None:
        if self.time_dim != 256:
            # the reference's Down/Up emb heads are Linear(256, .) whatever time_dim is
            # (models/unet_cond.py:55,73), so its forward fails for any other width as well
            raise RuntimeError(f"time_dim={self.time_dim}: the reference's emb_layer heads take 256 inputs "
                               f"(models/unet_cond.py:64,84); only time_dim=256 has a forward pass")
        if not 1 <= self._dmx_in_ch <= 4:
            raise NotImplementedError(f"dmx implements in_ch in [1, 4] (got {self._dmx_in_ch})")

    def _cfg_dropout(self, y, cond_vals, cond_mask, cond_drop_prob):
        """models/unet_cond.py:199-211: training-mode label / condition dropout, drawn from the
        global generator in the reference's order (plain torch on the (B,) labels and (B, 12) rows)."""
        if self.training and self.cfg_drop_prob > 0:
            drop = torch.rand_like(y.float()) < self.cfg_drop_prob
            y = torch.where(drop, torch.zeros_like(y), y)
        if cond_vals is not None and cond_mask is not None:
            p = self.cfg_drop_prob if cond_drop_prob is None else cond_drop_prob
            if self.training and p > 0.0:
                keep = (torch.rand(cond_vals.size(0), device=cond_vals.device) > p).float().unsqueeze(1)
                cond_vals = cond_vals * keep
                cond_mask = cond_mask * keep
        return y, cond_vals, cond_mask

    def _run(self, x, t, y, vals, mask, want_geom=False):
        if self._dmx_training():
            return self._dmx_train_forward(x, t, y, vals, mask)
        return self.native().forward(x, t, y, vals, mask, want_geom=want_geom)

    def forward(self, x: torch.Tensor, t: torch.Tensor, y: torch.Tensor, cond_vals: torch.Tensor = None,
                cond_mask: torch.Tensor = None, cond_drop_prob: float = None):
        y, cond_vals, cond_mask = self._cfg_dropout(y, cond_vals, cond_mask, cond_drop_prob)
        use = cond_vals is not None and cond_mask is not None  # models/unet_cond.py:205
        eps, _ = self._run(x, t, y, cond_vals if use else None, cond_mask if use else None)
        return eps
