"""Drop-in ``models.vae`` (reference models/vae.py:6-76).

``decode`` — the frozen decoder on the sampling path — runs natively in libdmx
(conv3x3 / 4-phase ConvTranspose implicit GEMMs, GroupNorm(8)+GELU fused into
the next layer's operand load, sigmoid + uint8 quantisation in the last kernel).

``encode`` is not on the denoising hot path (SURVEY.md §8f, rank 1 "next"): the
sampler only uses it on a zero dummy to infer the latent shape, which
``diff.Diffuser`` does analytically (replaying its RNG draw).  It is provided here
with plain torch ops so that the class stays API-complete; it is NOT a native path.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from dmx import _lib, spec
from models._native import NativeBacked, build_param_tree


def latent_hw(h: int, w: int):
    """Spatial size after the encoder's three 4x4/s2/p1 convs (models/vae.py:20,24,28)."""
    for _ in range(3):
        h = (h + 2 - 4) // 2 + 1
        w = (w + 2 - 4) // 2 + 1
    return h, w


class VAE(NativeBacked):
    _dmx_kind = _lib.DMX_VAE

    def __init__(self, in_channels=3, z_channels=4, base_channels=64, scale_factor=0.18215):
        super().__init__()
        if (in_channels, z_channels, base_channels) != (3, 4, 64) or scale_factor != 0.18215:
            raise ValueError("dmx implements the reference VAE configuration (3, 4, 64, 0.18215)")
        self.z_channels = z_channels
        self.scale_factor = scale_factor
        build_param_tree(self, spec.vae_spec(in_channels, z_channels, base_channels), seed=1)

    # ---- native ------------------------------------------------------------------------
    def decode(self, z: torch.Tensor) -> torch.Tensor:
        """z (B,4,h,w) -> images (B,3,8h,8w) in [0,1] (models/vae.py:64-69)."""
        img, _ = self.native().decode(z, want_img=True, want_u8=False)
        return img

    def decode_uint8(self, z: torch.Tensor) -> torch.Tensor:
        """decode + diff.py:58-62's x*255 -> clamp -> uint8, as (B, 8h, 8w, 3) HWC."""
        _, u8 = self.native().decode(z, want_img=False, want_u8=True)
        return u8

    # ---- off the hot path (torch ops) -------------------------------------------------------
    def encode(self, x: torch.Tensor):
        """models/vae.py:51-62 (consumes one randn_like draw like the reference)."""
        sd = dict(self.named_parameters())
        h = x
        for i, k in ((0, 3), (3, 4), (6, 3), (9, 4), (12, 3), (15, 4)):
            stride, pad = (1, 1) if k == 3 else (2, 1)
            h = F.conv2d(h, sd[f"enc.{i}.weight"], sd[f"enc.{i}.bias"], stride, pad)
            h = F.gelu(F.group_norm(h, 8, sd[f"enc.{i + 1}.weight"], sd[f"enc.{i + 1}.bias"], 1e-5))
        mu = F.conv2d(h, sd["to_mu.weight"], sd["to_mu.bias"])
        logvar = F.conv2d(h, sd["to_logvar.weight"], sd["to_logvar.bias"]).clamp(-30.0, 20.0)
        std = torch.exp(0.5 * logvar)
        z = (mu + torch.randn_like(std) * std) * self.scale_factor
        kl = 0.5 * torch.sum(torch.exp(logvar) + mu ** 2 - 1.0 - logvar, dim=(1, 2, 3)) / (x.size(2) * x.size(3))
        return z, kl.mean()

    def forward(self, x):
        raise NotImplementedError("VAE.forward is the training objective (models/vae.py:71-76) — out of dmx scope")
