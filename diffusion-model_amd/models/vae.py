"""Drop-in ``models.vae`` (reference models/vae.py:6-76).

``decode`` — the frozen decoder on the sampling path — runs natively in libdmx
(conv3x3 / 4-phase ConvTranspose implicit GEMMs, GroupNorm(8)+GELU fused into
the next layer's operand load, sigmoid + uint8 quantisation in the last kernel).

``encode`` (SURVEY.md §8f, rank 1 "next") runs natively too (dmx_vae_encode:
conv3x3 / conv4x4-stride-2 implicit GEMMs, GroupNorm(8)+GELU, then mu / logvar heads,
reparameterisation and the KL term in one tail kernel).  The sampler itself only needs
the latent shape of a zero dummy, which ``diff.Diffuser`` derives analytically while
replaying the encoder's RNG draw.
"""
from __future__ import annotations

import torch

from dmx import _lib
from models._modules import build_vae
from models._native import NativeBacked


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
        self.z_channels = z_channels
        self.scale_factor = scale_factor
        self._dmx_shape = (in_channels, z_channels, base_channels)
        build_vae(self, in_channels, z_channels, base_channels)

    def _dmx_config(self) -> dict:
        return {"scale_factor": float(self.scale_factor)}

    def _dmx_check_supported(self) -> None:
        if self._dmx_shape != (3, 4, 64):
            raise NotImplementedError("dmx implements the reference VAE widths in_channels=3, z_channels=4, "
                                      f"base_channels=64 (got {self._dmx_shape}); scale_factor is free")

    # ---- native ------------------------------------------------------------------------
    def decode(self, z: torch.Tensor) -> torch.Tensor:
        """z (B,4,h,w) -> images (B,3,8h,8w) in [0,1] (models/vae.py:64-69)."""
        img, _ = self.native().decode(z, want_img=True, want_u8=False)
        return img

    def decode_uint8(self, z: torch.Tensor) -> torch.Tensor:
        """decode + diff.py:58-62's x*255 -> clamp -> uint8, as (B, 8h, 8w, 3) HWC."""
        _, u8 = self.native().decode(z, want_img=False, want_u8=True)
        return u8

    def encode(self, x: torch.Tensor):
        """models/vae.py:51-62 -> (z, kl.mean()), natively (dmx_vae_encode: conv3x3 / conv4x4-s2
        implicit GEMMs + GN(8)+GELU, then the mu / logvar heads, reparameterisation and KL in one
        tail kernel).  The randn_like(std) draw is made here with torch on x's device, so the
        global RNG stream advances exactly as in the reference.  Image sides must be multiples
        of 8 (the three stride-2 convs halve them exactly)."""
        n, _, h, w = x.shape
        hl, wl = latent_hw(h, w)
        eps = torch.randn((n, self.z_channels, hl, wl), device=x.device, dtype=torch.float32)
        z, kl = self.native().encode(x, eps)
        return z, kl.mean()

    def forward(self, x):
        """models/vae.py:71-76, forward only: native encode (same randn_like draw) -> native
        decode -> recon MSE + 1e-6 * KL, all on x's device.  Returns (x_recon, z, loss,
        {'recon_mse', 'kl'}).  No autograd graph: VAE training stays out of dmx scope."""
        z, kl = self.encode(x)
        x_recon = self.decode(z)
        recon = torch.nn.functional.mse_loss(x_recon, x.float(), reduction="mean")
        return x_recon, z, recon + 1e-6 * kl, {"recon_mse": recon.detach(), "kl": kl.detach()}
