"""The reference networks' module trees, built from stock ``torch.nn`` layers.

The drop-in networks need three things from their parameter tree:

* the reference's state_dict names and shapes (the checkpoint contract of
  ``Utils.loadModel``, reference ``utils.py:68-73``);
* the reference's *module* paths (``model.inc.double_conv[0]`` etc.), so that code
  poking at sub-modules keeps working;
* the reference's construction side effect: every ``nn.Conv2d`` / ``nn.Linear`` /
  ``nn.Embedding`` / ``nn.MultiheadAttention`` initialiser draws from the global torch
  generator, in construction order.  A script that seeds, builds the models and then
  samples must see the same x_T and noise stream as with the reference.

Building the tree from the very ``torch.nn`` layers the reference instantiates, in the
reference's order, gives all three by construction.  The containers hold parameters
only: the networks' forward passes run in libdmx (``models/_native.py``), and calling a
container directly raises.

Reference structure: ``models/unet_cond.py:10-100`` (ResBlock, AttenionBlock, Down, Up),
``models/unet_cond.py:113-153`` / ``models/unet.py:101-129`` (U-Net topology),
``models/unet_cond_geom.py:8-49`` (GeomHead), ``models/vae.py:11-49`` (VAE stacks).
"""
from __future__ import annotations

from torch import nn

from dmx import spec


class _Holder(nn.Module):
    """Parameter container of one reference sub-module (no host compute)."""

    def forward(self, *args, **kwargs):  # noqa: D401
        raise RuntimeError(f"{type(self).__name__} is a parameter container of a dmx network; the forward pass "
                           f"runs natively for the whole network (call the top-level model)")


class ResBlock(_Holder):
    """conv3x3 -> GN(1) -> GELU -> conv3x3 -> GN(1) (models/unet_cond.py:10-24)."""

    def __init__(self, in_channels, out_channels, mid_channels=None, residual=False):
        super().__init__()
        self.residual = residual
        mid = mid_channels or out_channels
        layers = [nn.Conv2d(in_channels, mid, kernel_size=3, padding=1, bias=False), nn.GroupNorm(1, mid), nn.GELU(),
                  nn.Conv2d(mid, out_channels, kernel_size=3, padding=1, bias=False), nn.GroupNorm(1, out_channels)]
        self.double_conv = nn.Sequential(*layers)


class AttenionBlock(_Holder):
    """LN -> 4-head MHA -> residual -> LN/Linear/GELU/Linear -> residual (models/unet_cond.py:32-43)."""

    def __init__(self, channels):
        super().__init__()
        self.channels = channels
        self.mha = nn.MultiheadAttention(channels, 4, batch_first=True)
        self.ln = nn.LayerNorm([channels])
        self.ff_self = nn.Sequential(nn.LayerNorm([channels]), nn.Linear(channels, channels), nn.GELU(),
                                     nn.Linear(channels, channels))


def _emb_head(emb_dim, out_channels):
    return nn.Sequential(nn.SiLU(), nn.Linear(emb_dim, out_channels))


class Down(_Holder):
    """MaxPool2 -> residual ResBlock -> ResBlock, + SiLU/Linear emb shift (models/unet_cond.py:54-65)."""

    def __init__(self, in_channels, out_channels, emb_dim=256):
        super().__init__()
        self.maxpool_conv = nn.Sequential(nn.MaxPool2d(2), ResBlock(in_channels, in_channels, residual=True),
                                          ResBlock(in_channels, out_channels))
        self.emb_layer = _emb_head(emb_dim, out_channels)


class Up(_Holder):
    """bilinear x2 -> pad -> cat -> residual ResBlock -> ResBlock(mid=in/2), + emb (models/unet_cond.py:72-85)."""

    def __init__(self, in_channels, out_channels, emb_dim=256):
        super().__init__()
        self.up = nn.Upsample(scale_factor=2, mode="bilinear", align_corners=True)
        self.conv = nn.Sequential(ResBlock(in_channels, in_channels, residual=True),
                                  ResBlock(in_channels, out_channels, in_channels // 2))
        self.emb_layer = _emb_head(emb_dim, out_channels)


class GeomHead(_Holder):
    """GAP -> Linear -> SiLU -> Linear (models/unet_cond_geom.py:8-18)."""

    def __init__(self, in_ch, out_dim, hidden=256):
        super().__init__()
        self.mlp = nn.Sequential(nn.Linear(in_ch, hidden), nn.SiLU(), nn.Linear(hidden, out_dim))


def build_unet_body(model: nn.Module, in_ch: int, remove_deep_conv: bool) -> None:
    """inc .. sa6, out in the reference's assignment order (models/unet_cond.py:131-153,
    models/unet.py:107-129); Down/Up keep their emb_dim=256 default like the reference."""
    kinds = {"res": lambda a: ResBlock(a[0], a[1]), "down": lambda a: Down(a[0], a[1]),
             "up": lambda a: Up(a[0], a[1]), "attn": lambda a: AttenionBlock(a[0])}
    for kind, name, args in spec.unet_topology(in_ch, remove_deep_conv):
        setattr(model, name, kinds[kind](args))
    model.out = nn.Conv2d(64, in_ch, kernel_size=1)


def build_cond_embedding(model: nn.Module, num_classes: int, time_dim: int) -> None:
    """class_emb + cond_mlp (models/unet_cond.py:121-129)."""
    model.class_emb = nn.Embedding(num_classes + 1, time_dim)
    model.cond_mlp = nn.Sequential(nn.Linear(12 * 2, time_dim), nn.SiLU(), nn.Linear(time_dim, time_dim))


def _vae_stack(table, in_channels: int, z_channels: int, base: int) -> nn.Sequential:
    width = {3: in_channels, 4: z_channels, 64: base, 128: base * 2, 256: base * 4}
    layers = []
    for ent in table:
        if ent[1] == "gn":
            layers += [nn.GroupNorm(8, width[ent[2]]), nn.GELU()]
            continue
        cin, cout, k = width[ent[2]], width[ent[3]], ent[4]
        if ent[1] == "convt":
            layers.append(nn.ConvTranspose2d(cin, cout, k, stride=2, padding=1))
        elif k == 4:
            layers.append(nn.Conv2d(cin, cout, k, stride=2, padding=1))
        else:
            layers.append(nn.Conv2d(cin, cout, k, stride=1, padding=1))
    return nn.Sequential(*layers)


def build_vae(model: nn.Module, in_channels: int, z_channels: int, base_channels: int) -> None:
    """enc, to_mu, to_logvar, dec (models/vae.py:17-49)."""
    model.enc = _vae_stack(spec.VAE_ENC, in_channels, z_channels, base_channels)
    model.to_mu = nn.Conv2d(base_channels * 4, z_channels, 1)
    model.to_logvar = nn.Conv2d(base_channels * 4, z_channels, 1)
    model.dec = _vae_stack(spec.VAE_DEC, in_channels, z_channels, base_channels)
