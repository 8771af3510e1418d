"""Parameter specifications of the reference networks on the hot path.

The state_dict key names and shapes are the checkpoint contract of the
reference (``Utils.loadModel`` -> ``load_state_dict(strict=True)``,
reference ``utils.py:68-73``).  They are derived here from an architecture
table instead of from module instantiation so that both the drop-in
``nn.Module`` classes and the native engine (which repacks weights into its
own layouts) read one source of truth.

Reference architecture sources:
  * ``models/unet_cond.py:10-30``  ResBlock (conv3x3 -> GN(1) -> GELU -> conv3x3 -> GN(1))
  * ``models/unet_cond.py:32-52``  AttenionBlock (LN, MHA(4 heads), LN/Linear/GELU/Linear)
  * ``models/unet_cond.py:54-100`` Down / Up (+ SiLU->Linear emb head)
  * ``models/unet_cond.py:113-153`` UnetCond topology
  * ``models/unet_cond_geom.py:8-49`` GeomHead + UnetCondWithGeomHead
  * ``models/unet.py:101-129``     unconditional Unet
  * ``models/vae.py:11-49``        VAE encoder/decoder
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, List, Tuple

Shape = Tuple[int, ...]

# Parameter "kinds" tell the synthetic generator which default-init
# distribution the reference framework would use for the tensor.
KIND_CONV_W = "conv_w"        # U(-1/sqrt(fan_in), +)
KIND_CONVT_W = "convt_w"      # ConvTranspose: fan_in from dim 1
KIND_BIAS = "bias"            # U(-1/sqrt(fan_in), +) -> carries fan_in
KIND_NORM_W = "norm_w"        # 1 + small perturbation
KIND_NORM_B = "norm_b"        # small perturbation
KIND_EMBED = "embed"          # N(0, 1)
KIND_XAVIER = "xavier"        # MHA in_proj_weight


class ParamSpec(OrderedDict):
    """name -> (shape, kind, fan_in)."""

    def add(self, name: str, shape: Shape, kind: str, fan_in: int = 0) -> None:
        self[name] = (tuple(int(s) for s in shape), kind, int(fan_in))

    def shapes(self) -> Dict[str, Shape]:
        return OrderedDict((k, v[0]) for k, v in self.items())


def _resblock(sp: ParamSpec, p: str, cin: int, cout: int, mid: int = 0) -> None:
    mid = mid or cout
    sp.add(f"{p}.double_conv.0.weight", (mid, cin, 3, 3), KIND_CONV_W, cin * 9)
    sp.add(f"{p}.double_conv.1.weight", (mid,), KIND_NORM_W)
    sp.add(f"{p}.double_conv.1.bias", (mid,), KIND_NORM_B)
    sp.add(f"{p}.double_conv.3.weight", (cout, mid, 3, 3), KIND_CONV_W, mid * 9)
    sp.add(f"{p}.double_conv.4.weight", (cout,), KIND_NORM_W)
    sp.add(f"{p}.double_conv.4.bias", (cout,), KIND_NORM_B)


def _linear(sp: ParamSpec, p: str, fin: int, fout: int) -> None:
    sp.add(f"{p}.weight", (fout, fin), KIND_CONV_W, fin)
    sp.add(f"{p}.bias", (fout,), KIND_BIAS, fin)


def _down(sp: ParamSpec, p: str, cin: int, cout: int, emb: int) -> None:
    _resblock(sp, f"{p}.maxpool_conv.1", cin, cin)
    _resblock(sp, f"{p}.maxpool_conv.2", cin, cout)
    _linear(sp, f"{p}.emb_layer.1", emb, cout)


def _up(sp: ParamSpec, p: str, cin: int, cout: int, emb: int) -> None:
    _resblock(sp, f"{p}.conv.0", cin, cin)
    _resblock(sp, f"{p}.conv.1", cin, cout, cin // 2)
    _linear(sp, f"{p}.emb_layer.1", emb, cout)


def _attn(sp: ParamSpec, p: str, c: int) -> None:
    sp.add(f"{p}.mha.in_proj_weight", (3 * c, c), KIND_XAVIER, c)
    sp.add(f"{p}.mha.in_proj_bias", (3 * c,), KIND_NORM_B)
    sp.add(f"{p}.mha.out_proj.weight", (c, c), KIND_CONV_W, c)
    sp.add(f"{p}.mha.out_proj.bias", (c,), KIND_NORM_B)
    sp.add(f"{p}.ln.weight", (c,), KIND_NORM_W)
    sp.add(f"{p}.ln.bias", (c,), KIND_NORM_B)
    sp.add(f"{p}.ff_self.0.weight", (c,), KIND_NORM_W)
    sp.add(f"{p}.ff_self.0.bias", (c,), KIND_NORM_B)
    _linear(sp, f"{p}.ff_self.1", c, c)
    _linear(sp, f"{p}.ff_self.3", c, c)


# Topology table shared by UnetCond and Unet (models/unet_cond.py:131-153,
# models/unet.py:107-129).  Entries: (kind, name, args).
def unet_topology(in_ch: int = 4, remove_deep_conv: bool = False) -> List[tuple]:
    topo = [
        ("res", "inc", (in_ch, 64, 0)),
        ("down", "down1", (64, 128)),
        ("attn", "sa1", (128,)),
        ("down", "down2", (128, 256)),
        ("attn", "sa2", (256,)),
        ("down", "down3", (256, 256)),
        ("attn", "sa3", (256,)),
    ]
    if remove_deep_conv:
        topo += [("res", "bot1", (256, 256, 0)), ("res", "bot3", (256, 256, 0))]
    else:
        topo += [("res", "bot1", (256, 512, 0)), ("res", "bot2", (512, 512, 0)),
                 ("res", "bot3", (512, 256, 0))]
    topo += [
        ("up", "up1", (512, 128)),
        ("attn", "sa4", (128,)),
        ("up", "up2", (256, 64)),
        ("attn", "sa5", (64,)),
        ("up", "up3", (128, 64)),
        ("attn", "sa6", (64,)),
    ]
    return topo


def _unet_body(sp: ParamSpec, in_ch: int, time_dim: int, remove_deep_conv: bool) -> None:
    for kind, name, args in unet_topology(in_ch, remove_deep_conv):
        if kind == "res":
            _resblock(sp, name, *args)
        elif kind == "down":
            _down(sp, name, args[0], args[1], time_dim)
        elif kind == "up":
            _up(sp, name, args[0], args[1], time_dim)
        else:
            _attn(sp, name, args[0])
    sp.add("out.weight", (in_ch, 64, 1, 1), KIND_CONV_W, 64)
    sp.add("out.bias", (in_ch,), KIND_BIAS, 64)


def unet_cond_geom_spec(in_ch: int = 4, time_dim: int = 256, num_classes: int = 3,
                        remove_deep_conv: bool = False, geom_dim: int = 12,
                        geom_hidden: int = 256) -> ParamSpec:
    """Keys of ``UnetCondWithGeomHead`` (models/unet_cond_geom.py:26-49)."""
    sp = ParamSpec()
    sp.add("class_emb.weight", (num_classes + 1, time_dim), KIND_EMBED)
    _linear(sp, "cond_mlp.0", 24, time_dim)
    _linear(sp, "cond_mlp.2", time_dim, time_dim)
    _unet_body(sp, in_ch, time_dim, remove_deep_conv)
    _linear(sp, "geom_head.mlp.0", 64, geom_hidden)
    _linear(sp, "geom_head.mlp.2", geom_hidden, geom_dim)
    return sp


def unet_cond_spec(in_ch: int = 4, time_dim: int = 256, num_classes: int = 3,
                   remove_deep_conv: bool = False) -> ParamSpec:
    """Keys of ``UnetCond`` (models/unet_cond.py:113-153)."""
    sp = ParamSpec()
    sp.add("class_emb.weight", (num_classes + 1, time_dim), KIND_EMBED)
    _linear(sp, "cond_mlp.0", 24, time_dim)
    _linear(sp, "cond_mlp.2", time_dim, time_dim)
    _unet_body(sp, in_ch, time_dim, remove_deep_conv)
    return sp


def unet_spec(in_ch: int = 3, time_dim: int = 256, remove_deep_conv: bool = False) -> ParamSpec:
    """Keys of the unconditional ``Unet`` (models/unet.py:101-129)."""
    sp = ParamSpec()
    _unet_body(sp, in_ch, time_dim, remove_deep_conv)
    return sp


# VAE layer table (models/vae.py:17-49): (index, kind, cin, cout, k)
VAE_ENC = [(0, "conv", 3, 64, 3), (1, "gn", 64), (3, "conv", 64, 64, 4), (4, "gn", 64),
           (6, "conv", 64, 128, 3), (7, "gn", 128), (9, "conv", 128, 128, 4), (10, "gn", 128),
           (12, "conv", 128, 256, 3), (13, "gn", 256), (15, "conv", 256, 256, 4), (16, "gn", 256)]
VAE_DEC = [(0, "conv", 4, 256, 3), (1, "gn", 256), (3, "convt", 256, 256, 4), (4, "gn", 256),
           (6, "conv", 256, 128, 3), (7, "gn", 128), (9, "convt", 128, 128, 4), (10, "gn", 128),
           (12, "conv", 128, 64, 3), (13, "gn", 64), (15, "convt", 64, 64, 4), (16, "gn", 64),
           (18, "conv", 64, 3, 3)]


def _vae_seq(sp: ParamSpec, prefix: str, table, in_ch: int, z_ch: int, base: int) -> None:
    scale = {3: in_ch, 4: z_ch, 64: base, 128: base * 2, 256: base * 4}
    for ent in table:
        idx, kind = ent[0], ent[1]
        if kind == "gn":
            c = scale[ent[2]]
            sp.add(f"{prefix}.{idx}.weight", (c,), KIND_NORM_W)
            sp.add(f"{prefix}.{idx}.bias", (c,), KIND_NORM_B)
        else:
            cin, cout, k = scale[ent[2]], scale[ent[3]], ent[4]
            if kind == "conv":
                sp.add(f"{prefix}.{idx}.weight", (cout, cin, k, k), KIND_CONV_W, cin * k * k)
                sp.add(f"{prefix}.{idx}.bias", (cout,), KIND_BIAS, cin * k * k)
            else:  # ConvTranspose2d weight is [Cin, Cout, k, k]; torch fan_in = Cout*k*k
                sp.add(f"{prefix}.{idx}.weight", (cin, cout, k, k), KIND_CONVT_W, cout * k * k)
                sp.add(f"{prefix}.{idx}.bias", (cout,), KIND_BIAS, cout * k * k)


def vae_spec(in_channels: int = 3, z_channels: int = 4, base_channels: int = 64) -> ParamSpec:
    """Keys of ``VAE`` (models/vae.py:11-49)."""
    sp = ParamSpec()
    _vae_seq(sp, "enc", VAE_ENC, in_channels, z_channels, base_channels)
    c4 = base_channels * 4
    sp.add("to_mu.weight", (z_channels, c4, 1, 1), KIND_CONV_W, c4)
    sp.add("to_mu.bias", (z_channels,), KIND_BIAS, c4)
    sp.add("to_logvar.weight", (z_channels, c4, 1, 1), KIND_CONV_W, c4)
    sp.add("to_logvar.bias", (z_channels,), KIND_BIAS, c4)
    _vae_seq(sp, "dec", VAE_DEC, in_channels, z_channels, base_channels)
    return sp
