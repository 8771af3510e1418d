"""Functional CPU restatement of the reference hot path (TEST INFRASTRUCTURE).

All tensors are fp32 NCHW on the CPU; weights come as a plain
``{name: tensor}`` dict with the reference's state_dict keys.  See
``oracle/__init__.py`` for the rules on who may import this module.
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Tuple

import torch
import torch.nn.functional as F

SD = Dict[str, torch.Tensor]


# ---------------------------------------------------------------------------
# U-Net building blocks
# ---------------------------------------------------------------------------
def resblock(sd: SD, p: str, x: torch.Tensor, residual: bool) -> torch.Tensor:
    """models/unet_cond.py:10-30 — conv3x3 -> GN(1) -> GELU -> conv3x3 -> GN(1) [-> GELU(x + .)]."""
    h = F.conv2d(x, sd[f"{p}.double_conv.0.weight"], None, 1, 1)
    h = F.group_norm(h, 1, sd[f"{p}.double_conv.1.weight"], sd[f"{p}.double_conv.1.bias"], 1e-5)
    h = F.gelu(h)
    h = F.conv2d(h, sd[f"{p}.double_conv.3.weight"], None, 1, 1)
    h = F.group_norm(h, 1, sd[f"{p}.double_conv.4.weight"], sd[f"{p}.double_conv.4.bias"], 1e-5)
    return F.gelu(x + h) if residual else h


def emb_head(sd: SD, p: str, emb: torch.Tensor) -> torch.Tensor:
    """models/unet_cond.py:62-65 / 82-85 — SiLU -> Linear, broadcast over H, W (69, 99)."""
    return F.linear(F.silu(emb), sd[f"{p}.emb_layer.1.weight"], sd[f"{p}.emb_layer.1.bias"])[:, :, None, None]


def down(sd: SD, p: str, x: torch.Tensor, emb: torch.Tensor) -> torch.Tensor:
    """models/unet_cond.py:54-70 — MaxPool2 -> ResBlock(res) -> ResBlock -> + emb."""
    h = F.max_pool2d(x, 2)
    h = resblock(sd, f"{p}.maxpool_conv.1", h, True)
    h = resblock(sd, f"{p}.maxpool_conv.2", h, False)
    return h + emb_head(sd, p, emb)


def up(sd: SD, p: str, x: torch.Tensor, skip: torch.Tensor, emb: torch.Tensor) -> torch.Tensor:
    """models/unet_cond.py:72-100 — bilinear x2 (align_corners) -> pad -> cat[skip, x] -> 2 ResBlocks -> + emb."""
    h = F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=True)
    dy = skip.size(2) - h.size(2)
    dx = skip.size(3) - h.size(3)
    if dy != 0 or dx != 0:
        h = F.pad(h, [max(0, dx // 2), max(0, dx - dx // 2), max(0, dy // 2), max(0, dy - dy // 2)])
    h = torch.cat([skip, h], dim=1)
    h = resblock(sd, f"{p}.conv.0", h, True)
    h = resblock(sd, f"{p}.conv.1", h, False)
    return h + emb_head(sd, p, emb)


def attention(sd: SD, p: str, x: torch.Tensor) -> torch.Tensor:
    """models/unet_cond.py:32-52 — tokens = NCHW->(N,L,C); the residual is the LN *output* (48)."""
    n, c, hh, ww = x.shape
    heads = 4
    tok = x.reshape(n, c, hh * ww).transpose(1, 2)
    xl = F.layer_norm(tok, (c,), sd[f"{p}.ln.weight"], sd[f"{p}.ln.bias"], 1e-5)
    qkv = F.linear(xl, sd[f"{p}.mha.in_proj_weight"], sd[f"{p}.mha.in_proj_bias"])
    q, k, v = qkv.split(c, dim=-1)
    d = c // heads

    def split(z):
        return z.reshape(n, hh * ww, heads, d).transpose(1, 2)

    q, k, v = split(q), split(k), split(v)
    s = torch.matmul(q * (1.0 / math.sqrt(d)), k.transpose(-1, -2))
    a = torch.matmul(torch.softmax(s, dim=-1), v)
    a = a.transpose(1, 2).reshape(n, hh * ww, c)
    a = F.linear(a, sd[f"{p}.mha.out_proj.weight"], sd[f"{p}.mha.out_proj.bias"]) + xl
    f = F.layer_norm(a, (c,), sd[f"{p}.ff_self.0.weight"], sd[f"{p}.ff_self.0.bias"], 1e-5)
    f = F.linear(f, sd[f"{p}.ff_self.1.weight"], sd[f"{p}.ff_self.1.bias"])
    f = F.linear(F.gelu(f), sd[f"{p}.ff_self.3.weight"], sd[f"{p}.ff_self.3.bias"])
    out = f + a
    return out.transpose(1, 2).reshape(n, c, hh, ww)


def pos_encoding(t: torch.Tensor, channels: int = 256) -> torch.Tensor:
    """models/unet_cond.py:155-161 — [sin(t f), cos(t f)] halves, f = 1/10000^(2k/C)."""
    inv_freq = 1.0 / (10000 ** (torch.arange(0, channels, 2).float() / channels))
    tt = t.reshape(-1, 1).repeat(1, channels // 2)
    return torch.cat([torch.sin(tt * inv_freq), torch.cos(tt * inv_freq)], dim=-1)


def unet_trunk(sd: SD, x: torch.Tensor, emb: torch.Tensor, remove_deep_conv: bool = False):
    """models/unet_cond_geom.py:52-76 (== models/unet_cond.py:169-195) -> (eps, feat)."""
    x1 = resblock(sd, "inc", x, False)
    x2 = attention(sd, "sa1", down(sd, "down1", x1, emb))
    x3 = attention(sd, "sa2", down(sd, "down2", x2, emb))
    x4 = attention(sd, "sa3", down(sd, "down3", x3, emb))
    x4 = resblock(sd, "bot1", x4, False)
    if not remove_deep_conv:
        x4 = resblock(sd, "bot2", x4, False)
    x4 = resblock(sd, "bot3", x4, False)
    h = attention(sd, "sa4", up(sd, "up1", x4, x3, emb))
    h = attention(sd, "sa5", up(sd, "up2", h, x2, emb))
    feat = attention(sd, "sa6", up(sd, "up3", h, x1, emb))
    eps = F.conv2d(feat, sd["out.weight"], sd["out.bias"])
    return eps, feat


def cond_embedding(sd: SD, t: torch.Tensor, y: torch.Tensor,
                   vals: Optional[torch.Tensor], mask: Optional[torch.Tensor]) -> torch.Tensor:
    """models/unet_cond.py:163-167 + unet_cond_geom.py:89-95."""
    emb = pos_encoding(t.float()) + F.embedding(y, sd["class_emb.weight"])
    if vals is not None and mask is not None:
        h = torch.cat([vals, mask], dim=1)
        h = F.linear(F.silu(F.linear(h, sd["cond_mlp.0.weight"], sd["cond_mlp.0.bias"])),
                     sd["cond_mlp.2.weight"], sd["cond_mlp.2.bias"])
        emb = emb + h
    return emb


def unet_cond_geom_forward(sd: SD, x, t, y, vals=None, mask=None, remove_deep_conv=False):
    """models/unet_cond_geom.py:79-100 -> (eps, geom)."""
    emb = cond_embedding(sd, t, y, vals, mask)
    eps, feat = unet_trunk(sd, x, emb, remove_deep_conv)
    g = feat.mean(dim=(2, 3))
    g = F.linear(F.silu(F.linear(g, sd["geom_head.mlp.0.weight"], sd["geom_head.mlp.0.bias"])),
                 sd["geom_head.mlp.2.weight"], sd["geom_head.mlp.2.bias"])
    return eps, g


def unet_forward(sd: SD, x, t, remove_deep_conv=False):
    """models/unet.py:167-170 — unconditional: emb = pos_encoding(t) only."""
    eps, _ = unet_trunk(sd, x, pos_encoding(t.float()), remove_deep_conv)
    return eps


# ---------------------------------------------------------------------------
# VAE decoder
# ---------------------------------------------------------------------------
def vae_decode(sd: SD, z: torch.Tensor, scale_factor: float = 0.18215) -> torch.Tensor:
    """models/vae.py:64-69 (decoder layers 35-49): z/s -> dec -> sigmoid."""
    h = z / scale_factor

    def gn_gelu(h, i):
        return F.gelu(F.group_norm(h, 8, sd[f"dec.{i}.weight"], sd[f"dec.{i}.bias"], 1e-5))

    h = gn_gelu(F.conv2d(h, sd["dec.0.weight"], sd["dec.0.bias"], 1, 1), 1)
    h = gn_gelu(F.conv_transpose2d(h, sd["dec.3.weight"], sd["dec.3.bias"], 2, 1), 4)
    h = gn_gelu(F.conv2d(h, sd["dec.6.weight"], sd["dec.6.bias"], 1, 1), 7)
    h = gn_gelu(F.conv_transpose2d(h, sd["dec.9.weight"], sd["dec.9.bias"], 2, 1), 10)
    h = gn_gelu(F.conv2d(h, sd["dec.12.weight"], sd["dec.12.bias"], 1, 1), 13)
    h = gn_gelu(F.conv_transpose2d(h, sd["dec.15.weight"], sd["dec.15.bias"], 2, 1), 16)
    h = F.conv2d(h, sd["dec.18.weight"], sd["dec.18.bias"], 1, 1)
    return torch.sigmoid(h)


def vae_encode(sd: SD, x: torch.Tensor, eps: torch.Tensor, scale_factor: float = 0.18215):
    """models/vae.py:51-62 (encoder layers 17-30) with the randn_like draw passed in as eps:
    returns (z, kl.mean(), mu, clamped logvar)."""
    h = x
    for i, (stride, pad) in ((0, (1, 1)), (3, (2, 1)), (6, (1, 1)), (9, (2, 1)), (12, (1, 1)), (15, (2, 1))):
        h = F.conv2d(h, sd[f"enc.{i}.weight"], sd[f"enc.{i}.bias"], stride, pad)
        h = F.gelu(F.group_norm(h, 8, sd[f"enc.{i + 1}.weight"], sd[f"enc.{i + 1}.bias"], 1e-5))
    mu = F.conv2d(h, sd["to_mu.weight"], sd["to_mu.bias"])
    logvar = F.conv2d(h, sd["to_logvar.weight"], sd["to_logvar.bias"]).clamp(-30.0, 20.0)
    z = (mu + eps * torch.exp(0.5 * logvar)) * scale_factor
    kl = 0.5 * torch.sum(torch.exp(logvar) + mu ** 2 - 1.0 - logvar, dim=(1, 2, 3)) / (x.size(2) * x.size(3))
    return z, kl.mean(), mu, logvar


def vae_forward(sd: SD, x: torch.Tensor, eps: torch.Tensor, scale_factor: float = 0.18215):
    """models/vae.py:71-76 (inference form, eps passed in): encode -> decode -> mean-squared
    reconstruction error + 1e-6 * KL.  Returns (x_recon, z, loss, recon_mse, kl)."""
    z, kl, _, _ = vae_encode(sd, x, eps, scale_factor)
    x_recon = vae_decode(sd, z, scale_factor)
    recon = F.mse_loss(x_recon, x, reduction="mean")
    return x_recon, z, recon + 1e-6 * kl, recon, kl


def to_uint8(img: torch.Tensor) -> torch.Tensor:
    """diff.py:58-62 — x*255 -> clamp(0,255) -> .to(uint8) (truncation)."""
    return (img * 255).clamp(0, 255).to(torch.uint8)


# ---------------------------------------------------------------------------
# DDPM schedule and CFG step
# ---------------------------------------------------------------------------
def schedule(T: int = 1000, beta_start: float = 1e-4, beta_end: float = 0.02):
    """diff.py:11-16."""
    betas = torch.linspace(beta_start, beta_end, T)
    alphas = 1 - betas
    return betas, alphas, torch.cumprod(alphas, dim=0)


def ddpm_update(x, eps, t, alphas, alpha_bars, noise, clamp_prev: bool = True):
    """diff.py:141-144,158-162 (clamp_prev=True, denoise_cond) / diff.py:36-56 (False, denoise)."""
    t_idx = t - 1
    a = alphas[t_idx].view(-1, 1, 1, 1)
    ab = alpha_bars[t_idx].view(-1, 1, 1, 1)
    prev_idx = torch.clamp(t_idx - 1, min=0) if clamp_prev else t_idx - 1
    abp = alpha_bars[prev_idx].view(-1, 1, 1, 1)
    noise = noise.clone()
    noise[t == 1] = 0
    mu = (x - ((1 - a) / torch.sqrt(1 - ab)) * eps) / torch.sqrt(a)
    std = torch.sqrt((1 - a) * (1 - abp) / (1 - ab))
    return mu + noise * std


def cfg_step(sd: SD, x, t, y, alphas, alpha_bars, guidance: float, null_label: int,
             vals, mask, noise, remove_deep_conv=False):
    """diff.py:127-162 — two model calls (uncond y=null, cond y), CFG mix, DDPM update."""
    y_null = torch.full_like(y, null_label)
    eu, _ = unet_cond_geom_forward(sd, x, t, y_null, vals, mask, remove_deep_conv)
    ec, _ = unet_cond_geom_forward(sd, x, t, y, vals, mask, remove_deep_conv)
    eps = eu + guidance * (ec - eu)
    return ddpm_update(x, eps, t, alphas, alpha_bars, noise)


def sample_latent_cond(sd: SD, y, vals, mask, z_shape, T=1000, guidance=3.0, null_label=0,
                       checkpoints=(), gen: Optional[torch.Generator] = None):
    """diff.py:327-344 — x_T ~ randn, then T CFG steps drawing one randn per step.

    Returns (x_0, {t: x_t-after-step-t}) using the global (or given) CPU generator
    in the same draw order as the reference.
    """
    _, alphas, alpha_bars = schedule(T)
    B = y.shape[0]
    x = torch.randn((B,) + tuple(z_shape), generator=gen)
    saved = {}
    with torch.no_grad():
        for i in range(T, 0, -1):
            t = torch.full((B,), i, dtype=torch.long)
            noise = torch.randn(x.shape, generator=gen)
            x = cfg_step(sd, x, t, y, alphas, alpha_bars, guidance, null_label, vals, mask, noise)
            if i in checkpoints:
                saved[i] = x.clone()
    return x, saved


# ---------------------------------------------------------------------------
# CSV conditioning (host numpy) — entityCsvSampler.py:101-163, 192-199
# ---------------------------------------------------------------------------
KEY_ORDER = ["x1", "y1", "x2", "y2", "cx", "cy", "cr", "ax", "ay", "ar", "theta1", "theta2"]


def build_vals_mask(table, class_id: int, base_wh: Tuple[float, float]):
    """entityCsvSampler.py:101-163 on a (rows, 13) float array."""
    import numpy as np
    W, H = base_wh
    tab = np.asarray(table, dtype=np.float32)
    B = tab.shape[0]
    vals = np.zeros((B, 12), np.float32)
    mask = np.zeros((B, 12), np.float32)
    fx = lambda c: tab[:, c].astype(np.float32) / np.float32(W)
    fy = lambda c: 1.0 - tab[:, c].astype(np.float32) / np.float32(H)

    def ang(v):
        out = v.astype(np.float32).copy()
        m = np.abs(out) > 1.0
        out[m] = (out[m] % 360.0) / 360.0
        return out

    if class_id == 1:
        cols = {0: fx(1), 1: fy(2), 2: fx(3), 3: fy(4)}
    elif class_id == 2:
        cols = {4: fx(5), 5: fy(6), 6: fx(7)}
    elif class_id == 3:
        cols = {7: fx(8), 8: fy(9), 9: fx(10), 10: ang(tab[:, 11]), 11: ang(tab[:, 12])}
    else:
        raise ValueError("class_id must be 1(line), 2(circle), or 3(arc).")
    for j, v in cols.items():
        vals[:, j] = v
        mask[:, j] = 1.0
    return vals, mask
