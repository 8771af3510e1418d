"""CPU restatement of one training step of the conditional U-Net (TEST INFRASTRUCTURE ONLY; see
``oracle/__init__.py`` for who may import it).

train_latent_cond.py:136-163: z_noisy, noise = diffuser.add_noise(z, t) (diff.py:18-30);
noise_pred, geom_pred = model(z_noisy, t, y_used, cond_vals=vals_used, cond_mask=mask_used);
loss = F.mse_loss(noise_pred, noise) + geom_lambda * masked_geom_mse(geom_pred, vals, geom_mask_eff)
(losses/geom_losses.py:4-17); loss.backward(); Adam(lr).step().  The network is the functional
restatement in ``oracle/ref.py`` with the parameters as autograd leaves, so the gradients are
torch autograd's over the same graph.  Pinned by tests/golden/train_step.npz (the reference
module's own loss.backward(), see tests/golden/make_golden_train.py).
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch
import torch.nn.functional as F

from . import ref


def masked_geom_mse(pred: torch.Tensor, gt: torch.Tensor, mask: torch.Tensor, eps: float = 1e-6) -> torch.Tensor:
    """losses/geom_losses.py:4-17: sum(mask (pred - gt)^2) / max(sum(mask), eps)."""
    return ((pred - gt) ** 2 * mask).sum() / mask.sum().clamp_min(eps)


def forward(sd, x, t, y, vals=None, mask=None, geom: bool = True, remove_deep_conv: bool = False):
    """UnetCondWithGeomHead (geom=True, unet_cond_geom.py:79-100) or UnetCond (unet_cond.py:197-216
    with cfg_drop_prob 0) -> (eps, geom_pred or None)."""
    if geom:
        return ref.unet_cond_geom_forward(sd, x, t, y, vals, mask, remove_deep_conv)
    emb = ref.cond_embedding(sd, t, y, vals, mask)
    eps, _ = ref.unet_trunk(sd, x, emb, remove_deep_conv)
    return eps, None


def loss_and_grads(sd: Dict[str, torch.Tensor], x, t, y, vals, mask, noise, geom_gt=None, geom_mask=None,
                   geom_lambda: float = 0.0, geom: bool = True, remove_deep_conv: bool = False
                   ) -> Tuple[torch.Tensor, torch.Tensor, Optional[torch.Tensor], Dict[str, Optional[torch.Tensor]]]:
    """-> (loss, eps, geom_pred, {name: dLoss/dparam or None}) for the train_latent_cond loss."""
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in sd.items()}
    eps, g = forward(leaves, x, t, y, vals, mask, geom, remove_deep_conv)
    loss = F.mse_loss(eps, noise)
    if g is not None and geom_gt is not None:
        loss = loss + geom_lambda * masked_geom_mse(g, geom_gt, geom_mask)
    loss.backward()
    return loss.detach(), eps.detach(), (g.detach() if g is not None else None), {k: v.grad for k, v in leaves.items()}
