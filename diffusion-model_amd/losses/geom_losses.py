"""Drop-in ``losses.geom_losses`` (reference losses/geom_losses.py:4-17).

The training loop's masked regression loss on GeomHead's output; a handful of (B, K)
elementwise ops, left to torch (autograd then feeds its gradient into the native backward,
dmx_train_backward's d_geom)."""
import torch


def masked_geom_mse(geom_pred: torch.Tensor, geom_gt: torch.Tensor, geom_mask: torch.Tensor,
                    eps: float = 1e-6, denom: torch.Tensor = None) -> torch.Tensor:
    """sum(mask * (pred - gt)^2) / clamp_min(sum(mask), eps).

    ``denom`` (extension, default None = the reference's formula): use this mask sum instead of
    the local one.  Data-parallel training passes ``dmx.distributed.global_mask_mean(geom_mask)``
    — the mean over ranks of the local mask sums — so that the rank-averaged gradient
    (``GradAllReducer``) is the gradient of the global batch's masked mean (sum of all ranks'
    numerators over the sum of all ranks' mask sums)."""
    num = (geom_mask * (geom_pred - geom_gt).pow(2)).sum()
    d = geom_mask.sum() if denom is None else denom
    return num / d.clamp_min(eps)
