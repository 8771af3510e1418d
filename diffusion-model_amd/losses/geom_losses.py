"""Drop-in ``losses.geom_losses`` (reference losses/geom_losses.py:4-17).

The training loop's masked regression loss on GeomHead's output; a handful of (B, K)
elementwise ops, left to torch (autograd then feeds its gradient into the native backward,
dmx_train_backward's d_geom)."""
import torch


def masked_geom_mse(geom_pred: torch.Tensor, geom_gt: torch.Tensor, geom_mask: torch.Tensor,
                    eps: float = 1e-6) -> torch.Tensor:
    """sum(mask * (pred - gt)^2) / clamp_min(sum(mask), eps)."""
    num = (geom_mask * (geom_pred - geom_gt).pow(2)).sum()
    return num / geom_mask.sum().clamp_min(eps)
