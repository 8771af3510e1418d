"""Golden vectors for VAE.encode (reference models/vae.py:51-62), build container only.

Run from the repo root:  python tests/golden/make_golden_encode.py
Imports the reference VAE read-only with the seeded synthetic weights of ``dmx.synth``
(VAE seed 1, as make_golden.py) and records, for two input sizes, the image x, the
randn_like draw eps (re-drawn from the same global seed: the encoder consumes no other
random numbers before it), z and the per-batch KL (``kl.mean()``) and the pre-sampling
mu / logvar.  Writes tests/golden/vae_encode.npz.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
VAE_SEED = 1


def main():
    torch.set_num_threads(8)
    sys.path.insert(0, os.path.join(REPO, "diffusion-model_amd"))
    from dmx import synth  # our seeded weight generator (no reference code)
    sys.path.insert(0, REF)
    from models.vae import VAE  # noqa: E402  (reference)

    vae = VAE()
    vae.load_state_dict(synth.vae_weights(VAE_SEED), strict=True)
    vae.eval()
    out = {}
    for tag, (b, hw, seed) in {"64": (2, 64, 31), "56": (3, 56, 32)}.items():
        g = torch.Generator().manual_seed(seed)
        x = torch.rand((b, 3, hw, hw), generator=g)
        torch.manual_seed(seed + 100)
        with torch.no_grad():
            z, kl = vae.encode(x)
            h = vae.enc(x)
            mu = vae.to_mu(h)
            lv = vae.to_logvar(h).clamp(-30.0, 20.0)
        torch.manual_seed(seed + 100)
        eps = torch.randn(z.shape)
        assert torch.equal((mu + eps * torch.exp(0.5 * lv)) * vae.scale_factor, z)
        out.update({f"x{tag}": x.numpy(), f"eps{tag}": eps.numpy(), f"z{tag}": z.numpy(),
                    f"kl{tag}": np.float32(kl.item()), f"mu{tag}": mu.numpy(), f"lv{tag}": lv.numpy(),
                    f"seed{tag}": seed + 100})
    np.savez_compressed(os.path.join(HERE, "vae_encode.npz"), **out)
    print("[golden] vae_encode.npz", {k: v.shape for k, v in out.items() if hasattr(v, "shape")})


if __name__ == "__main__":
    main()
