"""Round-5 golden vector: a T=1000 CFG trajectory at the Winograd batch class.

Run from the repo root:  python tests/golden/make_golden_r5.py [28]
Same rules as make_golden.py: the reference is imported read-only from /root/reference
(one harness-side ``torchvision.transforms.ToPILImage`` stub), only the fixture written
here travels to the GPU box.

traj_T1000_B32.npz — the reference's ``Diffuser.denoise_cond`` (diff.py:127-162) looped
T=1000..1 as ``sample_latent_cond`` does (diff.py:326-344) at B=32, 32x32x4 latents,
CFG 3.0 — a 64-sample CFG forward per step, i.e. the batch class (>= 64 samples) whose
3x3 convs run dmx's Winograd kernels, the kernels bench.py times.  Conditions: classes
1..3, random vals and masks.  Stored: the final latents of all 32 samples; the latents
after t = 900, 500, 100 for samples 0..7 (samples evolve independently, so a subset pins
the intermediate states); the reference's VAE.decode -> reverse_to_img uint8 images of
samples 0..5.

traj_T1000_B32_28.npz (argument 28) — the same at 28x28x4 latents, the shape the reference's own
sampler draws (diff.py:315-322 with the 224 encode dummy): the 28 / 14 / 7 / 3 maps whose 3x3 convs
dmx runs in the Winograd kernel's 32 / 16 / 8 / 4 geometries with the missing rows / columns as
zero padding (seed 51).
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, HERE)
from make_golden import UNET_SEED, VAE_SEED, _install_torchvision_stub  # noqa: E402

B, T, SEED, SUB, IMGS = 32, 1000, 50, 8, 6
CKPTS = (900, 500, 100)


def main():
    hw = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    seed = SEED if hw == 32 else SEED + 1
    name = "traj_T1000_B32.npz" if hw == 32 else f"traj_T1000_B32_{hw}.npz"
    torch.set_num_threads(int(os.environ.get("GOLDEN_THREADS", "8")))
    _install_torchvision_stub()
    sys.path.insert(0, os.path.join(REPO, "diffusion-model_amd"))
    from dmx import synth  # our seeded weight generator (no reference code)
    sys.path.insert(0, REF)
    import diff as rdiff  # noqa: E402  (reference)
    from models.unet_cond_geom import UnetCondWithGeomHead  # noqa: E402
    from models.vae import VAE  # noqa: E402

    t0 = time.time()
    unet = UnetCondWithGeomHead()
    unet.load_state_dict(synth.unet_cond_geom_weights(UNET_SEED), strict=True)
    unet.eval()
    vae = VAE()
    vae.load_state_dict(synth.vae_weights(VAE_SEED), strict=True)
    vae.eval()
    d = rdiff.Diffuser(num_timesteps=T, device="cpu")

    y = torch.tensor([1 + i % 3 for i in range(B)], dtype=torch.long)
    g = torch.Generator().manual_seed(seed - 1)
    vals = torch.rand((B, 12), generator=g)
    mask = (torch.rand((B, 12), generator=g) > 0.3).float()
    torch.manual_seed(seed)
    x = torch.randn((B, 4, hw, hw))
    ck = {}
    with torch.no_grad():
        for i in range(T, 0, -1):
            t = torch.full((B,), i, dtype=torch.long)
            x = d.denoise_cond(unet, x, t, y=y, guidance_scale=3.0, null_label=0, cond_vals=vals, cond_mask=mask)
            if i in CKPTS:
                ck[f"x_{i}"] = x[:SUB].numpy().copy()
            if i % 50 == 0:
                print(f"[golden-r5] t={i} {time.time() - t0:.0f}s", flush=True)
        img = vae.decode(x[:IMGS])
    u8 = np.stack([np.asarray(d.reverse_to_img(img[i])) for i in range(IMGS)])
    np.savez_compressed(os.path.join(HERE, name), seed=seed, y=y.numpy(), vals=vals.numpy(),
                        mask=mask.numpy(), x_final=x.numpy(), u8=u8, sub=SUB, **ck)
    print(f"[golden-r5] done {time.time() - t0:.0f}s", flush=True)


if __name__ == "__main__":
    main()
