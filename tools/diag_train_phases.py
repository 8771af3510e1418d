"""Diagnostic: wall time of each phase of the bench training step (synchronised between phases)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "diffusion-model_amd"), REPO):
    sys.path.insert(0, p)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import diff  # noqa: E402
from dmx import synth  # noqa: E402
from losses.geom_losses import masked_geom_mse  # noqa: E402
from models.unet_cond_geom import UnetCondWithGeomHead  # noqa: E402
from models.vae import VAE  # noqa: E402

dev = torch.device("cuda:0")
B = 32
g = torch.Generator().manual_seed(7)
model = UnetCondWithGeomHead()
model.load_state_dict(synth.unet_cond_geom_weights(0))
model.to(dev).train()
vae = VAE()
vae.load_state_dict(synth.vae_weights(1))
vae.to(dev).eval()
for p in vae.parameters():
    p.requires_grad = False
opt = torch.optim.Adam(model.parameters(), lr=1e-4)
d = diff.Diffuser(1000, device=dev)
images = torch.rand((B, 3, 224, 224), generator=g).to(dev)
vals = torch.rand((B, 12), generator=g).to(dev)
mask = (torch.rand((B, 12), generator=g) > 0.3).float().to(dev)
classes = torch.randint(1, 4, (B,), generator=g).to(dev)
T = {}


def tick(name, t0):
    torch.cuda.synchronize()
    t = time.perf_counter()
    T[name] = T.get(name, 0.0) + (t - t0)
    return t


for it in range(12):
    if it == 2:
        T.clear()
    t0 = time.perf_counter()
    with torch.no_grad():
        z = torch.cat([vae.encode(mb)[0] for mb in images.split(8, dim=0)], dim=0)
    t0 = tick("vae_encode", t0)
    t = torch.randint(1, 1001, (B,), device=dev)
    z_noisy, noise = d.add_noise(z, t)
    drop = torch.rand(B, device=dev) < 0.1
    y_used = torch.where(drop, torch.zeros_like(classes), classes)
    keep = (~drop).float().unsqueeze(1)
    t0 = tick("add_noise", t0)
    eps, geom = model(z_noisy, t, y_used, cond_vals=vals * keep, cond_mask=mask * keep)
    t0 = tick("forward", t0)
    loss = F.mse_loss(eps, noise) + 0.5 * masked_geom_mse(geom, vals, mask * keep)
    opt.zero_grad(set_to_none=True)
    t0 = tick("loss", t0)
    loss.backward()
    t0 = tick("backward", t0)
    opt.step()
    t0 = tick("adam", t0)
for k, v in T.items():
    print(f"{k:12s} {v / 10 * 1e3:8.3f} ms")
print("total", sum(T.values()) / 10 * 1e3)
