"""The bench.py training step alone (bench.train_leg's step: VAE encode x4, add_noise, forward, losses,
native backward, Adam, then the next forward's weight refresh), 2 warm + 10 steps, for
rocprofv3 --kernel-trace --stats (per-kernel time of the whole training step, B = 32)."""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "diffusion-model_amd"), ROOT]
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
diffuser = diff.Diffuser(1000, device=dev)
images = torch.rand((B, 3, 224, 224), generator=g).to(dev)
vals = torch.rand((B, 12), generator=g).to(dev)
mask = (torch.rand((B, 12), generator=g) > 0.3).float().to(dev)
classes = torch.randint(1, 4, (B,), generator=g).to(dev)
for _ in range(12):
    with torch.no_grad():
        z = torch.cat([vae.encode(mb)[0] for mb in images.split(8, dim=0)], dim=0)
    t = torch.randint(1, 1001, (B,), device=dev)
    z_noisy, noise = diffuser.add_noise(z, t)
    drop = torch.rand(B, device=dev) < 0.1
    y_used = torch.where(drop, torch.zeros_like(classes), classes)
    keep = (~drop).float().unsqueeze(1)
    eps, geom = model(z_noisy, t, y_used, cond_vals=vals * keep, cond_mask=mask * keep)
    loss = F.mse_loss(eps, noise) + 0.5 * masked_geom_mse(geom, vals, mask * keep)
    opt.zero_grad(set_to_none=True)
    loss.backward()
    opt.step()
torch.cuda.synchronize()
print("[train_step_prof] done", float(loss), flush=True)
