"""Native training forward + backward at the train_latent_cond shape (B=32, 28x28x4), for
rocprofv3 --kernel-trace --stats (per-kernel time of the training step)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "diffusion-model_amd"), ROOT]
from dmx import synth  # noqa: E402
from models.unet_cond_geom import UnetCondWithGeomHead  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(3)
m = UnetCondWithGeomHead()
m.load_state_dict(synth.unet_cond_geom_weights(0))
m.to(dev).train()
nm = m.native()
z = torch.randn((B, 4, 28, 28), generator=g).to(dev)
t = torch.randint(1, 1001, (B,), generator=g).to(dev)
y = torch.randint(0, 4, (B,), generator=g).to(dev)
vals = torch.rand((B, 12), generator=g).to(dev)
mask = (torch.rand((B, 12), generator=g) > 0.3).float().to(dev)
d_eps, d_geom = torch.randn_like(z), torch.randn((B, nm.geom_dim), device=dev)
for _ in range(iters):
    _, _, tape = nm.train_forward(z, t, y, vals, mask)
    nm.train_backward(tape, d_eps, d_geom)
torch.cuda.synchronize()
print("[train_prof] done", flush=True)
