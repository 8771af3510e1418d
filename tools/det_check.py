"""Repeat one U-Net forward R times in one process and count runs whose eps differs bit-wise from the
first (GPU box): python tools/det_check.py [N] [hw] [R].  A race shows up as nondeterminism."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "diffusion-model_amd"), REPO]
import torch  # noqa: E402

from dmx import synth  # noqa: E402
from models.unet_cond_geom import UnetCondWithGeomHead  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 128
hw = int(sys.argv[2]) if len(sys.argv) > 2 else 32
R = int(sys.argv[3]) if len(sys.argv) > 3 else 20
m = UnetCondWithGeomHead()
m.load_state_dict(synth.unet_cond_geom_weights(0))
dev = torch.device("cuda:0")
m.to(dev).eval()
g = torch.Generator().manual_seed(128)
x = torch.randn((N, 4, hw, hw), generator=g).to(dev)
t = torch.randint(1, 1001, (N,), generator=g).to(dev)
y = torch.randint(0, 4, (N,), generator=g).to(dev)
vals = torch.rand((N, 12), generator=g).to(dev)
mask = (torch.rand((N, 12), generator=g) > 0.5).float().to(dev)
ref = None
bad = 0
samples = set()
with torch.no_grad():
    for r in range(R):
        eps, _ = m(x, t, y, cond_vals=vals, cond_mask=mask)
        e = eps.cpu()
        if ref is None:
            ref = e
        elif not torch.equal(e, ref):
            bad += 1
            diff = (e - ref).abs().flatten(1).amax(1)
            samples |= set(torch.nonzero(diff > 0).flatten().tolist())
print(f"N={N} hw={hw} env={[k + '=' + v for k, v in os.environ.items() if k.startswith('DMX_')]}: "
      f"{bad}/{R - 1} runs differ; samples {sorted(samples)[:12]}")
