"""Batch-composition invariance of the U-Net forward (GPU box): eps of an N-sample batch vs the same
samples run as two halves, bit-wise; prints which samples differ and by how much.
python tools/shard_eq.py [N] [hw]   (DMX_* env knobs select kernel variants for bisection)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "diffusion-model_amd"), REPO]
import torch  # noqa: E402

from dmx import synth  # noqa: E402
from models.unet_cond_geom import UnetCondWithGeomHead  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
hw = int(sys.argv[2]) if len(sys.argv) > 2 else 32
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
with torch.no_grad():
    full, gf = m(x, t, y, cond_vals=vals, cond_mask=mask)
    h = N // 2
    parts = [m(x[s], t[s], y[s], cond_vals=vals[s], cond_mask=mask[s]) for s in (slice(0, h), slice(h, N))]
    half = torch.cat([p[0] for p in parts])
    ghalf = torch.cat([p[1] for p in parts])
d = (full - half).abs().flatten(1).amax(1).cpu()
bad = torch.nonzero(d > 0).flatten().tolist()
rel = float((full - half).norm() / full.norm())
print(f"N={N} vs 2x{h} hw={hw} env={[k + '=' + v for k, v in os.environ.items() if k.startswith('DMX_')]}: "
      f"eps {len(bad)} samples differ (rel {rel:.2e}, first {bad[:8]}); geom equal {torch.equal(gf, ghalf)}")
