"""One U-Net forward of N samples vs the oracle (GPU box): python tools/fwd_check.py [N] [hw] [prec]
Prints eps / geom rel-L2 — a quick bisection aid for env knobs (DMX_WINO, DMX_WINO_SPLIT, DMX_GN_FUSE)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "diffusion-model_amd"), REPO]
import torch  # noqa: E402

from dmx import synth  # noqa: E402
from oracle import ref  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 128
hw = int(sys.argv[2]) if len(sys.argv) > 2 else 32
prec = sys.argv[3] if len(sys.argv) > 3 else "x3"
from models.unet_cond_geom import UnetCondWithGeomHead  # noqa: E402
sd = synth.unet_cond_geom_weights(0)
m = UnetCondWithGeomHead()
m.load_state_dict(sd)
dev = torch.device("cuda:0")
m.to(dev).eval()
m.native().set_precision(prec)
g = torch.Generator().manual_seed(128)
x = torch.randn((N, 4, hw, hw), generator=g)
t = torch.randint(1, 1001, (N,), generator=g)
y = torch.randint(0, 4, (N,), generator=g)
vals = torch.rand((N, 12), generator=g)
mask = (torch.rand((N, 12), generator=g) > 0.5).float()
with torch.no_grad():
    eps, geom = m(x.to(dev), t.to(dev), y.to(dev), cond_vals=vals.to(dev), cond_mask=mask.to(dev))
    e2, g2 = ref.unet_cond_geom_forward(sd, x, t, y, vals, mask)
r = lambda a, b: float((a.double().cpu() - b.double()).norm() / b.double().norm())
per = [(i, r(eps[i], e2[i])) for i in range(N)]
bad = [i for i, v in per if v > 2e-5]
print(f"N={N} hw={hw} {prec} env={[k + '=' + v for k, v in os.environ.items() if k.startswith('DMX_')]}: "
      f"eps {r(eps, e2):.2e} geom {r(geom, g2):.2e}; samples over 2e-5: {len(bad)} first {bad[:8]}")
