"""Determinism of the native CFG step (GPU box): R identical dmx_step calls (host noise given) on an
S-sample batch (CFG forward of 2S), outputs compared bit-wise with the first; then the same for the
plain forward at 2S.  Run two at once to add contention.  python tools/step_det.py [S] [hw] [R]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "diffusion-model_amd"), REPO]
import torch  # noqa: E402

import diff  # noqa: E402
from dmx import synth  # noqa: E402
from models.unet_cond_geom import UnetCondWithGeomHead  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 64
hw = int(sys.argv[2]) if len(sys.argv) > 2 else 32
R = int(sys.argv[3]) if len(sys.argv) > 3 else 10
dev = torch.device("cuda:0")
m = UnetCondWithGeomHead()
m.load_state_dict(synth.unet_cond_geom_weights(0))
m.to(dev).eval()
nm = m.native()
d = diff.Diffuser(1000, device=dev)
tables = d.coef_tables(dev, clamp_prev=True)
g = torch.Generator().manual_seed(7)
x = torch.randn((S, 4, hw, hw), generator=g).to(dev)
noise = torch.randn((S, 4, hw, hw), generator=g).to(dev)
t = torch.randint(1, 1001, (S,), generator=g).to(dev)
y = torch.randint(1, 4, (S,), generator=g).to(dev)
vals = torch.rand((S, 12), generator=g).to(dev)
mask = (torch.rand((S, 12), generator=g) > 0.3).float().to(dev)
ref, bad, samp = None, 0, set()
with torch.no_grad():
    for r in range(R):
        out = torch.empty_like(x)
        nm.step(x, out, t, y, 0, vals, mask, 3.0, tables, noise)
        o = out.cpu()
        if ref is None:
            ref = o
        elif not torch.equal(o, ref):
            bad += 1
            samp |= set(torch.nonzero((o - ref).abs().flatten(1).amax(1) > 0).flatten().tolist())
print(f"step S={S} hw={hw}: {bad}/{R - 1} runs differ; samples {sorted(samp)[:12]}", flush=True)
x2 = torch.cat([x, x])
t2, y2 = torch.cat([t, t]), torch.cat([y, torch.zeros_like(y)])
v2, m2 = torch.cat([vals, torch.zeros_like(vals)]), torch.cat([mask, torch.zeros_like(mask)])
ref, bad, samp = None, 0, set()
with torch.no_grad():
    for r in range(R):
        e = m(x2, t2, y2, cond_vals=v2, cond_mask=m2)[0].cpu()
        if ref is None:
            ref = e
        elif not torch.equal(e, ref):
            bad += 1
            samp |= set(torch.nonzero((e - ref).abs().flatten(1).amax(1) > 0).flatten().tolist())
print(f"forward N={2 * S} hw={hw}: {bad}/{R - 1} runs differ; samples {sorted(samp)[:12]}", flush=True)
