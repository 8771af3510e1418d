"""Batch-split consistency probe: one CFG step on B samples vs the same samples split into
shards (as ShardedCondSampler runs them), per precision mode.  Prints rel-L2 per mode."""
import sys

import torch

sys.path.insert(0, "diffusion-model_amd")
import diff  # noqa: E402
from dmx import synth  # noqa: E402
from models.unet_cond_geom import UnetCondWithGeomHead  # noqa: E402

dev = torch.device("cuda:0")
m = UnetCondWithGeomHead()
m.load_state_dict(synth.unet_cond_geom_weights(0))
m.to(dev).eval()
d = diff.Diffuser(4, device=dev)
tables = d.coef_tables(dev, clamp_prev=True)
nm = m.native()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 5
g = torch.Generator().manual_seed(40)
vals = torch.rand((B, 12), generator=g).to(dev)
mask = (torch.rand((B, 12), generator=g) > 0.3).float().to(dev)
y = torch.tensor([1] * 3 + [3] * (B - 3), device=dev)
x = torch.randn((B, 4, 16, 16), generator=g).to(dev)
noise = torch.randn((B, 4, 16, 16), generator=g).to(dev)
splits = [(0, 3), (3, B)]
for prec in ("fp32", "x3"):
    with nm.precision_override(prec):
        for t in (4, 1):
            tt = torch.full((B,), t, dtype=torch.long, device=dev)
            full = torch.empty_like(x)
            nm.step(x, full, tt, y, 0, vals, mask, 3.0, tables, noise)
            parts = []
            for s, e in splits:
                o = torch.empty_like(x[s:e])
                nm.step(x[s:e].contiguous(), o, tt[s:e], y[s:e], 0, vals[s:e].contiguous(), mask[s:e].contiguous(),
                        3.0, tables, noise[s:e].contiguous())
                parts.append(o)
            sp = torch.cat(parts)
            torch.cuda.synchronize()
            rel = float((sp - full).norm() / full.norm())
            per = [float((sp[i] - full[i]).norm() / full[i].norm()) for i in range(B)]
            print(f"[diag] prec={prec} t={t} rel={rel:.3e} per-sample={['%.1e' % v for v in per]}", flush=True)
