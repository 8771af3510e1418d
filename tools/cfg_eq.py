"""Sampler-level shard check (GPU box, one process): ShardedCondSampler world 1 at B vs the same call
with B // 2 (the first half of the batch), device noise; prints the range-guard replays and the
latent difference of the common samples.  python tools/cfg_eq.py [B] [hw] [T]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "diffusion-model_amd"), REPO]
import torch  # noqa: E402

import diff  # noqa: E402
from dmx import distributed as dd  # noqa: E402
from dmx import synth  # noqa: E402
from models.unet_cond_geom import UnetCondWithGeomHead  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
hw = int(sys.argv[2]) if len(sys.argv) > 2 else 32
T = int(sys.argv[3]) if len(sys.argv) > 3 else 8
dev = torch.device("cuda:0")
m = UnetCondWithGeomHead()
m.load_state_dict(synth.unet_cond_geom_weights(0))
m.to(dev).eval()
g = torch.Generator().manual_seed(40)
vals = torch.rand((B, 12), generator=g).to(dev)
mask = (torch.rand((B, 12), generator=g) > 0.3).float().to(dev)
outs = []
for b in (B, B // 2):
    d = diff.Diffuser(T, device=dev)
    d.noise_source = "device"
    torch.manual_seed(41)
    s = dd.ShardedCondSampler(d, m, None)
    lat = s.sample({1: 3, 3: b - 3}, z_shape=(4, hw, hw), cond=vals[:b], cond_mask=mask[:b], decode=False)
    print(f"B={b}: range_fallbacks={s.range_fallbacks} d.range_fallbacks={getattr(d, 'range_fallbacks', None)}")
    outs.append(lat)
h = B // 2
a, c = outs[0][:h], outs[1]
diffs = (a - c).abs().flatten(1).amax(1)
print(f"first {h}: equal={torch.equal(a, c)} rel={float((a - c).norm() / c.norm()):.2e} "
      f"samples differing {int((diffs > 0).sum())} first {torch.nonzero(diffs > 0).flatten().tolist()[:10]}")
