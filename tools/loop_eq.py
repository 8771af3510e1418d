"""Sharded-sampler invariance in one process (GPU box): ShardedCondSampler as rank 0 of a world of 2
(world / broadcast / gather patched to local no-ops) vs world 1, device noise, no decode; compares
rank 0's latents with the first half of the single run bit-wise.
python tools/loop_eq.py [B] [hw] [T]   (DMX_* env knobs select kernel variants for bisection)"""
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


def run(ws):
    dd.world = lambda: (ws, 0)
    dd.any_rank = lambda t, dev: bool(t)
    dd.gather_rows = lambda x, n: x
    dd.dist.broadcast = lambda *a, **k: None
    dd.dist.get_backend = lambda *a, **k: "gloo"
    d = diff.Diffuser(T, device=dev)
    d.noise_source = "device"
    d.use_graph = os.environ.get("LOOP_GRAPH", "1") != "0"
    torch.manual_seed(41)
    return dd.ShardedCondSampler(d, m, None).sample({1: 3, 3: B - 3}, z_shape=(4, hw, hw), cond=vals,
                                                   cond_mask=mask, decode=False)


single, r0 = run(1), run(2)
h = r0.shape[0]
a = single[:h]
dif = (a - r0).abs().flatten(1).amax(1)
print(f"B={B} hw={hw} T={T} env={[k + '=' + v for k, v in os.environ.items() if k.startswith('DMX_') or k == 'LOOP_GRAPH']}: "
      f"rank0 rows {h} equal={torch.equal(a, r0)} rel={float((a - r0).norm() / a.norm()):.2e} "
      f"samples differing {int((dif > 0).sum())} first {torch.nonzero(dif > 0).flatten().tolist()[:10]}")
