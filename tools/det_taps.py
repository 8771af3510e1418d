"""Layer-level determinism (GPU box): R debug-tap forwards of one N-sample batch in one process;
for each run that differs from the first, the first tap (layer output, in execution order) that
differs and how many samples it touches.  Debug taps run the unfused kernel sequence (no
GroupNorm-on-load, no split-K reduce fusion), so this localises races in the kernels that sequence
uses.  python tools/det_taps.py [N] [hw] [R]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "diffusion-model_amd"), REPO]
import torch  # noqa: E402

from dmx import synth  # noqa: E402
from models.unet_cond_geom import UnetCondWithGeomHead  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 128
hw = int(sys.argv[2]) if len(sys.argv) > 2 else 32
R = int(sys.argv[3]) if len(sys.argv) > 3 else 10
m = UnetCondWithGeomHead()
m.load_state_dict(synth.unet_cond_geom_weights(0))
dev = torch.device("cuda:0")
m.to(dev).eval()
nat = m.native()
g = torch.Generator().manual_seed(128)
x = torch.randn((N, 4, hw, hw), generator=g).to(dev)
t = torch.randint(1, 1001, (N,), generator=g).to(dev)
y = torch.randint(0, 4, (N,), generator=g).to(dev)
vals = torch.rand((N, 12), generator=g).to(dev)
mask = (torch.rand((N, 12), generator=g) > 0.5).float().to(dev)
ref = None
first = {}
with torch.no_grad():
    for r in range(R):
        taps = {k: v.cpu() for k, v in nat.forward_taps(x, t, y, vals, mask).items()}
        if ref is None:
            ref = taps
            continue
        for k, v in taps.items():
            if not torch.equal(v, ref[k]):
                nd = int((v != ref[k]).sum())
                first[k] = first.get(k, 0) + 1
                print(f"run {r}: first differing tap {k} ({nd} values)", flush=True)
                break
print(f"N={N} hw={hw}: {sum(first.values())}/{R - 1} runs differ; first taps {first}; taps {len(ref)}")
