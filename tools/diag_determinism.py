"""Diagnostic: is the device-noise sampler (and the U-Net step) bit-deterministic across repeats
and across batch compositions?  Runs in one process on cuda:0."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "diffusion-model_amd"), REPO, os.path.join(REPO, "tests")):
    sys.path.insert(0, p)
import torch  # noqa: E402

from test_gpu_multi import _job  # noqa: E402

for mode in ("device", "host"):
    a = _job(mode, decode=False)
    b = _job(mode, decode=False)
    print(mode, "latents repeat bit-equal:", torch.equal(a, b), "max|d|", float((a - b).abs().max()))
# step determinism at fixed batch
import diff  # noqa: E402
from dmx import synth  # noqa: E402
from models.unet_cond_geom import UnetCondWithGeomHead  # noqa: E402
dev = torch.device("cuda:0")
m = UnetCondWithGeomHead()
m.load_state_dict(synth.unet_cond_geom_weights(0))
m.to(dev).eval()
nm = m.native()
for hw in (16, 32):
    g = torch.Generator().manual_seed(1)
    x = torch.randn((5, 4, hw, hw), generator=g).to(dev)
    t = torch.full((5,), 500, dtype=torch.long, device=dev)
    y = torch.tensor([1, 1, 1, 3, 3], device=dev)
    outs = [nm.forward(x, t, y)[0].clone() for _ in range(3)]
    print(hw, "forward repeat bit-equal:", all(torch.equal(outs[0], o) for o in outs[1:]))
    o3 = nm.forward(x[:3].contiguous(), t[:3], y[:3])[0]
    print(hw, "batch 3 vs 5 rows 0-2 max rel:", float((o3 - outs[0][:3]).norm() / outs[0][:3].norm()))
