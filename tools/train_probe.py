"""Training-step probe: forward, sync, backward, sync on the golden case, printing each phase
(run with AMD_SERIALIZE_KERNEL=3 to attribute an asynchronous device error to its launch)."""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "diffusion-model_amd"), ROOT, os.path.join(ROOT, "tests")]
from test_train_oracle import case_inputs, case_weights  # noqa: E402
from models.unet_cond_geom import UnetCondWithGeomHead  # noqa: E402

dev = torch.device("cuda:0")
sd, _, _ = case_weights("g")
m = UnetCondWithGeomHead()
m.load_state_dict(sd)
m.to(dev).train()
x, t, y, vals, mask, noise, gt = (v.to(dev) if v is not None else None for v in case_inputs("g"))
nm = m.native()
torch.cuda.synchronize()
print("[probe] native built", flush=True)
eps, geom, tape = nm.train_forward(x, t, y, vals, mask)
torch.cuda.synchronize()
print("[probe] forward ok", float(eps.abs().mean()), float(geom.abs().mean()), flush=True)
d_eps = torch.randn_like(eps)
d_geom = torch.randn_like(geom)
grads = nm.train_backward(tape, d_eps, d_geom)
torch.cuda.synchronize()
print("[probe] backward ok", sum(float(g.abs().sum()) for g in grads.values()), flush=True)
