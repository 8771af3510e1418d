"""Diagnostic: CFG step throughput at B=64 as one batch on one stream vs two B=32 halves on two
native model instances (own workspaces / graphs / side streams) running concurrently."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "diffusion-model_amd"), REPO):
    sys.path.insert(0, p)
import torch  # noqa: E402

import bench  # noqa: E402
import diff  # noqa: E402
from dmx import synth  # noqa: E402
from models.unet_cond_geom import UnetCondWithGeomHead  # noqa: E402

dev = torch.device("cuda:0")
B, K = 64, 60
m1 = UnetCondWithGeomHead()
m1.load_state_dict(synth.unet_cond_geom_weights(0))
m1.to(dev).eval()
m2 = UnetCondWithGeomHead()
m2.load_state_dict(synth.unet_cond_geom_weights(0))
m2.to(dev).eval()
n1, n2 = m1.native(), m2.native()
d = diff.Diffuser(1000, device=dev)
tables = d.coef_tables(dev, True)
x, y, vals, mask = bench.make_inputs(B, 32, dev)


def one(steps):
    t = torch.full((1,), 1000, dtype=torch.long, device=dev)
    n1.sample_loop(x, t, y, 0, vals, mask, 3.0, tables, steps, seed=1)


h = B // 2
xa, xb = x[:h].clone(), x[h:].clone()


sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
ya, yb, va, vb, ma, mb = y[:h].clone(), y[h:].clone(), vals[:h].clone(), vals[h:].clone(), mask[:h].clone(), mask[h:].clone()


def two(steps):
    ta = torch.full((1,), 1000, dtype=torch.long, device=dev)
    tb = torch.full((1,), 1000, dtype=torch.long, device=dev)
    cur = torch.cuda.current_stream(dev)
    sa.wait_stream(cur)
    sb.wait_stream(cur)
    with torch.cuda.stream(sa):
        n1.sample_loop(xa, ta, ya, 0, va, ma, 3.0, tables, steps, seed=1, sample_offset=0)
    with torch.cuda.stream(sb):
        n2.sample_loop(xb, tb, yb, 0, vb, mb, 3.0, tables, steps, seed=1, sample_offset=h)
    cur.wait_stream(sa)
    cur.wait_stream(sb)


for name, f in (("one", one), ("two", two), ("one", one), ("two", two)):
    f(3)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    f(K)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"{name}: {K / dt:.1f} CFG batch-steps/s (B={B})", flush=True)
