"""No kernel reads workspace it did not write: the same inference step (CFG, B = 5 and its 3 + 2
shards) and training forward / backward run in two fresh processes, one with every workspace
filled with 0xFF bytes (fp32 NaN) before use (DMX_POISON=1, engine.hip poison()), one without.
Outputs must be finite and bit-identical: a read of stale memory would turn them NaN (or make
results depend on what a previous model left in reused device memory)."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

WORKER = r'''
import os, sys
import torch
import torch.nn.functional as F
sys.path[:0] = [os.path.join(ROOT, "diffusion-model_amd"), ROOT, os.path.join(ROOT, "tests")]
import diff
from dmx import synth
from models.unet_cond_geom import UnetCondWithGeomHead
dev = torch.device("cuda:0")
m = UnetCondWithGeomHead()
m.load_state_dict(synth.unet_cond_geom_weights(0))
m.to(dev).eval()
d = diff.Diffuser(4, device=dev)
tables = d.coef_tables(dev, clamp_prev=True)
nm = m.native()
g = torch.Generator().manual_seed(40)
B = 5
vals = torch.rand((B, 12), generator=g).to(dev)
mask = (torch.rand((B, 12), generator=g) > 0.3).float().to(dev)
y = torch.tensor([1] * 3 + [3] * (B - 3), device=dev)
out = {}
for hw in (16, 28):
    x = torch.randn((B, 4, hw, hw), generator=g).to(dev)
    noise = torch.randn((B, 4, hw, hw), generator=g).to(dev)
    for prec in ("x3", "fp32"):
        with nm.precision_override(prec):
            tt = torch.full((B,), 4, dtype=torch.long, device=dev)
            for s, e in ((0, B), (0, 3), (3, B)):
                o = torch.empty_like(x[s:e])
                nm.step(x[s:e].contiguous(), o, tt[s:e], y[s:e], 0, vals[s:e].contiguous(), mask[s:e].contiguous(),
                        3.0, tables, noise[s:e].contiguous())
                out[f"step{hw}_{prec}_{s}_{e}"] = o.cpu()
# the benchmark shape (B = 64 CFG, 32 x 32): the large-grid kernels only this batch reaches
# (Winograd F(2x2, 3x3) convs at 16 x 16 / 32 x 32, igemm_wino.h) under the same poison check
Bb = 64
xb = torch.randn((Bb, 4, 32, 32), generator=g).to(dev)
nb = torch.randn((Bb, 4, 32, 32), generator=g).to(dev)
vb = torch.rand((Bb, 12), generator=g).to(dev)
mb = (torch.rand((Bb, 12), generator=g) > 0.3).float().to(dev)
yb = torch.tensor([1 + i % 3 for i in range(Bb)], device=dev)
ob = torch.empty_like(xb)
nm.step(xb, ob, torch.full((Bb,), 3, dtype=torch.long, device=dev), yb, 0, vb, mb, 3.0, tables, nb)
out["step32_b64_x3"] = ob.cpu()
m.train()
x = torch.randn((2, 4, 28, 28), generator=g).to(dev)
t = torch.tensor([17, 900], device=dev)
eps, geom, tape = nm.train_forward(x, t, y[:2], vals[:2], mask[:2])
grads = nm.train_backward(tape, torch.randn(eps.shape, generator=g).to(dev), torch.randn(geom.shape, generator=g).to(dev))
out["train_eps"], out["train_geom"] = eps.cpu(), geom.cpu()
for k, v in grads.items():
    out["grad_" + k] = v.cpu()
torch.cuda.synchronize()
torch.save(out, sys.argv[1])
print("[poison-worker] ok", flush=True)
'''


def _run(tmp_path, tag, worker=WORKER, **env_over):
    path = str(tmp_path / f"out_{tag}.pt")
    env = dict(os.environ, **env_over)
    for k in ("DMX_POISON", "DMX_CHECK", "DMX_PRECISION"):
        if k not in env_over:
            env.pop(k, None)
    r = subprocess.run([sys.executable, "-c", f"ROOT = {ROOT!r}\n" + worker, path], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return torch.load(path, weights_only=True)


def test_no_reads_of_unwritten_workspace(cuda, tmp_path):
    clean = _run(tmp_path, "clean")
    poisoned = _run(tmp_path, "poison", DMX_POISON="1")
    bad = [k for k in clean if not torch.isfinite(poisoned[k]).all() or not torch.equal(clean[k], poisoned[k])]
    assert bad == [], bad[:10]
    # DMX_CHECK=1 (operand-range and plan/run allocation checks before every GEMM launch) raises on
    # nothing and changes nothing
    checked = _run(tmp_path, "check", DMX_CHECK="1")
    bad = [k for k in clean if not torch.equal(clean[k], checked[k])]
    assert bad == [], bad[:10]
    # shard consistency (same process, same kernels): B = 5 equals its 3 + 2 shards
    for hw in (16, 28):
        for prec in ("x3", "fp32"):
            full = clean[f"step{hw}_{prec}_0_5"]
            parts = torch.cat([clean[f"step{hw}_{prec}_0_3"], clean[f"step{hw}_{prec}_3_5"]])
            assert torch.equal(full, parts), (hw, prec, float((full - parts).abs().max()))


PREC_WORKER = r'''
import os, sys
import torch
sys.path[:0] = [os.path.join(ROOT, "diffusion-model_amd"), ROOT, os.path.join(ROOT, "tests")]
import diff
from dmx import synth
from models.unet_cond_geom import UnetCondWithGeomHead
dev = torch.device("cuda:0")
m = UnetCondWithGeomHead()
m.load_state_dict(synth.unet_cond_geom_weights(0))
m.to(dev).eval()
d = diff.Diffuser(4, device=dev)
tables = d.coef_tables(dev, clamp_prev=True)
nm = m.native()
g = torch.Generator().manual_seed(41)
B = 3
x = torch.randn((B, 4, 16, 16), generator=g).to(dev)
noise = torch.randn((B, 4, 16, 16), generator=g).to(dev)
vals = torch.rand((B, 12), generator=g).to(dev)
mask = (torch.rand((B, 12), generator=g) > 0.3).float().to(dev)
y = torch.tensor([1, 2, 3], device=dev)
tt = torch.full((B,), 4, dtype=torch.long, device=dev)
out = {"prec": torch.tensor(["fp32", "x3", "f16"].index(nm.precision))}
o = torch.empty_like(x)
nm.step(x, o, tt, y, 0, vals, mask, 3.0, tables, noise)
out["default"] = o.cpu()
for p in ("fp32", "x3", "f16"):
    with nm.precision_override(p):
        o = torch.empty_like(x)
        nm.step(x, o, tt, y, 0, vals, mask, 3.0, tables, noise)
        out[p] = o.cpu()
torch.cuda.synchronize()
torch.save(out, sys.argv[1])
'''


@pytest.mark.parametrize("prec", ["fp32", "x3", "f16"])
def test_precision_env_selects_the_default_mode(cuda, tmp_path, prec):
    """DMX_PRECISION sets the precision new native models start in: the default
    step equals the explicitly selected mode's step bit for bit."""
    r = _run(tmp_path, "prec_" + prec, PREC_WORKER, DMX_PRECISION=prec)
    assert int(r["prec"]) == ["fp32", "x3", "f16"].index(prec)
    assert torch.equal(r["default"], r[prec])
    assert not torch.equal(r["fp32"], r["f16"])  # (the modes do differ)
