"""why the inference GELU fit (common.h gelu) is kept out of the training forward.

CPU only (oracle/train_ref.py autograd over oracle/ref.py): the bench-shape training gradients of
tests/test_gpu_train.py::test_native_grads_at_bench_shape_vs_oracle (B = 32, 28 x 28, same seed)
computed four ways — float64 / float32, erf GELU / the fit — and compared per tensor against the
float64 erf gradients.  rel(f32 erf) is the fp32 noise floor every native kernel sits on; rel(f64
fit) is the fit's own effect on the gradients, with no rounding in the way.

    python tools/gelu_train_study.py [B] [hw]
"""
import math
import os
import sys

import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "diffusion-model_amd"))

from oracle import train_ref  # noqa: E402
from dmx import synth  # noqa: E402

_ERF_GELU = F.gelu
# the erfc Chebyshev fit of common.h (gelu), evaluated in the input's dtype
_P = [0.17087277, -0.82215223, 1.48851587, -1.13520398, 0.27886807, -0.18628806, 0.09678418, 0.37409196,
      1.00002368, -1.26551223]


def gelu_fit(x, approximate="none"):
    z = x.abs() * (1.0 / math.sqrt(2.0))
    t = 1.0 / (1.0 + 0.5 * z)
    p = torch.full_like(t, _P[0])
    for c in _P[1:]:
        p = p * t + c
    e = t * torch.exp(-z * z + p)
    phi = torch.where(x >= 0, 1.0 - 0.5 * e, 0.5 * e)
    return x * phi


def inputs(B, hw):
    g = torch.Generator().manual_seed(21)
    x = torch.randn((B, 4, hw, hw), generator=g)
    t = torch.randint(1, 1001, (B,), generator=g)
    classes = torch.randint(1, 4, (B,), generator=g)
    drop = torch.rand(B, generator=g) < 0.1
    drop[:2] = True
    y = torch.where(drop, torch.zeros_like(classes), classes)
    keep = (~drop).float().unsqueeze(1)
    vals = torch.rand((B, 12), generator=g) * keep
    mask = (torch.rand((B, 12), generator=g) > 0.3).float() * keep
    noise = torch.randn((B, 4, hw, hw), generator=g)
    gt = torch.rand((B, 12), generator=g)
    return x, t, y, vals, mask, noise, gt


def grads(dtype, fit, B, hw):
    x, t, y, vals, mask, noise, gt = inputs(B, hw)
    sd = {k: v.to(dtype) if v.is_floating_point() else v for k, v in synth.unet_cond_geom_weights(0).items()}
    cast = lambda a: a.to(dtype)
    F.gelu = gelu_fit if fit else _ERF_GELU
    try:
        _, _, _, g = train_ref.loss_and_grads(sd, cast(x), t, y, cast(vals), cast(mask), cast(noise), cast(gt),
                                              cast(mask), 0.5, True, False)
    finally:
        F.gelu = _ERF_GELU
    return {k: v.double() for k, v in g.items() if v is not None}


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    hw = int(sys.argv[2]) if len(sys.argv) > 2 else 28
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    ref = grads(torch.float64, False, B, hw)
    arms = {"f32 erf": (torch.float32, False), "f64 fit": (torch.float64, True), "f32 fit": (torch.float32, True)}
    res = {k: grads(*v, B, hw) for k, v in arms.items()}
    rows = []
    for n, r in ref.items():
        nr = max(float(r.norm()), 1e-300)
        rows.append((n, *[float((res[k][n] - r).norm()) / nr for k in arms]))
    print(f"B={B} hw={hw}: per-tensor rel-L2 vs float64 erf-GELU gradients")
    for i, k in enumerate(arms):
        w = sorted(rows, key=lambda r: -r[1 + i])[:3]
        print(f"  {k:8s} worst: " + ", ".join(f"{row[0]} {row[1 + i]:.2e}" for row in w))
    for n in ("inc.double_conv.0.weight", "outc.weight"):
        row = next((r for r in rows if r[0] == n), None)
        if row:
            print(f"  {n}: " + ", ".join(f"{k} {row[1 + i]:.2e}" for i, k in enumerate(arms)))


if __name__ == "__main__":
    main()
