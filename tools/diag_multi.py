"""Diagnostic: the 2-rank (gloo, one GPU) host-noise sharded sampler run several times; latents per
rank compared across repeats (rel-L2), with and without DMX_POISON (workspace NaN-filled)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "diffusion-model_amd"), REPO, os.path.join(REPO, "tests")):
    sys.path.insert(0, p)
import torch  # noqa: E402

from test_gpu_multi import _job, _run2  # noqa: E402


def rel(a, b):
    return float((a - b).norm() / b.norm())


if __name__ == "__main__":
    single = _job("host", decode=False)
    print("single finite:", bool(torch.isfinite(single).all()), flush=True)
    for rep in range(4):
        r = _run2("host", False)[0]
        print(rep, "sharded rows 0-2 rel:", rel(r[:3], single[:3]), "rows 3-4 rel:", rel(r[3:], single[3:]),
              "finite:", bool(torch.isfinite(r).all()), flush=True)
