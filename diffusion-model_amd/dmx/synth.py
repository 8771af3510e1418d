"""Deterministic synthetic weights with the reference's exact state_dict keys.

The reference ships no checkpoints (``.gitignore:2-8`` ignores ``vae/`` and
``result/``), so parity fixtures, tests and the benchmark all run on seeded
synthetic weights.  Every tensor is drawn from its own numpy PCG64 stream
keyed by ``(seed, crc32(name))`` so a tensor's values do not depend on the
order in which keys are visited; the GPU box regenerates identical weights
from the seed (numpy's PCG64 and ``Generator.random`` are platform stable).

Distributions mimic PyTorch's default initialisers (kaiming-uniform with
a=sqrt(5) => U(+-1/sqrt(fan_in)); Embedding N(0,1); MHA xavier) but norm
affine parameters and MHA biases are perturbed away from 1/0 so that the
kernels' affine paths are exercised.
"""
from __future__ import annotations

import hashlib
import zlib
from collections import OrderedDict
from typing import Dict

import numpy as np

from . import spec as _spec


def _draw(seed: int, name: str, shape, kind: str, fan_in: int) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(np.random.SeedSequence([int(seed), zlib.crc32(name.encode())])))
    n = int(np.prod(shape)) if len(shape) else 1
    if kind in (_spec.KIND_CONV_W, _spec.KIND_BIAS, _spec.KIND_CONVT_W):
        bound = 1.0 / np.sqrt(max(fan_in, 1))
        v = (rng.random(n) * 2.0 - 1.0) * bound
    elif kind == _spec.KIND_NORM_W:
        v = 1.0 + (rng.random(n) * 2.0 - 1.0) * 0.1
    elif kind == _spec.KIND_NORM_B:
        v = (rng.random(n) * 2.0 - 1.0) * 0.1
    elif kind == _spec.KIND_EMBED:
        v = rng.standard_normal(n)
    elif kind == _spec.KIND_XAVIER:
        fan_out, fan_in_x = shape[0] // 3, shape[1]
        bound = np.sqrt(6.0 / (fan_in_x + fan_out))
        v = (rng.random(n) * 2.0 - 1.0) * bound
    else:  # pragma: no cover - spec bug
        raise ValueError(f"unknown param kind {kind!r} for {name}")
    return v.astype(np.float32).reshape(shape)


def make_state_dict(param_spec: "_spec.ParamSpec", seed: int) -> "OrderedDict[str, np.ndarray]":
    """Return name -> float32 ndarray for every key of ``param_spec``."""
    out = OrderedDict()
    for name, (shape, kind, fan_in) in param_spec.items():
        out[name] = _draw(seed, name, shape, kind, fan_in)
    return out


def make_torch_state_dict(param_spec, seed: int):
    import torch
    return OrderedDict((k, torch.from_numpy(v)) for k, v in make_state_dict(param_spec, seed).items())


def state_dict_sha256(sd: Dict[str, np.ndarray]) -> str:
    """SHA-256 over (name, shape, bytes) of every tensor in key order."""
    h = hashlib.sha256()
    for k, v in sd.items():
        a = np.ascontiguousarray(np.asarray(v, dtype=np.float32))
        h.update(k.encode())
        h.update(str(a.shape).encode())
        h.update(a.tobytes())
    return h.hexdigest()


def unet_cond_geom_weights(seed: int = 0, **kw):
    return make_torch_state_dict(_spec.unet_cond_geom_spec(**kw), seed)


def unet_weights(seed: int = 0, **kw):
    return make_torch_state_dict(_spec.unet_spec(**kw), seed)


def vae_weights(seed: int = 0, **kw):
    return make_torch_state_dict(_spec.vae_spec(**kw), seed)
