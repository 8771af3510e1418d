"""Shared base of the drop-in networks: a parameter tree with the reference's
state_dict names, backed by a repacked native copy inside libdmx.

The parameter layout (names, shapes, registration order) follows dmx.spec, so
``load_state_dict`` of a reference checkpoint works unchanged
(reference ``utils.py:68-73``).  ``forward`` never computes on the host: the
first call on a device packs the weights into libdmx (cached until a parameter
is modified or moved) and every call after that is a native launch.
"""
from __future__ import annotations

import os
import sys

import torch
from torch import nn

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)

from dmx import engine as _engine  # noqa: E402
from dmx import synth as _synth  # noqa: E402


def build_param_tree(module: nn.Module, param_spec, seed: int = 0) -> None:
    """Register every spec entry as an nn.Parameter under its dotted name,
    initialised with the deterministic synthetic generator (dmx.synth)."""
    values = _synth.make_state_dict(param_spec, seed)
    for name, arr in values.items():
        parts = name.split(".")
        m = module
        for p in parts[:-1]:
            if p not in m._modules:
                m.add_module(p, nn.Module())
            m = m._modules[p]
        m.register_parameter(parts[-1], nn.Parameter(torch.from_numpy(arr.copy())))


class NativeBacked(nn.Module):
    """nn.Module whose compute lives in libdmx."""

    _dmx_kind = 0

    def __init__(self):
        super().__init__()
        object.__setattr__(self, "_dmx_cache", None)

    def _dmx_key(self):
        ps = [p for _, p in self.named_parameters()]
        return (ps[0].device, tuple((p.data_ptr(), p._version) for p in ps))

    def native(self) -> "_engine.NativeModel":
        key = self._dmx_key()
        cache = self._dmx_cache
        if cache is not None and cache[0] == key:
            return cache[1]
        params = {k: v.detach() for k, v in self.named_parameters()}
        nm = _engine.NativeModel(self._dmx_kind, params, in_ch=getattr(self, "_dmx_in_ch", 4),
                                 remove_deep_conv=getattr(self, "remove_deep_conv", False))
        object.__setattr__(self, "_dmx_cache", (key, nm))
        return nm

    def _apply(self, fn, *args, **kwargs):  # .to()/.cuda() invalidate the native copy
        object.__setattr__(self, "_dmx_cache", None)
        return super()._apply(fn, *args, **kwargs)
