"""Shared base of the drop-in networks: the reference's module tree (models/_modules.py)
backed by a repacked native copy inside libdmx.

The parameter layout (names, shapes, registration order, default initialisation) is
the reference's, so ``load_state_dict`` of a reference checkpoint works unchanged
(reference ``utils.py:68-73``).  ``forward`` never computes on the host: the first
call on a device packs the weights into libdmx (cached until a parameter is modified
or moved) and every call after that is a native launch.
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


class NativeBacked(nn.Module):
    """nn.Module whose compute lives in libdmx."""

    _dmx_kind = 0

    def __init__(self):
        super().__init__()
        object.__setattr__(self, "_dmx_cache", None)

    def _dmx_key(self):
        ps = [p for _, p in self.named_parameters()]
        return (ps[0].device, tuple((p.data_ptr(), p._version) for p in ps), tuple(sorted(self._dmx_config().items())))

    def native(self) -> "_engine.NativeModel":
        key = self._dmx_key()
        cache = self._dmx_cache
        if cache is not None and cache[0] == key:
            return cache[1]
        self._dmx_check_supported()
        params = {k: v.detach() for k, v in self.named_parameters()}
        nm = _engine.NativeModel(self._dmx_kind, params, in_ch=getattr(self, "_dmx_in_ch", 4),
                                 remove_deep_conv=getattr(self, "remove_deep_conv", False), **self._dmx_config())
        object.__setattr__(self, "_dmx_cache", (key, nm))
        return nm

    def _dmx_config(self) -> dict:
        """Extra dmx_model_config fields (num_classes, geom_dim, geom_hidden, scale_factor)."""
        return {}

    def _dmx_check_supported(self) -> None:
        """Raise for constructor arguments whose network libdmx does not implement."""

    def _apply(self, fn, *args, **kwargs):  # .to()/.cuda() invalidate the native copy
        object.__setattr__(self, "_dmx_cache", None)
        return super()._apply(fn, *args, **kwargs)
