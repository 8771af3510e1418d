"""Shared base of the drop-in networks: the reference's module tree (models/_modules.py)
backed by a repacked native copy inside libdmx.

The parameter layout (names, shapes, registration order, default initialisation) is
the reference's, so ``load_state_dict`` of a reference checkpoint works unchanged
(reference ``utils.py:68-73``).  ``forward`` never computes on the host: the first
call on a device packs the weights into libdmx (cached until a parameter is moved or
replaced; modified in place — optimizer.step, load_state_dict — it is repacked on the
device by ``NativeModel.refresh``) and every call after that is a native launch.

With autograd recording (grad mode on, trainable parameters) the U-Nets run the native
training forward and backward (``_NativeTrainFn``, include/dmx.h dmx_train_forward /
dmx_train_backward): ``loss.backward()`` of the reference training loop
(train_latent_cond.py:148-162) fills every parameter's ``.grad``.
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
        return (ps[0].device, tuple(p.data_ptr() for p in ps), tuple(sorted(self._dmx_config().items())))

    def native(self) -> "_engine.NativeModel":
        key = self._dmx_key()
        versions = tuple(p._version for p in self.parameters())
        cache = self._dmx_cache
        if cache is not None and cache[0] == key:
            nm = cache[1]
            if cache[2] != versions:
                if not nm.aliases_params:  # converted copies were registered: rebuild
                    cache = None
                else:  # same storage, new values: repack in place on the device
                    nm.refresh()
                    object.__setattr__(self, "_dmx_cache", (key, nm, versions))
            if cache is not None:
                return nm
        self._dmx_check_supported()
        params = {k: v.detach() for k, v in self.named_parameters()}
        nm = _engine.NativeModel(self._dmx_kind, params, in_ch=getattr(self, "_dmx_in_ch", 4),
                                 remove_deep_conv=getattr(self, "remove_deep_conv", False), **self._dmx_config())
        object.__setattr__(self, "_dmx_cache", (key, nm, versions))
        return nm

    def _dmx_training(self) -> bool:
        """Autograd is recording and some parameter is trainable: run the native training step."""
        return torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())

    def _dmx_train_forward(self, x, t, y, vals, mask):
        """(eps, geom) through _NativeTrainFn; geom is None for networks without a GeomHead."""
        for name, v in (("x", x), ("cond_vals", vals), ("cond_mask", mask)):
            if v is not None and v.requires_grad:
                raise NotImplementedError(f"dmx training computes parameter gradients only ({name} requires grad)")
        bad = [n for n, p in self.named_parameters() if p.dtype != torch.float32 or not p.is_contiguous()]
        if bad:
            raise NotImplementedError(f"dmx training needs contiguous fp32 parameters ({bad[0]})")
        names = [n for n, _ in self.named_parameters()]
        eps, geom = _NativeTrainFn.apply(self, names, x, t, y, vals, mask, *self.parameters())
        return eps, (geom if geom.numel() else None)

    def _dmx_config(self) -> dict:
        """Extra dmx_model_config fields (num_classes, geom_dim, geom_hidden, scale_factor)."""
        return {}

    def _dmx_check_supported(self) -> None:
        """Raise for constructor arguments whose network libdmx does not implement."""

    def _apply(self, fn, *args, **kwargs):  # .to()/.cuda() invalidate the native copy
        object.__setattr__(self, "_dmx_cache", None)
        return super()._apply(fn, *args, **kwargs)


class _NativeTrainFn(torch.autograd.Function):
    """Native forward with a tape / native backward of the conditional U-Nets.

    Inputs after (module, names): x, t, y, vals, mask, *parameters (named_parameters order);
    outputs (eps, geom) — geom is an empty tensor for UnetCond.  Gradients flow to the
    parameters only (x, t, y, vals, mask take none, as in train_latent_cond.py:148).  A
    branch that did not run (cond_mlp without cond_vals) gets None, as torch autograd gives."""

    @staticmethod
    def forward(ctx, module, names, x, t, y, vals, mask, *params):
        nm = module.native()
        eps, geom, tape = nm.train_forward(x, t, y, vals, mask)
        ctx.nm, ctx.tape, ctx.names, ctx.cond = nm, tape, names, vals is not None
        ctx.set_materialize_grads(False)
        if geom is None:
            geom = eps.new_empty(0)
            ctx.mark_non_differentiable(geom)
        return eps, geom

    @staticmethod
    def backward(ctx, d_eps, d_geom):
        if d_geom is not None and d_geom.numel() == 0:
            d_geom = None
        grads = ctx.nm.train_backward(ctx.tape, d_eps, d_geom)
        out = []
        for n in ctx.names:  # parameters outside the graph of the used outputs get None, as in torch
            unused = ((not ctx.cond and n.startswith("cond_mlp.")) or (d_geom is None and n.startswith("geom_head."))
                      or (d_eps is None and n.startswith("out.")))
            out.append(None if unused else grads[n])
        return (None, None, None, None, None, None, None, *out)
