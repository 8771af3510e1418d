"""Python side of the native engine: contexts, weight loading, step / loop / decode.

All arithmetic happens in libdmx.so (HIP kernels for gfx950).  This module only
moves pointers: torch provides device memory and streams.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import threading
from typing import Dict, Optional, Tuple

import torch

from . import _lib
from ._lib import StepArgs, check

TIME_DIM = 256


def pos_table(tmax: int) -> torch.Tensor:
    """pos[t-1] for t = 1..tmax with the reference's exact fp32 formula
    (models/unet_cond.py:155-161: long t repeated, times the fp32 inv_freq, sin|cos)."""
    inv_freq = 1.0 / (10000 ** (torch.arange(0, TIME_DIM, 2).float() / TIME_DIM))
    t = torch.arange(1, tmax + 1, dtype=torch.long).unsqueeze(-1)
    tt = t.repeat(1, TIME_DIM // 2) * inv_freq
    return torch.cat([torch.sin(tt), torch.cos(tt)], dim=-1).contiguous()


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


class Context:
    """One dmx_ctx per device per process."""

    _ctxs: Dict[int, "Context"] = {}
    _lock = threading.Lock()

    def __init__(self, index: int):
        self.lib = _lib.load()
        self.index = index
        h = ctypes.c_void_p()
        check(self.lib.dmx_create(index, ctypes.byref(h)))
        self.handle = h
        self.tmax = 0

    @classmethod
    def get(cls, device: torch.device) -> "Context":
        idx = device.index if device.index is not None else torch.cuda.current_device()
        with cls._lock:
            if idx not in cls._ctxs:
                cls._ctxs[idx] = Context(idx)
            return cls._ctxs[idx]

    def ensure_time_table(self, tmax: int) -> None:
        if tmax <= self.tmax:
            return
        tmax = max(tmax, 1000)
        tab = pos_table(tmax)
        check(self.lib.dmx_set_time_table(self.handle, ctypes.c_void_p(tab.data_ptr()), tmax))
        self.tmax = tmax


def require_cuda(t: torch.Tensor, what: str) -> None:
    if not t.is_cuda:
        raise _lib.DmxUnavailable(
            f"{what} is on {t.device}; the dmx path runs only on an MI355X (HIP) device — move the model and "
            f"inputs with .to('cuda') (there is no CPU fallback)")


class NativeModel:
    """A repacked copy of one reference network inside libdmx (U-Net or VAE)."""

    def __init__(self, kind: int, params: Dict[str, torch.Tensor], in_ch: int = 4, remove_deep_conv: bool = False,
                 **cfg):
        self.kind = kind
        self.in_ch = in_ch
        some = next(iter(params.values()))
        require_cuda(some, "model weights")
        self.device = some.device
        self.ctx = Context.get(self.device)
        self.lib = self.ctx.lib
        h = ctypes.c_void_p()
        conf = _lib.ModelConfig.make(kind, in_ch, remove_deep_conv, **cfg)
        self.geom_dim = int(conf.geom_dim)
        self.keys = _lib.model_keys(kind, in_ch, remove_deep_conv, **cfg)
        check(self.lib.dmx_model_create_cfg(self.ctx.handle, ctypes.byref(conf), ctypes.byref(h)))
        self.handle = h
        keep = []
        for name, t in params.items():
            tt = t.detach().to(dtype=torch.float32).contiguous()
            keep.append(tt)
            shape = (ctypes.c_int64 * max(tt.dim(), 1))(*tt.shape)
            check(self.lib.dmx_model_set_tensor(self.handle, name.encode(), ctypes.c_void_p(tt.data_ptr()), shape,
                                                tt.dim()))
        with torch.cuda.device(self.device):
            check(self.lib.dmx_model_finalize(self.handle, ctypes.c_void_p(_stream(self.device))))
        # the registered tensors (views of the module's fp32 parameters, or converted copies) are
        # re-read by refresh() and the training entry points (include/dmx.h dmx_model_set_tensor)
        self._registered = keep
        self.aliases_params = all(k.data_ptr() == p.data_ptr() for k, p in zip(keep, params.values()))
        self._side_stream = None
        env = os.environ.get("DMX_PRECISION")
        if env:
            self.set_precision(env)

    PRECISIONS = {"fp32": 0, "x3": 1, "f16": 2}

    def set_precision(self, prec) -> None:
        """GEMM arithmetic: "x3" (default; fp32 split into fp16 hi+lo, 3 MFMAs, fp32 accumulate),
        "fp32" (fp32 MFMA, exact fp32 products) or "f16" (BASELINE config 4: GEMM / attention
        operands rounded to fp16, one MFMA, fp32 accumulate; norms, softmax and the scheduler stay fp32)."""
        code = self.PRECISIONS[prec] if isinstance(prec, str) else int(prec)
        check(self.lib.dmx_model_set_precision(self.handle, code))

    def range_tripped(self, reset: bool = True) -> bool:
        """True when an output kernel saw a non-finite value since the last reset (include/dmx.h
        dmx_model_range_check: the split-precision range guard).  Synchronises the current stream."""
        f = ctypes.c_int(0)
        with torch.cuda.device(self.device):
            check(self.lib.dmx_model_range_check(self.handle, int(reset), ctypes.byref(f),
                                                 ctypes.c_void_p(_stream(self.device))))
        return bool(f.value)

    @contextlib.contextmanager
    def precision_override(self, prec):
        old = self.precision
        self.set_precision(prec)
        try:
            yield self
        finally:
            self.set_precision(old)

    @property
    def precision(self) -> str:
        code = self.lib.dmx_model_get_precision(self.handle)
        return {v: k for k, v in self.PRECISIONS.items()}[code]

    def __del__(self):
        try:
            if getattr(self, "handle", None):
                self.lib.dmx_model_destroy(self.handle)
                self.handle = None
        except Exception:
            pass

    def refresh(self) -> None:
        """Parameters changed in place (optimizer.step / load_state_dict): repack on the device."""
        with torch.cuda.device(self.device):
            check(self.lib.dmx_model_refresh(self.handle, ctypes.c_void_p(_stream(self.device))))

    # ---- training (include/dmx.h dmx_train_forward / dmx_train_backward) --------------------
    def train_forward(self, x, t, y, vals=None, mask=None):
        """Forward with a tape for dmx_train_backward -> (eps, geom or None, tape id)."""
        require_cuda(x, "x")
        n, c, h, w = x.shape
        dev = x.device
        self.ctx.ensure_time_table(max(1000, int(t.max().item()) if t.numel() else 1))
        x = x.detach().to(dtype=torch.float32).contiguous()
        t = t.to(device=dev, dtype=torch.long).contiguous()
        y = y.to(device=dev, dtype=torch.long).contiguous()
        if vals is not None:
            vals = vals.detach().to(device=dev, dtype=torch.float32).contiguous()
            mask = mask.detach().to(device=dev, dtype=torch.float32).contiguous()
        eps = torch.empty_like(x)
        geom = (torch.empty((n, self.geom_dim), device=dev, dtype=torch.float32)
                if self.kind == _lib.DMX_UNET_COND_GEOM else None)
        tid = ctypes.c_int64()
        with torch.cuda.device(dev):
            check(self.lib.dmx_train_forward(self.handle, _ptr(x), _ptr(t), _ptr(y), _ptr(vals), _ptr(mask), n, h, w,
                                             _ptr(eps), _ptr(geom), ctypes.byref(tid),
                                             ctypes.c_void_p(_stream(dev))))
        self._live_train = (x, t, y, vals, mask)
        return eps, geom, int(tid.value)

    def train_backward(self, tape_id: int, d_eps=None, d_geom=None) -> Dict[str, torch.Tensor]:
        """dLoss/dparam for every state_dict key, given dLoss/deps and dLoss/dgeom (None = 0)."""
        dev = self.device
        grads = {name: torch.empty(shape, device=dev, dtype=torch.float32) for name, shape in self.keys}
        ptrs = (ctypes.c_void_p * len(self.keys))(*[grads[name].data_ptr() for name, _ in self.keys])
        if d_eps is not None:
            d_eps = d_eps.to(device=dev, dtype=torch.float32).contiguous()
        if d_geom is not None:
            d_geom = d_geom.to(device=dev, dtype=torch.float32).contiguous()
        with torch.cuda.device(dev):
            check(self.lib.dmx_train_backward(self.handle, int(tape_id), _ptr(d_eps), _ptr(d_geom), ptrs,
                                              len(self.keys), ctypes.c_void_p(_stream(dev))))
        self._live_bwd = (d_eps, d_geom)
        return grads

    def workspace_bytes(self) -> int:
        return int(self.lib.dmx_model_workspace_bytes(self.handle))

    # ---- U-Net ---------------------------------------------------------------------------
    def forward(self, x, t, y=None, vals=None, mask=None, want_geom=False):
        n, c, h, w = x.shape
        self.ctx.ensure_time_table(int(t.max().item()) if t.numel() else 1)
        x = x.contiguous().float()
        t = t.to(device=x.device, dtype=torch.long).contiguous()
        if y is not None:
            y = y.to(device=x.device, dtype=torch.long).contiguous()
        if vals is not None:
            vals = vals.to(device=x.device, dtype=torch.float32).contiguous()
            mask = mask.to(device=x.device, dtype=torch.float32).contiguous()
        eps = torch.empty_like(x)
        geom = torch.empty((n, self.geom_dim), device=x.device, dtype=torch.float32) if want_geom else None
        with torch.cuda.device(x.device):
            check(self.lib.dmx_unet_forward(self.handle, _ptr(x), _ptr(t), _ptr(y), _ptr(vals), _ptr(mask),
                                            _ptr(eps), _ptr(geom), n, h, w, ctypes.c_void_p(_stream(x.device))))
        return eps, geom

    def forward_taps(self, x, t, y=None, vals=None, mask=None):
        """Forward with debug taps -> {name: flat float32 tensor (NHWC order)}."""
        check(self.lib.dmx_debug_enable(self.handle, 1))
        try:
            eps, geom = self.forward(x, t, y, vals, mask, want_geom=self.kind == _lib.DMX_UNET_COND_GEOM)
            out = {}
            buf = ctypes.create_string_buffer(128)
            cnt = ctypes.c_int64()
            for i in range(self.lib.dmx_debug_num_taps(self.handle)):
                check(self.lib.dmx_debug_tap(self.handle, i, buf, 128, ctypes.byref(cnt), None, None))
                dst = torch.empty(cnt.value, device=x.device, dtype=torch.float32)
                check(self.lib.dmx_debug_tap(self.handle, i, buf, 128, ctypes.byref(cnt), _ptr(dst),
                                             ctypes.c_void_p(_stream(x.device))))
                out[buf.value.decode()] = dst
            torch.cuda.synchronize(x.device)
            out["eps"] = eps
            return out
        finally:
            check(self.lib.dmx_debug_enable(self.handle, 0))

    def _norm_inputs(self, x_in, t, y, vals, mask, noise):
        """The kernels read raw bytes: t / y as contiguous int64, vals / mask / noise as contiguous fp32,
        all on x's device (a bool cond_mask, float64 values or a column slice are converted here, as the
        reference's torch.cat / arithmetic would promote them).  The converted tensors are kept alive on
        the model until the next call so the enqueued launches never read freed memory."""
        dev = x_in.device
        t = t.to(device=dev, dtype=torch.long).contiguous()
        if y is not None:
            y = y.to(device=dev, dtype=torch.long).contiguous()
        if vals is not None:
            vals = vals.to(device=dev, dtype=torch.float32).contiguous()
        if mask is not None:
            mask = mask.to(device=dev, dtype=torch.float32).contiguous()
        if noise is not None:
            noise = noise.to(device=dev, dtype=torch.float32).contiguous()
        self._live = (t, y, vals, mask, noise)
        return t, y, vals, mask, noise

    def _args(self, x_in, x_out, t, t_stride, y, null_label, vals, mask, guidance, tables, noise, seed,
              sample_offset) -> StepArgs:
        c1, c2, sd = tables
        n, _, h, w = x_in.shape
        a = StepArgs()
        a.x_in, a.x_out = x_in.data_ptr(), x_out.data_ptr()
        a.t, a.t_stride = t.data_ptr(), t_stride
        a.y = y.data_ptr() if y is not None else None
        a.null_label = int(null_label)
        a.vals = vals.data_ptr() if vals is not None else None
        a.mask = mask.data_ptr() if mask is not None else None
        a.guidance = float(guidance)
        a.c1, a.c2, a.sd, a.T = c1.data_ptr(), c2.data_ptr(), sd.data_ptr(), int(c1.numel())
        a.noise = noise.data_ptr() if noise is not None else None
        a.seed, a.sample_offset = int(seed) & 0xFFFFFFFFFFFFFFFF, int(sample_offset)
        a.n, a.h, a.w = n, h, w
        return a

    def step(self, x_in, x_out, t, y, null_label, vals, mask, guidance, tables, noise=None, seed=0,
             sample_offset=0, t_stride=1):
        """One denoising step: CFG (2n batched forward) when guidance > 0 and y given."""
        self.ctx.ensure_time_table(int(tables[0].numel()))
        _check_state(x_in, "x")
        _check_state(x_out, "x_out")
        t, y, vals, mask, noise = self._norm_inputs(x_in, t, y, vals, mask, noise)
        a = self._args(x_in, x_out, t, t_stride, y, null_label, vals, mask, guidance, tables, noise, seed,
                       sample_offset)
        with torch.cuda.device(x_in.device):
            check(self.lib.dmx_step(self.handle, ctypes.byref(a), ctypes.c_void_p(_stream(x_in.device))))

    def step_profile(self, x_in, x_out, t, y, null_label, vals, mask, guidance, tables, noise=None, seed=0,
                     t_stride=1, cap=1024):
        """One eager step with event timing per launch -> list of dicts."""
        self.ctx.ensure_time_table(int(tables[0].numel()))
        t, y, vals, mask, noise = self._norm_inputs(x_in, t, y, vals, mask, noise)
        a = self._args(x_in, x_out, t, t_stride, y, null_label, vals, mask, guidance, tables, noise, seed, 0)
        recs = (_lib.KernelRecord * cap)()
        n = ctypes.c_int()
        with torch.cuda.device(x_in.device):
            check(self.lib.dmx_step_profile(self.handle, ctypes.byref(a), recs, cap, ctypes.byref(n),
                                            ctypes.c_void_p(_stream(x_in.device))))
        return [dict(kernel=r.kernel.decode(), layer=r.layer.decode(), flops=r.flops, bytes=r.bytes, ms=r.ms)
                for r in recs[:n.value]]

    def side_stream(self) -> torch.cuda.Stream:
        if self._side_stream is None:
            self._side_stream = torch.cuda.Stream(self.device)
        return self._side_stream

    def sample_loop(self, x, t_dev, y, null_label, vals, mask, guidance, tables, steps, seed=0, sample_offset=0,
                    use_graph=True):
        """`steps` in-place steps on x with Philox noise; t_dev (device int64 scalar) is
        decremented on the device after each step.  Runs on a side stream (graph capture
        needs a non-default stream) ordered against the current stream."""
        self.ctx.ensure_time_table(int(tables[0].numel()))
        _check_state(x, "x")
        if t_dev.dtype != torch.long or not t_dev.is_contiguous() or t_dev.device != x.device:
            raise ValueError("sample_loop: t_dev must be a contiguous int64 device scalar on x's device "
                             "(it is decremented in place)")
        _, y, vals, mask, _ = self._norm_inputs(x, t_dev, y, vals, mask, None)
        a = self._args(x, x, t_dev, 0, y, null_label, vals, mask, guidance, tables, None, seed, sample_offset)
        cur = torch.cuda.current_stream(x.device)
        side = self.side_stream()
        side.wait_stream(cur)
        for keep in (x, t_dev, y, vals, mask) + tuple(tables):
            if keep is not None:
                keep.record_stream(side)
        with torch.cuda.device(x.device):
            check(self.lib.dmx_sample_loop(self.handle, ctypes.byref(a), int(steps), int(use_graph),
                                           ctypes.c_void_p(side.cuda_stream)))
        cur.wait_stream(side)

    # ---- VAE -----------------------------------------------------------------------------
    def decode(self, z, want_img=True, want_u8=False) -> Tuple[Optional[torch.Tensor], Optional[torch.Tensor]]:
        n, c, h, w = z.shape
        z = z.contiguous().float()
        img = torch.empty((n, 3, 8 * h, 8 * w), device=z.device, dtype=torch.float32) if want_img else None
        u8 = torch.empty((n, 8 * h, 8 * w, 3), device=z.device, dtype=torch.uint8) if want_u8 else None
        with torch.cuda.device(z.device):
            check(self.lib.dmx_vae_decode(self.handle, _ptr(z), _ptr(img), _ptr(u8), n, h, w,
                                          ctypes.c_void_p(_stream(z.device))))
        return img, u8

    def decode_u8_into(self, z, u8) -> None:
        """Decode z (n,4,h,w) straight into a caller-owned uint8 (n,8h,8w,3) HWC buffer."""
        n, c, h, w = z.shape
        zc = z.contiguous().float()
        if u8.dtype != torch.uint8 or not u8.is_contiguous() or tuple(u8.shape) != (n, 8 * h, 8 * w, 3):
            raise ValueError(f"u8 must be a contiguous uint8 tensor of shape {(n, 8 * h, 8 * w, 3)}")
        with torch.cuda.device(zc.device):
            check(self.lib.dmx_vae_decode(self.handle, _ptr(zc), None, _ptr(u8), n, h, w,
                                          ctypes.c_void_p(_stream(zc.device))))
        self._live_dec = zc

    def encode(self, x, eps) -> Tuple[torch.Tensor, torch.Tensor]:
        """x (n,3,h,w), eps (n,4,h/8,w/8) -> (z, per-sample KL (n,)) (models/vae.py:51-62)."""
        n, c, h, w = x.shape
        x = x.contiguous().float()
        eps = eps.contiguous().float()
        z = torch.empty((n, 4, h // 8, w // 8), device=x.device, dtype=torch.float32)
        kl = torch.empty((n,), device=x.device, dtype=torch.float32)
        with torch.cuda.device(x.device):
            check(self.lib.dmx_vae_encode(self.handle, _ptr(x), _ptr(eps), _ptr(z), _ptr(kl), n, h, w,
                                          ctypes.c_void_p(_stream(x.device))))
        return z, kl


def _check_state(x: torch.Tensor, what: str) -> None:
    """The step kernels read / write x as contiguous fp32 NCHW on the device."""
    require_cuda(x, what)
    if x.dtype != torch.float32 or not x.is_contiguous():
        raise ValueError(f"{what} must be a contiguous float32 tensor (got {x.dtype}, contiguous={x.is_contiguous()})")


def ddpm_update(x, eu, ec, guidance, t, tables, noise=None, seed=0, sample_offset=0):
    """Standalone K1 (diff.py:151,158-162) for duck-typed models: returns x'.

    Every converted operand is bound to a local for the duration of the launch (a temporary
    freed right after taking its pointer could be handed to the next conversion by the
    caching allocator)."""
    lib = _lib.load()
    c1, c2, sd = tables
    require_cuda(x, "x")
    dev = x.device
    x_c = x.to(dtype=torch.float32).contiguous()
    n, c, h, w = x_c.shape
    eu_c = eu.to(device=dev, dtype=torch.float32).contiguous()
    ec_c = ec.to(device=dev, dtype=torch.float32).contiguous() if ec is not None else None
    nz_c = noise.to(device=dev, dtype=torch.float32).contiguous() if noise is not None else None
    t_c = t.to(device=dev, dtype=torch.long).contiguous()
    for e, nm in ((eu_c, "eps"), (ec_c, "eps_cond"), (nz_c, "noise")):
        if e is not None and tuple(e.shape) != tuple(x_c.shape):
            raise ValueError(f"{nm} shape {tuple(e.shape)} != x shape {tuple(x_c.shape)}")
    if t_c.numel() != n:
        raise ValueError(f"t has {t_c.numel()} entries for a batch of {n}")
    out = torch.empty_like(x_c)
    with torch.cuda.device(dev):
        check(lib.dmx_ddpm_update(_ptr(x_c), _ptr(out), _ptr(eu_c), _ptr(ec_c), float(guidance), _ptr(t_c),
                                  1, _ptr(c1), _ptr(c2), _ptr(sd), int(c1.numel()), _ptr(nz_c), int(seed),
                                  int(sample_offset), n, c, h, w, ctypes.c_void_p(_stream(dev))))
    return out
