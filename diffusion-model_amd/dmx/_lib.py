"""ctypes binding of libdmx.so (include/dmx.h).

The library is built in-tree (``__graft_entry__.build()`` / ``dmx.build``) and
loaded after ``torch`` so that it binds to the HIP runtime torch already
loaded (both carry SONAME libamdhip64.so.7).  There is no fallback: a missing
or unloadable library raises ``DmxUnavailable``.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# DMX_LIB: an alternative in-tree build (same-box A/B of compiler options); default libdmx.so
LIB_PATH = os.path.join(_HERE, os.environ.get("DMX_LIB", "libdmx.so"))

DMX_UNET_COND_GEOM = 1
DMX_UNET_COND = 2
DMX_UNET = 3
DMX_VAE = 4

DMX_E_ARG = 1
DMX_E_STATE = 2


class DmxUnavailable(RuntimeError):
    """libdmx.so could not be loaded — the MI355X path is mandatory (no CPU fallback)."""


class DmxError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"dmx error {code}: {msg}")
        self.code = code


class StepArgs(ctypes.Structure):
    _fields_ = [
        ("x_in", ctypes.c_void_p), ("x_out", ctypes.c_void_p),
        ("t", ctypes.c_void_p), ("t_stride", ctypes.c_int),
        ("y", ctypes.c_void_p), ("null_label", ctypes.c_int64),
        ("vals", ctypes.c_void_p), ("mask", ctypes.c_void_p),
        ("guidance", ctypes.c_float),
        ("c1", ctypes.c_void_p), ("c2", ctypes.c_void_p), ("sd", ctypes.c_void_p), ("T", ctypes.c_int),
        ("noise", ctypes.c_void_p), ("seed", ctypes.c_uint64), ("sample_offset", ctypes.c_int64),
        ("n", ctypes.c_int), ("h", ctypes.c_int), ("w", ctypes.c_int),
    ]


class ModelConfig(ctypes.Structure):
    """dmx_model_config (include/dmx.h): reference constructor arguments that shape the network."""
    _fields_ = [("kind", ctypes.c_int), ("in_ch", ctypes.c_int), ("remove_deep_conv", ctypes.c_int),
                ("num_classes", ctypes.c_int), ("geom_dim", ctypes.c_int), ("geom_hidden", ctypes.c_int),
                ("scale_factor", ctypes.c_float)]

    @classmethod
    def make(cls, kind: int, in_ch: int = 4, remove_deep_conv: bool = False, num_classes: int = 3,
             geom_dim: int = 12, geom_hidden: int = 256, scale_factor: float = 0.18215) -> "ModelConfig":
        return cls(int(kind), int(in_ch), int(bool(remove_deep_conv)), int(num_classes), int(geom_dim),
                   int(geom_hidden), float(scale_factor))


class KernelRecord(ctypes.Structure):
    _fields_ = [("kernel", ctypes.c_char * 96), ("layer", ctypes.c_char * 48), ("flops", ctypes.c_double),
                ("bytes", ctypes.c_double), ("ms", ctypes.c_float)]


# (name, restype, argtypes) for every symbol declared in include/dmx.h
_P = ctypes.c_void_p
_I = ctypes.c_int
_I64 = ctypes.c_int64
SIGNATURES = [
    ("dmx_abi_version", _I, []),
    ("dmx_last_error", ctypes.c_char_p, []),
    ("dmx_create", _I, [_I, ctypes.POINTER(_P)]),
    ("dmx_destroy", _I, [_P]),
    ("dmx_set_time_table", _I, [_P, _P, _I]),
    ("dmx_model_num_keys", _I, [_I, _I, _I]),
    ("dmx_model_key", _I, [_I, _I, _I, _I, ctypes.c_char_p, _I, ctypes.POINTER(_I64), ctypes.POINTER(_I)]),
    ("dmx_model_create", _I, [_P, _I, _I, _I, ctypes.POINTER(_P)]),
    ("dmx_model_create_cfg", _I, [_P, ctypes.POINTER(ModelConfig), ctypes.POINTER(_P)]),
    ("dmx_model_cfg_num_keys", _I, [ctypes.POINTER(ModelConfig)]),
    ("dmx_model_cfg_key", _I, [ctypes.POINTER(ModelConfig), _I, ctypes.c_char_p, _I, ctypes.POINTER(_I64),
                               ctypes.POINTER(_I)]),
    ("dmx_model_destroy", _I, [_P]),
    ("dmx_model_set_tensor", _I, [_P, ctypes.c_char_p, _P, ctypes.POINTER(_I64), _I]),
    ("dmx_model_finalize", _I, [_P, _P]),
    ("dmx_model_refresh", _I, [_P, _P]),
    ("dmx_train_forward", _I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _P, _P, ctypes.POINTER(_I64), _P]),
    ("dmx_train_backward", _I, [_P, _I64, _P, _P, ctypes.POINTER(_P), _I, _P]),
    ("dmx_model_set_precision", _I, [_P, _I]),
    ("dmx_model_get_precision", _I, [_P]),
    ("dmx_model_range_check", _I, [_P, _I, ctypes.POINTER(_I), _P]),
    ("dmx_unet_forward", _I, [_P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _P]),
    ("dmx_step", _I, [_P, ctypes.POINTER(StepArgs), _P]),
    ("dmx_sample_loop", _I, [_P, ctypes.POINTER(StepArgs), _I, _I, _P]),
    ("dmx_ddpm_update", _I, [_P, _P, _P, _P, ctypes.c_float, _P, _I, _P, _P, _P, _I, _P, ctypes.c_uint64, _I64,
                             _I, _I, _I, _I, _P]),
    ("dmx_vae_decode", _I, [_P, _P, _P, _P, _I, _I, _I, _P]),
    ("dmx_latent_frames_u8", _I, [_P, _P, _I, _I, _I, _I, _P]),
    ("dmx_eval_metrics", _I, [_P, _P, _I, _I, _I, _I, _I, _I, ctypes.c_double, _P, _P, _P]),
    ("dmx_vae_encode", _I, [_P, _P, _P, _P, _P, _I, _I, _I, _P]),
    ("dmx_model_workspace_bytes", _I64, [_P]),
    ("dmx_debug_enable", _I, [_P, _I]),
    ("dmx_debug_num_taps", _I, [_P]),
    ("dmx_debug_tap", _I, [_P, _I, ctypes.c_char_p, _I, ctypes.POINTER(_I64), _P, _P]),
    ("dmx_step_profile", _I, [_P, ctypes.POINTER(StepArgs), ctypes.POINTER(KernelRecord), _I, ctypes.POINTER(_I), _P]),
    ("dmx_attn_core_backward", _I, [_P, _P, _P, _P, _I, _I, _I, _P]),
    ("dmx_diag_wino_stamps", _I, [_P, _I]),
]

_lib = None
_lock = threading.Lock()


def load():
    """Load libdmx.so once (after torch) and attach prototypes."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        import torch  # noqa: F401  (bind to torch's HIP runtime first)
        if not os.path.exists(LIB_PATH):
            raise DmxUnavailable(f"{LIB_PATH} not built — run `python -c 'import __graft_entry__ as g; g.build()'`")
        try:
            lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        except OSError as e:  # pragma: no cover - environment specific
            raise DmxUnavailable(f"cannot load {LIB_PATH}: {e}") from e
        for name, res, args in SIGNATURES:
            if "DMX_LIB" in os.environ and not hasattr(lib, name):
                continue  # an older A/B build may predate a symbol
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def check(rc: int) -> None:
    if rc != 0:
        msg = load().dmx_last_error()
        raise DmxError(rc, msg.decode() if msg else "")


def model_keys(kind: int, in_ch: int = 4, remove_deep_conv: bool = False, **cfg):
    """Reference state_dict keys the native loader expects (no GPU needed); ``cfg`` takes the
    other ModelConfig fields (num_classes, geom_dim, geom_hidden, scale_factor)."""
    lib = load()
    c = ModelConfig.make(kind, in_ch, remove_deep_conv, **cfg)
    n = lib.dmx_model_cfg_num_keys(ctypes.byref(c))
    if n < 0:
        raise DmxError(DMX_E_ARG, lib.dmx_last_error().decode())
    out = []
    buf = ctypes.create_string_buffer(256)
    shape = (ctypes.c_int64 * 4)()
    nd = ctypes.c_int()
    for i in range(n):
        check(lib.dmx_model_cfg_key(ctypes.byref(c), i, buf, 256, shape, ctypes.byref(nd)))
        out.append((buf.value.decode(), tuple(shape[j] for j in range(nd.value))))
    return out
