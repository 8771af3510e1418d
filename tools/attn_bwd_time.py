"""Event-timed dmx_attn_core_backward at the training shapes (B = 32, 28x28 latents: sa6 L = 784 C = 64,
sa1/sa5 L = 196, sa2/sa4 L = 49, sa3 L = 9), ms per call (MI355X only)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "diffusion-model_amd"))
from dmx import _lib  # noqa: E402

lib = _lib.load()
dev = torch.device("cuda:0")
for C, L in [(64, 784), (64, 196), (128, 196), (128, 49), (256, 49), (256, 9)]:
    n = 32
    qkv = torch.randn((n, L, 3 * C), device=dev)
    o = torch.randn((n, L, C), device=dev)
    dout = torch.randn((n, L, C), device=dev)
    dqkv = torch.empty_like(qkv)
    s = torch.cuda.current_stream()
    args = [ctypes.c_void_p(t.data_ptr()) for t in (qkv, o, dout, dqkv)] + [n, L, C, ctypes.c_void_p(s.cuda_stream)]
    for _ in range(3):
        _lib.check(lib.dmx_attn_core_backward(*args))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        lib.dmx_attn_core_backward(*args)
    e1.record()
    torch.cuda.synchronize()
    print(f"C={C} L={L}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us per call", flush=True)
