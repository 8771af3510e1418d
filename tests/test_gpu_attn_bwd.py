"""dmx_attn_core_backward (the training backward's attention-core adjoint, train.h
attn_dq_mfma_kernel / attn_dkv_mfma_kernel on the fp32 matrix cores) against torch autograd of
softmax(Q K^T / sqrt(D)) V in float64 — the core of nn.MultiheadAttention with 4 heads
(models/unet_cond.py:36,49).  Lengths: the training shapes (28x28 latents: 784, 196, 49, 9 tokens),
ragged lengths around the 16 / 64 tiles, and 1.  Tolerance: fp32 products with fp32 accumulation in
a different order than the float64 reference — relative L2 <= 2e-6 per gradient block."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(qkv, dout, C):
    n, L, _ = qkv.shape
    D = C // 4
    x = qkv.double().detach().requires_grad_(True)
    q, k, v = x.split(C, dim=2)
    hs = lambda t: t.reshape(n, L, 4, D).transpose(1, 2)  # noqa: E731
    p = torch.softmax(hs(q) @ hs(k).transpose(-1, -2) / D ** 0.5, dim=-1)
    o = (p @ hs(v)).transpose(1, 2).reshape(n, L, C)
    o.backward(dout.double())
    return o.float(), x.grad


def _native(qkv, o, dout, C):
    from dmx import _lib
    lib = _lib.load()
    n, L, _ = qkv.shape
    dqkv = torch.full_like(qkv, float("nan"))
    _lib.check(lib.dmx_attn_core_backward(ctypes.c_void_p(qkv.data_ptr()), ctypes.c_void_p(o.data_ptr()),
                                          ctypes.c_void_p(dout.data_ptr()), ctypes.c_void_p(dqkv.data_ptr()), n, L, C,
                                          ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
    torch.cuda.synchronize()
    return dqkv


@pytest.mark.parametrize("C,L", [(64, 784), (64, 196), (128, 196), (128, 49), (256, 49), (256, 9),
                                 (64, 100), (128, 65), (256, 17), (64, 1), (256, 64)])
def test_attn_core_backward_vs_autograd(cuda, C, L):
    g = torch.Generator().manual_seed(C * 1000 + L)
    n = 3
    qkv = (torch.randn((n, L, 3 * C), generator=g) * 1.5).to(cuda)
    dout = (torch.randn((n, L, C), generator=g) * 1e-3).to(cuda)  # gradient-sized
    o, ref = _ref(qkv, dout, C)
    got = _native(qkv, o.contiguous(), dout, C)
    assert torch.isfinite(got).all()
    vnorm = float(ref[..., 2 * C:].norm())
    for part in range(3):
        a, b = got[..., part * C:(part + 1) * C].double(), ref[..., part * C:(part + 1) * C]
        # (L = 1: softmax is constant, dQ = dK = 0 exactly — rounding residue measured against dV there)
        rel = float((a - b).norm() / max(float(b.norm()), vnorm))
        assert rel <= 2e-6, ("qkv"[part], rel)


def test_attn_core_backward_deterministic(cuda):
    g = torch.Generator().manual_seed(4)
    qkv = torch.randn((4, 196, 3 * 64), generator=g).to(cuda)
    dout = torch.randn((4, 196, 64), generator=g).to(cuda)
    o, _ = _ref(qkv, dout, 64)
    o = o.contiguous()
    assert torch.equal(_native(qkv, o, dout, 64), _native(qkv, o, dout, 64))
