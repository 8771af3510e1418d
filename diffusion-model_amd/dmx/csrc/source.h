// dmx — fused input sources: how a convolution's / GEMM's A operand element
// (n, iy, ix, c..c+3) is produced from HBM.  Every mode returns 4 consecutive
// channels (all channel counts on the path are multiples of 4).
#pragma once
#include "common.h"

namespace dmx {

DMX_DEV floatx4 ld4(const float* p) { return *reinterpret_cast<const floatx4*>(p); }

// GroupNorm affine (+ optional GELU) of 4 channels of one pixel.
// Reference: nn.GroupNorm (models/unet_cond.py:20,23; models/vae.py:36-48).
DMX_DEV floatx4 gn_apply4v(floatx4 v, float2 st, floatx4 g, floatx4 b, int act) {
  floatx4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float y = (v[j] - st.x) * st.y * g[j] + b[j];
    o[j] = act ? gelu(y) : y;
  }
  return o;
}
DMX_DEV floatx4 gn_apply4(floatx4 v, float2 st, const float* gamma, const float* beta, int c, int act) {
  return gn_apply4v(v, st, ld4(gamma + c), ld4(beta + c), act);
}

// Bilinear x2, align_corners=True (nn.Upsample, models/unet_cond.py:76) of the
// (Hs, Ws) map `s` sampled at output coordinate (uy, ux); 4 channels at c.
DMX_DEV floatx4 upsample4(const float* s, int n, int Hs, int Ws, int C, int uy, int ux, int c) {
  const int Ho = 2 * Hs, Wo = 2 * Ws;
  const float sh = Ho > 1 ? (float)(Hs - 1) / (float)(Ho - 1) : 0.f;
  const float sw = Wo > 1 ? (float)(Ws - 1) / (float)(Wo - 1) : 0.f;
  const float fy = sh * (float)uy, fx = sw * (float)ux;
  const int y0 = (int)fy, x0 = (int)fx;
  const int y1 = y0 + (y0 < Hs - 1 ? 1 : 0), x1 = x0 + (x0 < Ws - 1 ? 1 : 0);
  const float ly = fminf(fmaxf(fy - (float)y0, 0.f), 1.f), lx = fminf(fmaxf(fx - (float)x0, 0.f), 1.f);
  const float hy = 1.f - ly, hx = 1.f - lx;
  const float* base = s + (size_t)n * Hs * Ws * C + c;
  floatx4 v00 = ld4(base + ((size_t)y0 * Ws + x0) * C), v01 = ld4(base + ((size_t)y0 * Ws + x1) * C);
  floatx4 v10 = ld4(base + ((size_t)y1 * Ws + x0) * C), v11 = ld4(base + ((size_t)y1 * Ws + x1) * C);
  floatx4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = hy * (hx * v00[j] + lx * v01[j]) + ly * (hx * v10[j] + lx * v11[j]);
  return o;
}

// Element (n, iy, ix, c..c+3) of the source on an H x W grid; caller guarantees
// 0 <= iy < H, 0 <= ix < W.
template <int SRC>
DMX_DEV floatx4 load_src4(const SrcDesc& s, int n, int iy, int ix, int c, int H, int W) {
  if constexpr (SRC == SRC_PLAIN) {
    return ld4(s.src0 + (((size_t)n * H + iy) * W + ix) * s.C + c);
  } else if constexpr (SRC == SRC_GNACT) {
    floatx4 v = ld4(s.src0 + (((size_t)n * H + iy) * W + ix) * s.C + c);
    const int g = c / (s.C / s.G);
    return gn_apply4(v, s.stats[n * s.G + g], s.gamma, s.beta, c, s.act);
  } else if constexpr (SRC == SRC_MAXPOOL) {
    const float* b = s.src0 + (((size_t)n * s.Hs + 2 * iy) * s.Ws + 2 * ix) * s.C + c;
    floatx4 a = ld4(b), bb = ld4(b + s.C), cc = ld4(b + (size_t)s.Ws * s.C), d = ld4(b + (size_t)s.Ws * s.C + s.C);
    floatx4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = fmaxf(fmaxf(a[j], bb[j]), fmaxf(cc[j], d[j]));
    return o;
  } else if constexpr (SRC == SRC_UPCAT) {
    if (c < s.C0) {  // skip: sample n % n_mod when it was computed once for both CFG halves
      const int ns = s.n_mod ? n % s.n_mod : n;
      return ld4(s.src0 + (((size_t)ns * H + iy) * W + ix) * s.C0 + c);
    }
    const int uy = iy - s.padT, ux = ix - s.padL;
    if (uy < 0 || ux < 0 || uy >= 2 * s.Hs || ux >= 2 * s.Ws) return floatx4{0.f, 0.f, 0.f, 0.f};
    return upsample4(s.src1, n, s.Hs, s.Ws, s.C - s.C0, uy, ux, c - s.C0);
  } else {  // SRC_NCHW
    floatx4 o;
    const size_t plane = (size_t)H * W;
    const int ns = s.n_mod ? n % s.n_mod : n;
    const int creal = s.C0 ? s.C0 : s.C;  // channels actually present (input padded to a multiple of 4)
    const float* b = s.src0 + ((size_t)ns * creal + c) * plane + (size_t)iy * W + ix;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float v = (c + j < creal) ? b[j * plane] : 0.f;
      o[j] = (s.scale != 1.f) ? v / s.scale : v;
    }
    return o;
  }
}

}  // namespace dmx
