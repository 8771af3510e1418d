// dmx — non-GEMM device kernels of the CFG denoising step and the VAE decoder.
#pragma once
#include "common.h"
#include "source.h"

namespace dmx {

// ---------------------------------------------------------------------------
// Wave / block reductions (wave64)
// ---------------------------------------------------------------------------
DMX_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---------------------------------------------------------------------------
// K2 embed: emb = pos(t) + class_emb[y] (+ cond_mlp([vals, mask])), then all six
// per-block heads SiLU -> Linear(256 -> C_i) concatenated into one row.
// Reference: models/unet_cond.py:155-167 (pos/class), 125-129 (cond_mlp),
// 62-65/82-85 (emb_layer), models/unet_cond_geom.py:89-95, models/unet.py:167-170.
// pos_table[t-1][k] is computed on the host by torch (bit-exact with the
// reference's fp32 sin/cos); one 256-thread block per sample.
// ---------------------------------------------------------------------------
struct EmbedParams {
  const int64_t* t; int t_stride; int tmax;
  int t_mod;                   // CFG batching: sample n reads t[n % t_mod] (0 => t[n])
  const int64_t* y;            // null => no class embedding (unconditional Unet)
  int y_null_first;            // CFG batching: samples [0, n_half) use y = y_null
  int64_t y_null; int n_half;
  const float* vals; const float* mask;  // (n_half or n, 12) or null
  int cond_rows;               // rows of vals/mask (n or n_half => row = n % n_half)
  const float* pos_table;      // [tmax][256]
  const float* class_emb;      // [ncls][256]
  int ncls;
  const float* w0; const float* b0;   // cond_mlp.0: [256][24]
  const float* w2t; const float* b2;  // cond_mlp.2 transposed: [256 in][256 out]
  const float* wht; const float* bh;  // heads transposed: [256][Hsum]
  int hsum;
  float* out;                  // [n][hsum]
  int64_t* t_next;             // sample-loop graphs (scalar t): block (0, 0) stores t - 1 here
  const float* cnd;            // [cond_rows][256] cond_mlp outputs (cond_emb_kernel), or null: inline
};

// cond_mlp([vals, mask]) (models/unet_cond.py:125-129, 187-190) once per DISTINCT condition row: the
// CFG halves and every step of a sample loop share it (t-independent), so embed_kernel's blocks
// (N samples x head slices) read it instead of each recomputing the 256 x 256 product.  Same
// arithmetic and summation order as the inline path: the sums are bit-identical.
static __global__ __launch_bounds__(256) void cond_emb_kernel(const EmbedParams p, float* cnd) {
  __shared__ float h[256], in24[24];
  const int row = blockIdx.x, k = threadIdx.x;
  if (k < 12) in24[k] = p.vals[row * 12 + k];
  else if (k < 24) in24[k] = p.mask[row * 12 + (k - 12)];
  __syncthreads();
  float a = p.b0[k];
#pragma unroll
  for (int j = 0; j < 24; ++j) a += p.w0[k * 24 + j] * in24[j];
  h[k] = silu(a);
  __syncthreads();
  float c0 = 0.f, c1 = 0.f, c2 = 0.f, c3 = 0.f;
#pragma unroll
  for (int j = 0; j < 256; j += 4) {
    c0 += p.w2t[(j + 0) * 256 + k] * h[j + 0];
    c1 += p.w2t[(j + 1) * 256 + k] * h[j + 1];
    c2 += p.w2t[(j + 2) * 256 + k] * h[j + 2];
    c3 += p.w2t[(j + 3) * 256 + k] * h[j + 3];
  }
  cnd[row * 256 + k] = p.b2[k] + ((c0 + c1) + (c2 + c3));
}

// grid = (n, parts): every block recomputes the sample's 256-wide embedding (cheap) and
// produces its 1/parts slice of the concatenated head outputs (coalesced weight reads).
static __global__ __launch_bounds__(256) void embed_kernel(const EmbedParams p) {
  __shared__ float s[256], h[256], in24[24];
  const int n = blockIdx.x, k = threadIdx.x;
  int64_t t = p.t[(size_t)(p.t_mod ? n % p.t_mod : n) * p.t_stride];
  // the next step's t in the other buffer of a multi-step graph (this step's readers keep p.t)
  if (p.t_next != nullptr && n == 0 && blockIdx.y == 0 && k == 0) *p.t_next = t - 1;
  t = t < 1 ? 1 : (t > p.tmax ? p.tmax : t);
  float v = p.pos_table[(size_t)(t - 1) * 256 + k];
  if (p.y != nullptr) {
    int64_t yy;
    if (p.y_null_first) yy = (n < p.n_half) ? p.y_null : p.y[n - p.n_half];
    else yy = p.y[n];
    yy = yy < 0 ? 0 : (yy >= p.ncls ? p.ncls - 1 : yy);
    v += p.class_emb[yy * 256 + k];
  }
  if (p.cnd != nullptr) {
    v += p.cnd[(n % p.cond_rows) * 256 + k];
  } else if (p.vals != nullptr) {
    const int row = n % p.cond_rows;
    if (k < 12) in24[k] = p.vals[row * 12 + k];
    else if (k < 24) in24[k] = p.mask[row * 12 + (k - 12)];
    __syncthreads();
    float a = p.b0[k];
#pragma unroll
    for (int j = 0; j < 24; ++j) a += p.w0[k * 24 + j] * in24[j];
    h[k] = silu(a);
    __syncthreads();
    // all 256 weight loads of the dot product issued up front (fully unrolled: the latency of
    // one L2 round trip instead of one per unrolled trip), same four-way summation order
    float c0 = 0.f, c1 = 0.f, c2 = 0.f, c3 = 0.f;
#pragma unroll
    for (int j = 0; j < 256; j += 4) {
      c0 += p.w2t[(j + 0) * 256 + k] * h[j + 0];
      c1 += p.w2t[(j + 1) * 256 + k] * h[j + 1];
      c2 += p.w2t[(j + 2) * 256 + k] * h[j + 2];
      c3 += p.w2t[(j + 3) * 256 + k] * h[j + 3];
    }
    v += p.b2[k] + ((c0 + c1) + (c2 + c3));
  }
  s[k] = silu(v);
  __syncthreads();
  const int per = (p.hsum + gridDim.y - 1) / gridDim.y;
  const int o = blockIdx.y * per + k;
  if (k < per && o < p.hsum) {
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
    for (int j = 0; j < 256; j += 4) {
      a0 += p.wht[(size_t)(j + 0) * p.hsum + o] * s[j + 0];
      a1 += p.wht[(size_t)(j + 1) * p.hsum + o] * s[j + 1];
      a2 += p.wht[(size_t)(j + 2) * p.hsum + o] * s[j + 2];
      a3 += p.wht[(size_t)(j + 3) * p.hsum + o] * s[j + 3];
    }
    p.out[(size_t)n * p.hsum + o] = p.bh[o] + ((a0 + a1) + (a2 + a3));
  }
}

// ---------------------------------------------------------------------------
// inc's first conv (models/unet_cond.py:17, Conv2d(in_ch, 64, 3, padding=1, bias=False)) on the NCHW
// network input: K = 9 taps x <= 4 channels is far too thin for a GEMM (the implicit GEMM padded it
// to 64 and paid a global round trip per 16-deep K step), so it runs as a direct fp32 conv: a block
// owns PX consecutive output pixels of one sample x 64 channels — PX = 32: one image row segment
// (W % 32 == 0); PX = 16: any 16 pixels of a map 16..32 wide (H W % 16 == 0: the reference sampler's
// 28 x 28 latents), spanning at most two image rows — each output accumulates its 36 products in
// fixed (tap, channel) order with fp32 FMAs (exact fp32 semantics in every precision mode).  Output
// NHWC fp32 plus the GroupNorm (sum, sum of squares) partial of each (PX pixels, 32 channels) group —
// the layout igemm_epilogue writes (rgrp = PX, seg = 32).
// ---------------------------------------------------------------------------
struct ConvInParams {
  const float* x;      // NCHW [n][creal][H][W]
  int creal, n_mod;    // channels present; sample index modulo n_mod (0: none)
  float scale;         // divide the input by scale (1: identity)
  const float* B;      // packed [npad][kpad], k = tap * cin + c
  int cin, kpad;
  float* out;          // NHWC [n][H][W][64]
  float2* rowpart;     // [n][HW / PX][2]
  int H, W;
};
template <int PX>
__global__ __launch_bounds__(256) void conv_in_kernel(const ConvInParams p) {
  // thread (output channel co, pixel group pg): pixels PX / 4 pg .. + PX / 4 - 1 of the block's PX; its
  // 36 weights in registers, the input patch (PR rows x 34 columns x 4 channels) in LDS (float4 per
  // pixel: one broadcast ds_read_b128 per pixel and tap), one coalesced 256-byte row of channels per
  // pixel store
  static_assert(PX == 32 || PX == 16, "conv_in: 32- or 16-pixel blocks");
  constexpr int PR = PX == 32 ? 3 : 4, PP = PX / 4;
  __shared__ float ws[64][37];
  __shared__ __attribute__((aligned(16))) float inl[PR][34][4];
  __shared__ float2 red[4][2];
  const int tid = threadIdx.x, co = tid & 63, pg = tid >> 6;
  for (int i = tid; i < 64 * 36; i += 256) {
    const int o = i / 36, k = i - o * 36, tap = k >> 2, c = k & 3;
    ws[o][k] = c < p.cin ? p.B[(size_t)o * p.kpad + tap * p.cin + c] : 0.f;
  }
  const int HW = p.H * p.W;
  const int m0 = blockIdx.x * PX;
  const int n = m0 / HW, r = m0 - n * HW, y = r / p.W, x0 = PX == 32 ? r - y * p.W : 0;
  const int ns = p.n_mod ? n % p.n_mod : n;
  for (int i = tid; i < PR * 34 * 4; i += 256) {
    const int c = i / (PR * 34), rem = i - c * (PR * 34), ry = rem / 34, cx = rem - ry * 34;
    const int iy = y + ry - 1, ix = x0 + cx - 1;
    const bool ok = iy >= 0 && iy < p.H && ix >= 0 && ix < p.W && c < p.creal;
    const float v = ok ? p.x[((size_t)ns * p.creal + c) * HW + (size_t)iy * p.W + ix] : 0.f;
    inl[ry][cx][c] = p.scale != 1.f ? v / p.scale : v;
  }
  __syncthreads();
  float w[36];
#pragma unroll
  for (int k = 0; k < 36; ++k) w[k] = ws[co][k];
  float* o = p.out + (size_t)m0 * 64 + co;
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int j = 0; j < PP; ++j) {
    const int px = PP * pg + j;
    // patch row / column of the pixel (PX = 16: the block's pixels continue on the next image row)
    const int rr = PX == 32 ? 0 : (r - y * p.W + px) / p.W, cc = PX == 32 ? px : r - y * p.W + px - rr * p.W;
    float a = 0.f;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {  // (tap, channel) order as the packed weights
      const floatx4 v = *reinterpret_cast<const floatx4*>(&inl[rr + tap / 3][cc + tap % 3][0]);
#pragma unroll
      for (int c = 0; c < 4; ++c) a = fmaf(w[tap * 4 + c], v[c], a);
    }
    o[(size_t)px * 64] = a;
    s1 += a;
    s2 += a * a;
  }
  // GroupNorm partials: segment s = channels 32 s .. + 31 = lanes 32 s .. + 31 of every wave
#pragma unroll
  for (int off = 1; off < 32; off <<= 1) {
    s1 += __shfl_xor(s1, off, 64);
    s2 += __shfl_xor(s2, off, 64);
  }
  if ((tid & 31) == 0) red[pg][co >> 5] = make_float2(s1, s2);
  __syncthreads();
  if (tid < 2)
    p.rowpart[((size_t)n * (HW / PX) + r / PX) * 2 + tid] =
        make_float2((red[0][tid].x + red[1][tid].x) + (red[2][tid].x + red[3][tid].x),
                    (red[0][tid].y + red[1][tid].y) + (red[2][tid].y + red[3][tid].y));
}

// ---------------------------------------------------------------------------
// K4 GroupNorm finalize: (mean, rstd) per (n, g) from per-row partials written by
// the conv epilogue.  Sums are combined in double (deterministic order).
// nn.GroupNorm eps = 1e-5 (models/unet_cond.py:20, models/vae.py:36).
// ---------------------------------------------------------------------------
// rowpart layout: [n][R rows][nseg] (R = partial rows per sample); elements per
// group = HWo * C / G.
static __global__ __launch_bounds__(256) void gn_finalize_kernel(const float2* rowpart, float2* stats, int R, int nseg,
                                                           int G, int C, int HWo, float eps) {
  const int ng = blockIdx.x, n = ng / G, g = ng % G;
  const int spg = nseg / G;
  const int cnt = R * spg;
  double s1 = 0.0, s2 = 0.0;
  for (int i = threadIdx.x; i < cnt; i += 256) {
    const int r = i / spg, sg = g * spg + (i - r * spg);
    const float2 v = rowpart[((size_t)n * R + r) * nseg + sg];
    s1 += (double)v.x;
    s2 += (double)v.y;
  }
  __shared__ double r1[256], r2[256];
  r1[threadIdx.x] = s1;
  r2[threadIdx.x] = s2;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      r1[threadIdx.x] += r1[threadIdx.x + o];
      r2[threadIdx.x] += r2[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double cntd = (double)HWo * (double)(C / G);
    const double mean = r1[0] / cntd;
    double var = r2[0] / cntd - mean * mean;
    var = var < 0.0 ? 0.0 : var;
    stats[ng] = make_float2((float)mean, (float)(1.0 / sqrt(var + (double)eps)));
  }
}

// ---------------------------------------------------------------------------
// GroupNorm application, fused with the statistics reduction for G == 1
// (models/unet_cond.py:20-28):
//   out = GN(raw)                    (act=0, no res)     non-residual ResBlock output
//   out = GELU(GN(raw))              (act=1, no res)     mid-block activation / VAE stage
//   out = GELU(res + GN(raw))        (res != null)       residual ResBlock output
//   out += emb[n][emb_off + c]       (emb != null)       Down/Up "+ emb" (unet_cond.py:69,99)
// Stats: either precomputed (stats != null, any G) or reduced here from the conv
// epilogue's per-row partials (rowpart, G == 1): every block re-reduces its sample's
// partials (<= 32 KB, L2-resident) in double, in a fixed order, then normalises its
// chunk of the sample.  grid = (chunks, N).
// ---------------------------------------------------------------------------
struct NormParams {
  const float* raw; const float2* rowpart; int nseg; int rrows; const float2* stats;
  const float* gamma; const float* beta;
  int C, G, HW;
  const float* res; int act;
  int gexact;                      // 1: GELU in the erf form (exact-fp32 mode), 0: gelu()
  const float* emb; int emb_stride; int emb_off;
  int n_src;                       // >0: raw / stats / res of output sample n come from sample n % n_src
  float* out;                      // fp32 output, or null when only the planes are written
  _Float16* out_h; _Float16* out_l;  // optional fp16 hi/lo planes (split-precision GEMM operand)
};

// norm_kernel / prep_kernel outputs: plain stores (their consumers read them back from L2; the
// non-temporal hint measured -0.9 %, round 4)
DMX_DEV void st4(float* a, floatx4 v) { *reinterpret_cast<floatx4*>(a) = v; }
static __global__ __launch_bounds__(256) void norm_kernel(const NormParams p) {
  const int n = blockIdx.y, tid = threadIdx.x;
  const int ns = p.n_src > 0 ? n % p.n_src : n;  // source sample (CFG-shared trunk prefix)
  // This block's float4 range [beg, end) of the sample; chunks are multiples of 256, so when
  // C/4 divides 256 a thread's channel is loop-invariant.  4 float4 per thread per pass,
  // every load issued before any is used; the first pass's loads are issued before the
  // statistics reduction below, which they do not depend on.
  const int C4 = p.C >> 2;
  const int per = p.HW * C4;
  const int chunk = (((per + (int)gridDim.x - 1) / (int)gridDim.x) + 255) & ~255;
  const int beg = blockIdx.x * chunk, end = min(per, beg + chunk);
  const size_t base = (size_t)n * per * 4, sbase = (size_t)ns * per * 4;
  const float* raw = p.raw + sbase;
  const float* res = p.res != nullptr ? p.res + sbase : nullptr;
  floatx4 v[4], r[4];
  auto load = [&](int i0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int idx = min(i0 + 256 * k, end - 1);
      v[k] = ld4(raw + (size_t)idx * 4);
      if (res != nullptr) r[k] = ld4(res + (size_t)idx * 4);
    }
  };
  int i0 = beg + tid;
  if (i0 < end) load(i0);
  const int cpg = p.C / p.G;
  const bool cfix = (256 % C4) == 0;
  const int cthr = (tid % C4) * 4;
  floatx4 fg{}, fb{}, fe{};  // gamma / beta / emb of a loop-invariant channel, loaded up front
  if (cfix) {
    fg = ld4(p.gamma + cthr);
    fb = ld4(p.beta + cthr);
    if (p.emb != nullptr) fe = ld4(p.emb + (size_t)n * p.emb_stride + p.emb_off + cthr);
  }

  __shared__ double r1[4], r2[4];
  __shared__ float2 st_s;
  if (p.rowpart != nullptr) {  // GroupNorm(1, C): reduce this sample's (sum, sumsq) partials in double
    const int cnt = p.rrows * p.nseg;
    const float2* rp = p.rowpart + (size_t)ns * cnt;
    double s1 = 0.0, s2 = 0.0;
    for (int i = tid; i < cnt; i += 256) {
      const float2 q = rp[i];
      s1 += (double)q.x;
      s2 += (double)q.y;
    }
    s1 = wave_sum_dpp(s1);  // (DPP / permlane: no LDS round trips before the stores can start)
    s2 = wave_sum_dpp(s2);
    if ((tid & 63) == 0) {
      r1[tid >> 6] = s1;
      r2[tid >> 6] = s2;
    }
    __syncthreads();
    if (tid == 0) {
      const double cntd = (double)p.HW * (double)p.C;
      const double mean = ((r1[0] + r1[1]) + (r1[2] + r1[3])) / cntd;
      double var = ((r2[0] + r2[1]) + (r2[2] + r2[3])) / cntd - mean * mean;
      var = var < 0.0 ? 0.0 : var;
      st_s = make_float2((float)mean, (float)(1.0 / sqrt(var + 1e-5)));
    }
    __syncthreads();
  }
  for (; i0 < end; i0 += 1024) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int idx = i0 + 256 * k;
      if (idx >= end) break;
      const int c = cfix ? cthr : (idx % C4) * 4;
      const float2 st = p.rowpart != nullptr ? st_s : p.stats[ns * p.G + c / cpg];
      floatx4 o = cfix ? gn_apply4v(v[k], st, fg, fb, 0) : gn_apply4(v[k], st, p.gamma, p.beta, c, 0);
      if (res != nullptr) {
        if (p.gexact) {
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = gelu_exact(r[k][j] + o[j]);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = gelu(r[k][j] + o[j]);
        }
      } else if (p.act) {
        if (p.gexact) {
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = gelu_exact(o[j]);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = gelu(o[j]);
        }
      }
      if (p.emb != nullptr) {
        const floatx4 e = cfix ? fe : ld4(p.emb + (size_t)n * p.emb_stride + p.emb_off + c);
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] += e[j];
      }
      const size_t off = base + (size_t)idx * 4;
      if (p.out != nullptr) st4(p.out + off, o);
      if (p.out_h != nullptr) {
        half4 hh, ll;
        split4(o, hh, ll);
        *reinterpret_cast<half4*>(p.out_h + off) = hh;
        *reinterpret_cast<half4*>(p.out_l + off) = ll;
      }
    }
    if (i0 + 1024 < end) load(i0 + 1024);
  }
}

// Split-K reduction fused with GroupNorm(1, C) for the small low-resolution convolutions
// (one 1024-thread block per source sample, the whole sample — HW*C <= RN_MAXV*4096 values —
// held in registers): sums the split slabs in split order (+ bias), reduces the sample's
// (sum, sum of squares) in double in a fixed order, then applies exactly norm_kernel's
// GroupNorm (+GELU | +residual GELU) (+emb) and writes fp32 and / or f16 hi/lo planes,
// including the CFG fan-out (n_src > 0: outputs s and s + n_src both come from source s).
// Replaces splitk_reduce_kernel + norm_kernel (two launches, two HBM round trips of the
// conv output) at 8x8 / 4x4 where both are launch-latency bound.
constexpr int RN_MAXV = 8;  // float4 per thread

// KV = float4 per thread (power of two >= ceil(HW*C/4 / 1024)); the split slabs are read SB at
// a time with every load of a batch in flight together (one memory round trip per batch, not
// per slab) and summed in split order.  (Loading bias / gamma / beta / residual / emb up
// front with the first batch was measured slower.)
template <int KV>
__global__ __launch_bounds__(1024) void reduce_norm_kernel(const float* partial, int splits, const float* bias,
                                                           const NormParams p) {
  static_assert(KV >= 2, "reduce_norm_kernel: the KV = 1 instance is retired (engine.hip RN_MIN_KV)");
  constexpr int SB = KV >= 16 ? 1 : 16 / KV;  // slabs per batch (<= 64 VGPRs of loads)
  const int s = blockIdx.x, tid = threadIdx.x;
  const int C4 = p.C >> 2, per = p.HW * C4;
  const size_t sstride = (size_t)gridDim.x * per * 4;  // floats per split slab (all source samples)
  const size_t sbase = (size_t)s * per * 4;
  floatx4 v[KV];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int k = 0; k < KV; ++k) v[k] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int sp0 = 0; sp0 < splits; sp0 += SB) {
    floatx4 a[SB][KV];
#pragma unroll
    for (int b = 0; b < SB; ++b)
#pragma unroll
      for (int k = 0; k < KV; ++k) {
        const int idx = tid + 1024 * k;
        a[b][k] = (sp0 + b < splits && idx < per) ? ld4(partial + (sp0 + b) * sstride + sbase + (size_t)idx * 4)
                                                  : floatx4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
    for (int b = 0; b < SB; ++b)
#pragma unroll
      for (int k = 0; k < KV; ++k)
#pragma unroll
        for (int j = 0; j < 4; ++j) v[k][j] += a[b][k][j];
  }
#pragma unroll
  for (int k = 0; k < KV; ++k) {
    const int idx = tid + 1024 * k;
    if (idx < per) {
      if (bias != nullptr) {
        const floatx4 b = ld4(bias + (idx % C4) * 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[k][j] += b[j];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s1 += v[k][j];
        s2 += v[k][j] * v[k][j];
      }
    }
  }
  __shared__ double r1[16], r2[16];
  __shared__ float2 st_s;
  const double d1 = wave_sum_dpp((double)s1), d2 = wave_sum_dpp((double)s2);
  if ((tid & 63) == 0) {
    r1[tid >> 6] = d1;
    r2[tid >> 6] = d2;
  }
  __syncthreads();
  if (tid == 0) {
    double a1 = 0.0, a2 = 0.0;
    for (int w = 0; w < 16; ++w) {
      a1 += r1[w];
      a2 += r2[w];
    }
    const double cnt = (double)p.HW * (double)p.C;
    const double mean = a1 / cnt;
    double var = a2 / cnt - mean * mean;
    var = var < 0.0 ? 0.0 : var;
    st_s = make_float2((float)mean, (float)(1.0 / sqrt(var + 1e-5)));
  }
  __syncthreads();
  const float2 st = st_s;
  const int nout = p.n_src > 0 ? 2 : 1;
  for (int q = 0; q < nout; ++q) {
    const int n = s + q * (p.n_src > 0 ? p.n_src : 0);
    const size_t base = (size_t)n * per * 4;
#pragma unroll
    for (int k = 0; k < KV; ++k) {
      const int idx = tid + 1024 * k;
      if (idx >= per) break;
      const int c = (idx % C4) * 4;
      floatx4 o = gn_apply4(v[k], st, p.gamma, p.beta, c, 0);
      if (p.res != nullptr) {
        const floatx4 r = ld4(p.res + sbase + (size_t)idx * 4);
        if (p.gexact) {
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = gelu_exact(r[j] + o[j]);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = gelu(r[j] + o[j]);
        }
      } else if (p.act) {
        if (p.gexact) {
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = gelu_exact(o[j]);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = gelu(o[j]);
        }
      }
      if (p.emb != nullptr) {
        const floatx4 e = ld4(p.emb + (size_t)n * p.emb_stride + p.emb_off + c);
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] += e[j];
      }
      const size_t off = base + (size_t)idx * 4;
      if (p.out != nullptr) *reinterpret_cast<floatx4*>(p.out + off) = o;
      if (p.out_h != nullptr) {
        half4 hh, ll;
        split4(o, hh, ll);
        *reinterpret_cast<half4*>(p.out_h + off) = hh;
        *reinterpret_cast<half4*>(p.out_l + off) = ll;
      }
    }
  }
}

// Materialise a fused source (2x2 max-pool, bilinear-x2 + pad + concat) as a plain
// NHWC tensor [N][H][W][C] (models/unet_cond.py:58, 88-97).
// oh / ol (optional): the same values also as f16 hi / lo planes (the next conv's split-GEMM A).
template <int SRC>
__global__ __launch_bounds__(256) void prep_kernel(const SrcDesc s, float* out, int N, int H, int W, _Float16* oh,
                                                   _Float16* ol) {
  const int C4 = s.C / 4;
  const size_t total = (size_t)N * H * W * C4;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
    const int c = (int)(i % C4) * 4;
    const size_t pix = i / C4;
    const int n = (int)(pix / ((size_t)H * W));
    const int rr = (int)(pix - (size_t)n * H * W);
    const int y = rr / W, x = rr - y * W;
    const floatx4 v = load_src4<SRC>(s, n, y, x, c, H, W);
    st4(out + pix * s.C + c, v);
    if (oh != nullptr) {
      half4 hh, ll;
      split4(v, hh, ll);
      *reinterpret_cast<half4*>(oh + pix * s.C + c) = hh;
      *reinterpret_cast<half4*>(ol + pix * s.C + c) = ll;
    }
  }
}

// ---------------------------------------------------------------------------
// LayerNorm over C per token (nn.LayerNorm eps=1e-5, models/unet_cond.py:37-39).
// One wave per token, C in {64,128,256,512}: C/64 values per lane, two-pass.
// ---------------------------------------------------------------------------
template <int CPL>
__global__ __launch_bounds__(256) void layernorm_kernel(const float* x, float* y, const float* w, const float* b,
                                                        int M, float eps) {
  constexpr int C = CPL * 64;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  const float* xr = x + (size_t)row * C;
  float v[CPL];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    v[j] = xr[lane + 64 * j];
    s += v[j];
  }
  const float mean = wave_sum(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const float d = v[j] - mean;
    q += d * d;
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)C + eps);
  float* yr = y + (size_t)row * C;
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const int c = lane + 64 * j;
    yr[c] = (v[j] - mean) * rstd * w[c] + b[c];
  }
}

// ---------------------------------------------------------------------------
// K5 multi-head self-attention core, flash-style, fp32 MFMA 16x16x4.
// qkv: [N][L][3C] (q | k | v, heads of width D inside each), out: [N][L][C].
// softmax(q k^T / sqrt(D)) v per (sample, head)  (nn.MultiheadAttention, 4 heads,
// models/unet_cond.py:36,49).  Computed transposed (S^T = K Q^T, O^T = V^T P^T) so
// the query sits on the lane: the P accumulator is directly the B operand of PV.
// Each wave owns 16*QT queries; 64-key K/V chunks are staged in LDS.  st (training forward, else
// null): per (sample, head, query) the row max m and 1 / sum l, [N][4][L][3] (slot 2 is the
// backward's, train.h attn_dq_mfma_kernel).
// ---------------------------------------------------------------------------
template <int D, int QT>
__global__ __launch_bounds__(256) void attention_kernel(const float* qkv, float* out, int L, int C, float* st) {
  constexpr int KC = 64, DS = D + 4, DP = D / 4;
  __shared__ __attribute__((aligned(16))) float Ks[KC][DS];
  __shared__ __attribute__((aligned(16))) float Vs[KC][DS];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int hd = blockIdx.y, n = blockIdx.z;
  const int ql = lane & 15, g = lane >> 4;
  const size_t rs = (size_t)3 * C;
  const float* base = qkv + (size_t)n * L * rs;
  const float scale = 1.0f / sqrtf((float)D);

  float qf[QT][DP];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    const int qi = blockIdx.x * (64 * QT) + wid * 16 * QT + qt * 16 + ql;
#pragma unroll
    for (int s = 0; s < DP; ++s) qf[qt][s] = (qi < L) ? base[(size_t)qi * rs + hd * D + g * DP + s] * scale : 0.f;
  }
  floatx4 o[QT][D / 16];
  float mrun[QT], lrun[QT];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    mrun[qt] = -INFINITY;
    lrun[qt] = 0.f;
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt) o[qt][dt] = floatx4{0.f, 0.f, 0.f, 0.f};
  }

  for (int c0 = 0; c0 < L; c0 += KC) {
    // stage K, V chunk (zero beyond L)
    for (int i = tid; i < KC * (D / 4); i += 256) {
      const int key = i / (D / 4), d4 = (i % (D / 4)) * 4;
      floatx4 kv = {0.f, 0.f, 0.f, 0.f}, vv = {0.f, 0.f, 0.f, 0.f};
      if (c0 + key < L) {
        const float* r = base + (size_t)(c0 + key) * rs + hd * D + d4;
        kv = ld4(r + C);
        vv = ld4(r + 2 * C);
      }
      *reinterpret_cast<floatx4*>(&Ks[key][d4]) = kv;
      *reinterpret_cast<floatx4*>(&Vs[key][d4]) = vv;
    }
    __syncthreads();
    const int nvalid = L - c0;
    floatx4 sc[QT][4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      float kf[DP];
#pragma unroll
      for (int s = 0; s < DP; ++s) kf[s] = Ks[kt * 16 + ql][g * DP + s];
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) {
        floatx4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < DP; ++s) a = __builtin_amdgcn_mfma_f32_16x16x4f32(kf[s], qf[qt][s], a, 0, 0, 0);
        sc[qt][kt] = a;
      }
    }
    // online softmax over this chunk (keys >= L masked)
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kt * 16 + g * 4 + r;
          if (key >= nvalid) sc[qt][kt][r] = -INFINITY;
          mx = fmaxf(mx, sc[qt][kt][r]);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mnew = fmaxf(mrun[qt], mx);
      const float alpha = expf(mrun[qt] - mnew);
      float ls = 0.f;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pv = expf(sc[qt][kt][r] - mnew);
          sc[qt][kt][r] = pv;
          ls += pv;
        }
      lrun[qt] = lrun[qt] * alpha + ls;
      mrun[qt] = mnew;
#pragma unroll
      for (int dt = 0; dt < D / 16; ++dt)
#pragma unroll
        for (int r = 0; r < 4; ++r) o[qt][dt][r] *= alpha;
    }
    // O^T += V^T P^T
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float vf[D / 16];
#pragma unroll
        for (int dt = 0; dt < D / 16; ++dt) vf[dt] = Vs[kt * 16 + g * 4 + r][dt * 16 + ql];
#pragma unroll
        for (int qt = 0; qt < QT; ++qt)
#pragma unroll
          for (int dt = 0; dt < D / 16; ++dt)
            o[qt][dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(vf[dt], sc[qt][kt][r], o[qt][dt], 0, 0, 0);
      }
    __syncthreads();
  }
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    float l = lrun[qt];
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    const float inv = 1.0f / l;
    const int qi = blockIdx.x * (64 * QT) + wid * 16 * QT + qt * 16 + ql;
    if (st != nullptr && g == 0 && qi < L) {
      float* so = st + (((size_t)n * 4 + hd) * L + qi) * 3;
      so[0] = mrun[qt];
      so[1] = inv;
    }
    if (qi < L) {
#pragma unroll
      for (int dt = 0; dt < D / 16; ++dt) {
        floatx4 v = o[qt][dt];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] *= inv;
        *reinterpret_cast<floatx4*>(out + ((size_t)n * L + qi) * C + hd * D + dt * 16 + g * 4) = v;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Philox4x32-10 counter RNG + Box-Muller -> 4 N(0,1) per counter (perf mode K8).
// ---------------------------------------------------------------------------
DMX_DEV uint4 philox4x32(uint4 ctr, uint2 key) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, ctr.x), lo0 = 0xD2511F53u * ctr.x;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, ctr.z), lo1 = 0xCD9E8D57u * ctr.z;
    ctr = make_uint4(hi1 ^ ctr.y ^ key.x, lo1, hi0 ^ ctr.w ^ key.y, lo0);
    key.x += 0x9E3779B9u;
    key.y += 0xBB67AE85u;
  }
  return ctr;
}

DMX_DEV floatx4 normal4(uint64_t seed, uint64_t stream, uint64_t index) {
  const uint4 r = philox4x32(make_uint4((uint32_t)index, (uint32_t)(index >> 32), (uint32_t)stream,
                                        (uint32_t)(stream >> 32)),
                             make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
  const float k = 2.3283064365386963e-10f;  // 2^-32
  const float u1 = ((float)r.x + 0.5f) * k, u2 = ((float)r.y + 0.5f) * k;
  const float u3 = ((float)r.z + 0.5f) * k, u4 = ((float)r.w + 0.5f) * k;
  const float a = sqrtf(-2.0f * logf(u1)), b = sqrtf(-2.0f * logf(u3));
  const float t1 = 6.283185307179586f * u2, t2 = 6.283185307179586f * u4;
  return floatx4{a * cosf(t1), a * sinf(t1), b * cosf(t2), b * sinf(t2)};
}

// ---------------------------------------------------------------------------
// K1/K6: out head (conv1x1 64->Co + bias) fused with the CFG mix and the DDPM
// posterior step.  Reference: unet_cond.py:153 (out), diff.py:151 (CFG),
// diff.py:141-144,158-162 (update).  The update arithmetic is performed with one
// rounding per reference op, in the reference's op order, so given the same eps it
// is bit-identical to torch-CPU:
//   eps = eu + g*(ec - eu); mu = (x - c1[t]*eps) / c2[t]; x' = mu + noise*sd[t]
// with c1 = (1-a)/sqrt(1-ab), c2 = sqrt(a), sd = sqrt((1-a)(1-ab_prev)/(1-ab))
// tabulated on the host by torch.  noise = 0 where t == 1.
// feat: [2B or B][H][W][64] NHWC; x, x_out, noise: NCHW [B][Co][H][W].
// ---------------------------------------------------------------------------
struct StepTailParams {
  const float* feat; const float* w; const float* b;  // w: [Co][64]
  int Co, B, HW, cfg;                                 // cfg: feat holds [uncond B | cond B]
  float guidance;
  const float* eps_u; const float* eps_c;             // alternative: precomputed eps (NCHW), feat null
  const float* x; float* x_out;
  const int64_t* t; int t_stride; int tmax;
  const float* c1; const float* c2; const float* sd;  // [tmax], index t-1
  const float* noise;                                 // NCHW or null => Philox
  uint64_t seed; int64_t sample_offset;
  int* range_flag;                                    // set to 1 when eps is not finite (or null)
};

// Range guard of the split-precision modes: an operand beyond the f16 range (|v| >= 65520)
// becomes inf in its hi plane, and any inf / NaN reaching a network output makes that output
// non-finite.  Output kernels raise a sticky flag (a plain vector store) that the host reads
// at its checkpoints and answers by recomputing in exact-fp32 MFMA mode.
DMX_DEV void flag_nonfinite(int* flag, float v) {
  if (flag != nullptr && !(fabsf(v) <= 3.402823466e38f)) *flag = 1;
}

// One IEEE rounding per reference op: the product is forced through a register
// (opaque asm barrier) so no multiply-add pair can be contracted into an FMA,
// whatever the -ffp-contract mode of the including code.
DMX_DEV float rnd(float v) {
  asm volatile("" : "+v"(v));
  return v;
}
DMX_DEV float ddpm_elem(float x, float eps, float c1, float c2, float sd, float nz) {
  const float mu = rnd(x - rnd(c1 * eps)) / c2;
  return mu + rnd(nz * sd);
}

static __global__ __launch_bounds__(256) void step_tail_kernel(const StepTailParams p) {
  const int pix = blockIdx.x * 256 + threadIdx.x;
  const int n = blockIdx.y;
  if (pix >= p.HW) return;
  int64_t t = p.t[(size_t)n * p.t_stride];
  t = t < 1 ? 1 : (t > p.tmax ? p.tmax : t);
  float eu[4], ec[4];
  const int Co = p.Co;
  if (p.feat != nullptr) {
    const float* fu = p.feat + ((size_t)n * p.HW + pix) * 64;
    const float* fc = p.feat + ((size_t)(n + p.B) * p.HW + pix) * 64;
    for (int c = 0; c < Co; ++c) {
      eu[c] = p.b[c];
      ec[c] = p.b[c];
    }
    for (int k = 0; k < 64; k += 4) {
      const floatx4 a = ld4(fu + k);
      floatx4 bb = {0.f, 0.f, 0.f, 0.f};
      if (p.cfg) bb = ld4(fc + k);
      for (int c = 0; c < Co; ++c) {
        const floatx4 w = ld4(p.w + c * 64 + k);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          eu[c] += w[j] * a[j];
          ec[c] += w[j] * bb[j];
        }
      }
    }
  } else {
    for (int c = 0; c < Co; ++c) {
      eu[c] = p.eps_u[((size_t)n * Co + c) * p.HW + pix];
      ec[c] = p.cfg ? p.eps_c[((size_t)n * Co + c) * p.HW + pix] : 0.f;
    }
  }
  float nz[4] = {0.f, 0.f, 0.f, 0.f};
  if (t != 1) {
    if (p.noise != nullptr) {
      for (int c = 0; c < Co; ++c) nz[c] = p.noise[((size_t)n * Co + c) * p.HW + pix];
    } else {
      const floatx4 r = normal4(p.seed, (uint64_t)t, ((uint64_t)(n + p.sample_offset) * p.HW + pix));
      for (int c = 0; c < Co && c < 4; ++c) nz[c] = r[c];
    }
  }
  const float c1 = p.c1[t - 1], c2 = p.c2[t - 1], sd = p.sd[t - 1];
  for (int c = 0; c < Co; ++c) {
    const float eps = p.cfg ? eu[c] + rnd(p.guidance * rnd(ec[c] - eu[c])) : eu[c];
    flag_nonfinite(p.range_flag, eps);
    const size_t idx = ((size_t)n * Co + c) * p.HW + pix;
    p.x_out[idx] = ddpm_elem(p.x[idx], eps, c1, c2, sd, nz[c]);
  }
}

// step_tail_kernel for the network head path (feat given, Co = 4): 16 lanes per pixel, each
// loading one float4 of the pixel's 64 features (a wave reads 4 whole 256-byte rows, fully
// coalesced, instead of 64 rows at a 256-byte lane stride); the 1x1-conv dot products are
// reduced over the 16 lanes with DPP (fixed order), then lanes 0..3 of the group finish
// channel c = lane (CFG mix, posterior mean, Philox noise, store).
DMX_DEV float group_sum16(float s) {  // sum over aligned 16-lane rows (DPP), same bits in every lane
  auto dpp = [](float v, auto ctrl) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), decltype(ctrl)::value,
                                                                 0xF, 0xF, false));
  };
  s += dpp(s, std::integral_constant<int, 0xB1>{});   // quad_perm [1,0,3,2]
  s += dpp(s, std::integral_constant<int, 0x4E>{});   // quad_perm [2,3,0,1]
  s += dpp(s, std::integral_constant<int, 0x141>{});  // row_half_mirror
  s += dpp(s, std::integral_constant<int, 0x140>{});  // row_mirror
  return s;
}

static __global__ __launch_bounds__(256) void step_tail4_kernel(const StepTailParams p) {
  const int sub = threadIdx.x & 15, pix = blockIdx.x * 16 + (threadIdx.x >> 4), n = blockIdx.y;
  const bool valid = pix < p.HW;
  const int pc = valid ? pix : 0;
  const floatx4 a = ld4(p.feat + ((size_t)n * p.HW + pc) * 64 + 4 * sub);
  floatx4 bb = {0.f, 0.f, 0.f, 0.f};
  if (p.cfg) bb = ld4(p.feat + ((size_t)(n + p.B) * p.HW + pc) * 64 + 4 * sub);
  float eu[4], ec[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const floatx4 w = ld4(p.w + c * 64 + 4 * sub);
    float su = 0.f, sc = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      su += w[j] * a[j];
      sc += w[j] * bb[j];
    }
    eu[c] = p.b[c] + group_sum16(su);
    ec[c] = p.b[c] + group_sum16(sc);
  }
  if (!valid || sub >= 4) return;
  int64_t t = p.t[(size_t)n * p.t_stride];
  t = t < 1 ? 1 : (t > p.tmax ? p.tmax : t);
  const int c = sub;
  const float u = sub == 0 ? eu[0] : sub == 1 ? eu[1] : sub == 2 ? eu[2] : eu[3];
  const float v = sub == 0 ? ec[0] : sub == 1 ? ec[1] : sub == 2 ? ec[2] : ec[3];
  float nz = 0.f;
  const size_t idx = ((size_t)n * 4 + c) * p.HW + pix;
  if (t != 1) {
    if (p.noise != nullptr) {
      nz = p.noise[idx];
    } else {
      const floatx4 r = normal4(p.seed, (uint64_t)t, ((uint64_t)(n + p.sample_offset) * p.HW + pix));
      nz = c == 0 ? r[0] : c == 1 ? r[1] : c == 2 ? r[2] : r[3];
    }
  }
  const float eps = p.cfg ? u + rnd(p.guidance * rnd(v - u)) : u;
  flag_nonfinite(p.range_flag, eps);
  p.x_out[idx] = ddpm_elem(p.x[idx], eps, p.c1[t - 1], p.c2[t - 1], p.sd[t - 1], nz);
}

// conv1x1 64 -> Co + bias into NCHW (models/unet_cond.py:153, the `out` layer).
static __global__ __launch_bounds__(256) void out_head_kernel(const float* feat, const float* w, const float* b, float* eps,
                                                       int Co, int HW, int* range_flag) {
  const int pix = blockIdx.x * 256 + threadIdx.x, n = blockIdx.y;
  if (pix >= HW) return;
  const float* f = feat + ((size_t)n * HW + pix) * 64;
  float acc[4];
  for (int c = 0; c < Co; ++c) acc[c] = b[c];
  for (int k = 0; k < 64; k += 4) {
    const floatx4 a = ld4(f + k);
    for (int c = 0; c < Co; ++c) {
      const floatx4 ww = ld4(w + c * 64 + k);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[c] += ww[j] * a[j];
    }
  }
  for (int c = 0; c < Co; ++c) {
    flag_nonfinite(range_flag, acc[c]);
    eps[((size_t)n * Co + c) * HW + pix] = acc[c];
  }
}

// GeomHead: GAP over HW of feat (64 ch) -> Linear(64->hid) -> SiLU -> Linear(hid->gdim)
// (models/unet_cond_geom.py:8-23).  One block per sample; dynamic LDS = (64 + hid) floats.
static __global__ __launch_bounds__(256) void geom_head_kernel(const float* feat, int HW, const float* w0, const float* b0,
                                                        const float* w2, const float* b2, int hid, int gdim,
                                                        float* geom) {
  extern __shared__ float sm[];
  __shared__ float part[4][64];
  float* g = sm;
  float* h = sm + 64;
  const int n = blockIdx.x, tid = threadIdx.x, c = tid & 63, sl = tid >> 6;
  float s = 0.f;
  for (int pix = sl; pix < HW; pix += 4) s += feat[((size_t)n * HW + pix) * 64 + c];
  part[sl][c] = s;
  __syncthreads();
  if (tid < 64) g[tid] = (part[0][tid] + part[1][tid] + part[2][tid] + part[3][tid]) / (float)HW;
  __syncthreads();
  for (int j = tid; j < hid; j += 256) {
    float a = b0[j];
    for (int k = 0; k < 64; ++k) a += w0[j * 64 + k] * g[k];
    h[j] = silu(a);
  }
  __syncthreads();
  for (int o = tid; o < gdim; o += 256) {
    float acc = b2[o];
    for (int k = 0; k < hid; ++k) acc += w2[(size_t)o * hid + k] * h[k];
    geom[(size_t)n * gdim + o] = acc;
  }
}

// VAE tail: conv3x3 64->3 + bias (dec.18) -> sigmoid (models/vae.py:49,69), then
// diff.py:58-62's x*255 -> clamp(0,255) -> uint8 (truncation), HWC for PIL.
// in: materialised GELU(GN(dec.15)) NHWC [N][H][W][64].
static __global__ __launch_bounds__(256) void vae_tail_kernel(const float* in, const float* w, const float* b, int N, int H,
                                                       int W, float* img, uint8_t* u8, int* range_flag) {
  __shared__ float ws[9 * 64 * 3];  // [tap][c][co]
  for (int i = threadIdx.x; i < 9 * 64 * 3; i += 256) {
    const int co = i % 3, c = (i / 3) % 64, tap = i / 192;
    ws[i] = w[(co * 64 + c) * 9 + tap];
  }
  __syncthreads();
  const int pix = blockIdx.x * 256 + threadIdx.x, n = blockIdx.y;
  if (pix >= H * W) return;
  const int y = pix / W, x = pix - y * W;
  float a0 = b[0], a1 = b[1], a2 = b[2];
  for (int tap = 0; tap < 9; ++tap) {
    const int iy = y + tap / 3 - 1, ix = x + tap % 3 - 1;
    if (iy < 0 || ix < 0 || iy >= H || ix >= W) continue;
    const float* src = in + (((size_t)n * H + iy) * W + ix) * 64;
    const float* wt = ws + tap * 192;
    for (int c = 0; c < 64; c += 4) {
      const floatx4 v = ld4(src + c);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a0 += v[j] * wt[(c + j) * 3 + 0];
        a1 += v[j] * wt[(c + j) * 3 + 1];
        a2 += v[j] * wt[(c + j) * 3 + 2];
      }
    }
  }
  flag_nonfinite(range_flag, a0 + a1 + a2);
  const float o[3] = {1.f / (1.f + expf(-a0)), 1.f / (1.f + expf(-a1)), 1.f / (1.f + expf(-a2))};
  for (int co = 0; co < 3; ++co) {
    if (img != nullptr) img[((size_t)n * 3 + co) * H * W + pix] = o[co];
    if (u8 != nullptr) {
      float q = rnd(o[co] * 255.f);
      q = fminf(fmaxf(q, 0.f), 255.f);
      u8[((size_t)n * H * W + pix) * 3 + co] = (uint8_t)q;
    }
  }
}

// VAE encoder tail (models/vae.py:52-60): to_mu / to_logvar (1x1 convs 256 -> 4, bias),
// logvar.clamp(-30, 20), std = exp(0.5 logvar), z = (mu + eps * std) * scale with eps the
// reference's randn_like draw (passed in, NCHW), and the per-sample KL term
// 0.5 * sum_{c,y,x}(exp(lv) + mu^2 - 1 - lv) / (H_img * W_img).  Grid (cdiv(HW, 32), N): 32 pixels per
// block, 8 lanes per pixel (channels 4 lane + 32 i: 128-byte coalesced rows, conflict-free weight
// reads) reduced by shuffles; the KL terms per block in a fixed order to klp[n][block], summed in
// block order by vae_enc_kl_kernel.
// in: materialised GELU(GN(enc.15)) NHWC [N][HW][256].
static __global__ __launch_bounds__(256) void vae_enc_tail_kernel(const float* in, const float* wmu, const float* bmu,
                                                           const float* wlv, const float* blv, const float* eps,
                                                           float* z, float* klp, int HW, float scale,
                                                           int* range_flag) {
  __shared__ __attribute__((aligned(16))) float ws[8][256];  // rows 0-3: to_mu, 4-7: to_logvar ([out][in])
  __shared__ float red[4];
  for (int i = threadIdx.x; i < 8 * 256; i += 256) ws[i / 256][i % 256] = i < 1024 ? wmu[i] : wlv[i - 1024];
  __syncthreads();
  const int n = blockIdx.y, l8 = threadIdx.x & 7, pix = blockIdx.x * 32 + (threadIdx.x >> 3);
  float a[8];
#pragma unroll
  for (int o = 0; o < 8; ++o) a[o] = 0.f;
  if (pix < HW) {
    const float* src = in + ((size_t)n * HW + pix) * 256 + 4 * l8;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const floatx4 v = ld4(src + 32 * i);
#pragma unroll
      for (int o = 0; o < 8; ++o) {
        const floatx4 w = *reinterpret_cast<const floatx4*>(&ws[o][32 * i + 4 * l8]);
#pragma unroll
        for (int j = 0; j < 4; ++j) a[o] += v[j] * w[j];
      }
    }
  }
#pragma unroll
  for (int o = 0; o < 8; ++o) {
    a[o] += __shfl_xor(a[o], 1, 64);
    a[o] += __shfl_xor(a[o], 2, 64);
    a[o] += __shfl_xor(a[o], 4, 64);
  }
  float kacc = 0.f;
  if (l8 == 0 && pix < HW) {
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      const float mu0 = a[o] + bmu[o], lv0 = a[o + 4] + blv[o];
      flag_nonfinite(range_flag, mu0 + lv0);
      const float mu = mu0, lv = fminf(fmaxf(lv0, -30.f), 20.f);
      const size_t idx = ((size_t)n * 4 + o) * HW + pix;
      z[idx] = (mu + eps[idx] * expf(0.5f * lv)) * scale;
      kacc += ((expf(lv) + mu * mu) - 1.f) - lv;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) kacc += __shfl_xor(kacc, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = kacc;
  __syncthreads();
  if (threadIdx.x == 0) klp[(size_t)n * gridDim.x + blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}
// kl[n] = 0.5 * (sum of the tail's block partials in block order) / (H_img * W_img)
static __global__ void vae_enc_kl_kernel(const float* klp, int nb, int N, float inv_px, float* kl) {
  for (int n = blockIdx.x * blockDim.x + threadIdx.x; n < N; n += gridDim.x * blockDim.x) {
    float sacc = 0.f;
    for (int b = 0; b < nb; ++b) sacc += klp[(size_t)n * nb + b];
    kl[n] = 0.5f * sacc * inv_px;
  }
}

// Weight repack into the implicit-GEMM B layout [phase][Npad][Kpad] (zero pad).
//   kind 0: Conv2d [Cout][Cin][KS][KS], k = (ky*KS+kx)*Cin + c
//   kind 1: Linear [Cout][Cin],        k = c
//   kind 2: ConvTranspose2d(4,s2,p1) [Cin][Cout][4][4], phase (py,px), tap (jy,jx)
//   kind 3: data gradient of a conv3x3 pad 1 (training): src = the forward weight [Cin][Cout][3][3]
//           (the job's Cout = the forward's input channels), B[n][tap Cin + c] = src[c][n][8 - tap]
//           (flipped taps, channel roles swapped)
//   kind 4: data gradient of a Linear (training): src = the forward weight [Cin][Cout], B[n][k] = src[k][n]
// 32-bit index arithmetic (every B here holds < 2^32 elements; 64-bit divisions made the batched
// refresh VALU-bound).
struct RepackJob {
  float* dst; const float* src; int kind, P, Npad, Kpad, Cout, Cin, KS;
};
struct CopyJob {
  float* dst; const float* src; size_t n;
};

DMX_DEV void repack_range(float* dst, const float* src, int kind, int P, int Npad, int Kpad, int Cout, int Cin, int KS,
                          unsigned first, unsigned stride, unsigned end = ~0u) {
  const unsigned total = min((unsigned)P * (unsigned)Npad * (unsigned)Kpad, end), kp = (unsigned)Kpad, np = (unsigned)Npad;
  for (unsigned i = first; i < total; i += stride) {
    const unsigned row = i / kp;
    const int k = (int)(i - row * kp), nn = (int)(row % np), ph = (int)(row / np);
    float v = 0.f;
    if (kind == 0) {
      if (nn < Cout && k < KS * KS * Cin) {
        const int tap = k / Cin, c = k - tap * Cin;
        v = src[(((size_t)nn * Cin + c) * KS + tap / KS) * KS + tap % KS];
      }
    } else if (kind == 1) {
      if (nn < Cout && k < Cin) v = src[(size_t)nn * Cin + k];
    } else if (kind == 2) {
      if (nn < Cout && k < 4 * Cin) {
        const int j = k / Cin, c = k % Cin, jy = j >> 1, jx = j & 1, py = ph >> 1, px = ph & 1;
        const int ky = py == 0 ? (jy == 0 ? 1 : 3) : (jy == 0 ? 0 : 2);
        const int kx = px == 0 ? (jx == 0 ? 1 : 3) : (jx == 0 ? 0 : 2);
        v = src[(((size_t)c * Cout + nn) * 4 + ky) * 4 + kx];
      }
    } else if (kind == 3) {
      if (nn < Cout && k < 9 * Cin) {
        const int tap = k / Cin, c = k - tap * Cin;
        v = src[((size_t)c * Cout + nn) * 9 + (8 - tap)];
      }
    } else {
      if (nn < Cout && k < Cin) v = src[(size_t)k * Cout + nn];
    }
    dst[i] = v;
  }
}

static __global__ void repack_kernel(float* dst, const float* src, int kind, int P, int Npad, int Kpad, int Cout, int Cin,
                              int KS) {
  repack_range(dst, src, kind, P, Npad, Kpad, Cout, Cin, KS, blockIdx.x * blockDim.x + threadIdx.x,
               gridDim.x * blockDim.x);
}

// dmx_model_refresh: every weight repack / parameter copy of the model in one launch each instead of
// one launch per tensor (the refresh follows every optimizer step).  The jobs are cut into chunks of
// BATCH_CHUNK elements (one block each, table built on the host), so a launch's blocks carry equal
// work whatever the tensor sizes.
constexpr unsigned BATCH_CHUNK = 8192;
struct BatchChunk {
  unsigned job, first;
};
static __global__ __launch_bounds__(256) void repack_batch_kernel(const RepackJob* jobs, const BatchChunk* chunks) {
  const BatchChunk c = chunks[blockIdx.x];
  const RepackJob j = jobs[c.job];
  repack_range(j.dst, j.src, j.kind, j.P, j.Npad, j.Kpad, j.Cout, j.Cin, j.KS, c.first + threadIdx.x, 256,
               c.first + BATCH_CHUNK);
}
// The 3x3 conv repacks (kind 0: B[n][t Cin + c] = src[n][c][t]; kind 3: B[n][t Cin + c] =
// src[c][n][8 - t]) as LDS-tiled transposes: a block takes 16 rows n x 32 channels c (x 9 taps), reads
// the source in its contiguous runs (288 / 144 floats) and writes 128-byte runs of B.  Only the live
// region (n < Cout, k < 9 Cin) is rewritten: the zero padding of B never changes after the first pack.
struct RepackTile {
  unsigned job, n0, c0;
};
static __global__ __launch_bounds__(256) void repack_tile_kernel(const RepackJob* jobs, const RepackTile* tiles) {
  __shared__ float T[32 * 145];
  const RepackTile tl = tiles[blockIdx.x];
  const RepackJob j = jobs[tl.job];
  const int n0 = (int)tl.n0, c0 = (int)tl.c0, nr = min(16, j.Cout - n0), nc = min(32, j.Cin - c0);
  if (j.kind == 0) {  // src rows n: [Cin][9] contiguous; T[r][cl][t] at r * 288 + cl * 9 + t
    for (int e = threadIdx.x; e < 16 * 288; e += 256) {
      const int r = e / 288, q = e - r * 288;
      if (r < nr && q < nc * 9) T[e] = j.src[((size_t)(n0 + r) * j.Cin + c0) * 9 + q];
    }
  } else {  // src [Cin][Cout][9]: per channel c, rows n0 .. n0 + 15 contiguous; T[cl][r][t] at cl * 145 + r * 9 + t
    for (int e = threadIdx.x; e < 32 * 144; e += 256) {
      const int cl = e / 144, q = e - cl * 144;
      if (cl < nc && q < nr * 9) T[cl * 145 + q] = j.src[((size_t)(c0 + cl) * j.Cout + n0) * 9 + q];
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 16 * 9 * 32; e += 256) {
    const int cl = e & 31, t = (e >> 5) % 9, r = e / 288;
    if (r < nr && cl < nc) {
      const float v = j.kind == 0 ? T[r * 288 + cl * 9 + t] : T[cl * 145 + r * 9 + (8 - t)];
      j.dst[(size_t)(n0 + r) * j.Kpad + t * j.Cin + c0 + cl] = v;
    }
  }
}
static __global__ __launch_bounds__(256) void copy_batch_kernel(const CopyJob* jobs, const BatchChunk* chunks) {
  const BatchChunk c = chunks[blockIdx.x];
  const CopyJob j = jobs[c.job];
  const size_t end = min(j.n, (size_t)c.first + BATCH_CHUNK);
  for (size_t i = (size_t)c.first + threadIdx.x; i < end; i += 256) j.dst[i] = j.src[i];
}

// Transpose [R][Cc] -> [Cc][R] (embedding weights for coalesced access).
static __global__ void transpose_kernel(float* dst, const float* src, int R, int Cc) {
  const size_t total = (size_t)R * Cc;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / Cc), c = (int)(i % Cc);
    dst[(size_t)c * R + r] = src[i];
  }
}

// Latent-channel frames of generate_steps.py:47-64 (save_latent_channels_by_dir): per (sample,
// channel) min-max normalisation ch_norm = (ch - min) / (max - min) (0 where max == min), then
// numpy's (ch_norm * 255).astype(uint8) (float32 product, truncation toward zero).  One rounding
// per reference op (IEEE division), so the bytes equal the reference's.  One block per (n, c).
static __global__ __launch_bounds__(256) void latent_frames_kernel(const float* z, uint8_t* out, int HW) {
  __shared__ float smin[256], smax[256];
  const float* ch = z + (size_t)blockIdx.x * HW;
  float lo = 3.402823466e38f, hi = -3.402823466e38f;
  for (int i = threadIdx.x; i < HW; i += 256) {
    const float v = ch[i];
    lo = fminf(lo, v);
    hi = fmaxf(hi, v);
  }
  smin[threadIdx.x] = lo;
  smax[threadIdx.x] = hi;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      smin[threadIdx.x] = fminf(smin[threadIdx.x], smin[threadIdx.x + s]);
      smax[threadIdx.x] = fmaxf(smax[threadIdx.x], smax[threadIdx.x + s]);
    }
    __syncthreads();
  }
  lo = smin[0];
  hi = smax[0];
  const float den = rnd(hi - lo);
  for (int i = threadIdx.x; i < HW; i += 256) {
    const float nrm = hi > lo ? rnd(ch[i] - lo) / den : 0.f;
    out[(size_t)blockIdx.x * HW + i] = (uint8_t)rnd(nrm * 255.f);
  }
}

static __global__ void decrement_t_kernel(int64_t* t) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *t = *t - 1;
}

}  // namespace dmx
