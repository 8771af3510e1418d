// dmx — backward kernels of the U-Net training step (train_latent_cond.py:136-163
// forward / backward of UnetCondWithGeomHead, models/unet_cond.py + models/unet_cond_geom.py).
//
// Layout as the forward: activations NHWC fp32, GroupNorm(1, C) per sample, LayerNorm per token.
// Every reduction runs in a fixed order (per-block partials, then a fixed-order sum), so a
// backward pass is deterministic run to run.  Exact fp32 arithmetic throughout (the GEMM-shaped
// parts run on the fp32 MFMA path: igemm_f32 for the data gradients, wgrad_kernel below for the
// weight gradients).
#pragma once
#include "common.h"

namespace dmx {

DMX_DEV float gelu_grad(float x) {  // d/dx 0.5 x (1 + erf(x / sqrt 2)) = Phi(x) + x phi(x)
  return 0.5f * (1.0f + erff(x * 0.70710678118654752440f)) + x * 0.39894228040143267794f * expf(-0.5f * x * x);
}
DMX_DEV float silu_grad(float x) {
  const float s = 1.0f / (1.0f + expf(-x));
  return s * (1.0f + x * (1.0f - s));
}

// ---------------------------------------------------------------------------
// GroupNorm(1, C) backward, fused with what followed the normalisation in the forward
// (kernels.h norm_kernel):  y = GN(r);  out = act ? GELU(y) : res ? GELU(res + y) : y;  out += emb.
// Pass A (one block per sample): recompute the sample statistics from the conv epilogue's
// partials (same order as the forward), dy = dout * GELU'(pre), and reduce the sample sums
// S1 = sum(gamma dy), S2 = sum(gamma dy xhat) plus per-(sample, channel) partials of
// dgamma = sum(dy xhat), dbeta = sum(dy), demb = sum(dout).  Pass B (grid (chunks, N)):
// dr = rstd (gamma dy - S1/cnt - xhat S2/cnt); dres += dy (residual blocks).
// ---------------------------------------------------------------------------
struct GnBwdParams {
  const float* r;        // raw conv output [N][HW][C]
  const float2* rowpart; int nseg; int rrows;  // forward GroupNorm partials (stats recomputed)
  const float* gamma; const float* beta;
  const float* res;      // residual input of a residual ResBlock (or null)
  int act;               // 1: out = GELU(y)
  const float* dout;     // [N][HW][C]
  int C, HW;
  float* dr;             // [N][HW][C]
  float* dres;           // residual gradient dy (res != null): dres_mode 1 writes, 2 accumulates
  int dres_mode;
  float* chpart;         // [N][2][C]: per-sample dgamma, dbeta sums (pass B out)
  float* demb; int demb_stride, demb_off;  // or null: demb[n][off + c] = sum over pixels of dout
  int chunks, ppb;       // pass A: blocks per sample, pixels per block
  double* bsum;          // [N][chunks][2] block partials of S1, S2
  float* bch;            // [N][chunks][3][C] block partials of dgamma, dbeta, demb
  unsigned* amax_part;   // or null: per-block max |dr| ([N][gridDim.x], absmax_part_kernel's format) — the
                         // device-side operand scale of the x3 weight / data gradients that read dr
};

DMX_DEV float2 gn_stats_from_rowpart(const GnBwdParams& p, int n, double* red) {
  // identical reduction to norm_kernel's (kernels.h): per-thread double sums, wave shuffles, 4 waves
  const int tid = threadIdx.x;
  const int cnt = p.rrows * p.nseg;
  const float2* rp = p.rowpart + (size_t)n * cnt;
  double s1 = 0.0, s2 = 0.0;
  for (int i = tid; i < cnt; i += 256) {
    const float2 q = rp[i];
    s1 += (double)q.x;
    s2 += (double)q.y;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s1 += __shfl_xor(s1, o, 64);
    s2 += __shfl_xor(s2, o, 64);
  }
  __syncthreads();
  if ((tid & 63) == 0) {
    red[tid >> 6] = s1;
    red[4 + (tid >> 6)] = s2;
  }
  __syncthreads();
  const double cntd = (double)p.HW * (double)p.C;
  const double mean = ((red[0] + red[1]) + (red[2] + red[3])) / cntd;
  double var = ((red[4] + red[5]) + (red[6] + red[7])) / cntd - mean * mean;
  var = var < 0.0 ? 0.0 : var;
  return make_float2((float)mean, (float)(1.0 / sqrt(var + 1e-5)));
}

// dy = dLoss/d(GroupNorm output) from loaded values: dout through the GELU (+ residual) that followed the
// normalisation in the forward (kernels.h norm_kernel)
DMX_DEV float gn_dy_v(const GnBwdParams& p, float xh, float g, float bt, float d, float rs, float& dres_out) {
  const float y = xh * g + bt;
  dres_out = 0.f;
  if (p.res != nullptr) {
    const float dy = d * gelu_grad(rs + y);
    dres_out = dy;
    return dy;
  }
  if (p.act) return d * gelu_grad(y);
  return d;
}

// Pass A, grid (chunks, N): block b of sample n takes pixels [b ppb, (b + 1) ppb).  Thread ->
// (4 channels, pixels): channels 4 (tid % L4) .. + 3 with L4 = C / 4 (<= 128), pixels tid / L4 + k
// (256 / L4); float4 loads along coalesced rows.  Block partials are combined in a fixed order by
// gn_bwd_apply_kernel.
static __global__ __launch_bounds__(256) void gn_bwd_reduce_kernel(const GnBwdParams p) {
  __shared__ double red[8];
  __shared__ float tg[3][4][256];
  __shared__ double sr[8];
  const int n = blockIdx.y, b = blockIdx.x, tid = threadIdx.x;
  const float2 st = gn_stats_from_rowpart(p, n, red);
  const int L4 = p.C / 4, c4 = tid % L4, p0 = tid / L4, pstep = 256 / L4, c = 4 * c4;
  const size_t base = (size_t)n * p.HW * p.C;
  const int pbeg = b * p.ppb, pend = min(p.HW, pbeg + p.ppb);
  const floatx4 g4 = *reinterpret_cast<const floatx4*>(p.gamma + c), bt4 = *reinterpret_cast<const floatx4*>(p.beta + c);
  float s1 = 0.f, s2 = 0.f;
  floatx4 g1 = {0.f, 0.f, 0.f, 0.f}, b1 = g1, e1 = g1;
  for (int pix = pbeg + p0; pix < pend; pix += pstep) {
    const size_t idx = base + (size_t)pix * p.C + c;
    const floatx4 r4 = *reinterpret_cast<const floatx4*>(p.r + idx), d4 = *reinterpret_cast<const floatx4*>(p.dout + idx);
    const floatx4 rs4 = p.res != nullptr ? *reinterpret_cast<const floatx4*>(p.res + idx) : floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float xh = (r4[j] - st.x) * st.y;
      float dres;
      const float dy = gn_dy_v(p, xh, g4[j], bt4[j], d4[j], rs4[j], dres);
      const float gd = g4[j] * dy;
      s1 += gd;
      s2 += gd * xh;
      g1[j] += dy * xh;
      b1[j] += dy;
      e1[j] += d4[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    tg[0][j][tid] = g1[j];
    tg[1][j][tid] = b1[j];
    tg[2][j][tid] = e1[j];
  }
  double d1 = s1, d2 = s2;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    d1 += __shfl_xor(d1, o, 64);
    d2 += __shfl_xor(d2, o, 64);
  }
  if ((tid & 63) == 0) {
    sr[tid >> 6] = d1;
    sr[4 + (tid >> 6)] = d2;
  }
  __syncthreads();
  const size_t blk = (size_t)n * p.chunks + b;
  if (tid == 0) {
    p.bsum[2 * blk] = (sr[0] + sr[1]) + (sr[2] + sr[3]);
    p.bsum[2 * blk + 1] = (sr[4] + sr[5]) + (sr[6] + sr[7]);
  }
  // per-channel sums over the threads sharing a channel group, in thread order (deterministic)
  for (int cc = tid; cc < p.C; cc += 256) {
    const int q = cc >> 2, j = cc & 3;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f;
    for (int t = q; t < 256; t += L4) {
      a0 += tg[0][j][t];
      a1 += tg[1][j][t];
      a2 += tg[2][j][t];
    }
    float* o = p.bch + blk * 3 * p.C;
    o[cc] = a0;
    o[p.C + cc] = a1;
    o[2 * p.C + cc] = a2;
  }
}

// Pass B, grid (achunks, N): the block partials of pass A -> per-sample S1, S2 (wave 0: lanes over the
// chunks in double, then a fixed shuffle tree), block 0 of each sample also writes the dgamma / dbeta
// rows and the emb gradient (chunk order); then dr = rstd (gamma dy - S1/cnt - xhat S2/cnt), dres.
static __global__ __launch_bounds__(256) void gn_bwd_apply_kernel(const GnBwdParams p) {
  __shared__ double red[8];
  __shared__ float s12[2];
  const int n = blockIdx.y, tid = threadIdx.x;
  if (tid < 64) {
    double a = 0.0, b = 0.0;
    for (int k = tid; k < p.chunks; k += 64) {
      a += p.bsum[2 * ((size_t)n * p.chunks + k)];
      b += p.bsum[2 * ((size_t)n * p.chunks + k) + 1];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      a += __shfl_xor(a, o, 64);
      b += __shfl_xor(b, o, 64);
    }
    if (tid == 0) {
      s12[0] = (float)a;
      s12[1] = (float)b;
    }
  }
  if (blockIdx.x == 0) {
    for (int c = tid; c < p.C; c += 256) {
      float a0 = 0.f, a1 = 0.f, a2 = 0.f;
      for (int k = 0; k < p.chunks; ++k) {
        const float* o = p.bch + ((size_t)n * p.chunks + k) * 3 * p.C;
        a0 += o[c];
        a1 += o[p.C + c];
        a2 += o[2 * p.C + c];
      }
      p.chpart[((size_t)n * 2 + 0) * p.C + c] = a0;
      p.chpart[((size_t)n * 2 + 1) * p.C + c] = a1;
      if (p.demb != nullptr) p.demb[(size_t)n * p.demb_stride + p.demb_off + c] = a2;
    }
  }
  const float2 st = gn_stats_from_rowpart(p, n, red);  // (its barriers also publish s12)
  const float cnt = (float)p.HW * (float)p.C;
  const float m1 = s12[0] / cnt, m2 = s12[1] / cnt;
  const size_t base = (size_t)n * p.HW * p.C;
  const int per = p.HW * p.C;
  float mx = 0.f;
  for (int i4 = blockIdx.x * 256 + tid; i4 < per / 4; i4 += gridDim.x * 256) {  // float4 along the rows
    const int c = (4 * i4) % p.C;
    const size_t idx = base + 4 * (size_t)i4;
    const floatx4 r4 = *reinterpret_cast<const floatx4*>(p.r + idx), d4 = *reinterpret_cast<const floatx4*>(p.dout + idx);
    const floatx4 rs4 = p.res != nullptr ? *reinterpret_cast<const floatx4*>(p.res + idx) : floatx4{0.f, 0.f, 0.f, 0.f};
    const floatx4 g4 = *reinterpret_cast<const floatx4*>(p.gamma + c), bt4 = *reinterpret_cast<const floatx4*>(p.beta + c);
    floatx4 o4, q4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float xh = (r4[j] - st.x) * st.y;
      float dres;
      const float dy = gn_dy_v(p, xh, g4[j], bt4[j], d4[j], rs4[j], dres);
      o4[j] = st.y * (g4[j] * dy - m1 - xh * m2);
      q4[j] = dres;
      mx = fmaxf(mx, fabsf(o4[j]));
    }
    *reinterpret_cast<floatx4*>(p.dr + idx) = o4;
    if (p.dres_mode == 1) {
      *reinterpret_cast<floatx4*>(p.dres + idx) = q4;
    } else if (p.dres_mode == 2) {
      floatx4 a4 = *reinterpret_cast<const floatx4*>(p.dres + idx);
#pragma unroll
      for (int j = 0; j < 4; ++j) a4[j] += q4[j];
      *reinterpret_cast<floatx4*>(p.dres + idx) = a4;
    }
  }
  if (p.amax_part != nullptr) {
    __shared__ float wm[4];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    if ((tid & 63) == 0) wm[tid >> 6] = mx;
    __syncthreads();
    if (tid == 0)
      p.amax_part[(size_t)n * gridDim.x + blockIdx.x] = __float_as_uint(fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3])));
  }
}

// Column sums: out[y][c] (+)= sum over rows [y rpb, min(R, (y + 1) rpb)) of in[r * stride + c];
// grid (cdiv(C, 64), row blocks), 4 row groups x 64 columns per block, combined in a fixed order.
// out_b != nullptr: columns >= cb go to out_b[c - cb] (two adjacent column ranges of one table, e.g. the
// GroupNorm / LayerNorm gamma and beta gradients, summed by one launch)
DMX_DEV void colsum_body(const float* in, int R, int C, size_t stride, int rpb, float* out, int accumulate,
                         float* out_b, int cb, int bx, int by) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6, c = bx * 64 + cl;
  const int r0 = by * rpb, r1 = min(R, r0 + rpb);
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;  // 4 independent chains keep loads in flight
  if (c < C) {
    int r = r0 + rg;
    for (; r + 12 < r1; r += 16) {
      s0 += in[(size_t)r * stride + c];
      s1 += in[(size_t)(r + 4) * stride + c];
      s2 += in[(size_t)(r + 8) * stride + c];
      s3 += in[(size_t)(r + 12) * stride + c];
    }
    for (; r < r1; r += 4) s0 += in[(size_t)r * stride + c];
  }
  red[rg][cl] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (rg == 0 && c < C) {
    const float v = (red[0][cl] + red[1][cl]) + (red[2][cl] + red[3][cl]);
    float* o = (out_b != nullptr && c >= cb) ? out_b + (c - cb) : out + (size_t)by * C + c;
    *o = accumulate ? *o + v : v;
  }
}
static __global__ __launch_bounds__(256) void colsum_kernel(const float* in, int R, int C, size_t stride, int rpb,
                                                          float* out, int accumulate, float* out_b = nullptr,
                                                          int cb = 0) {
  colsum_body(in, R, C, stride, rpb, out, accumulate, out_b, cb, blockIdx.x, blockIdx.y);
}
// The backward's final-level column sums (parameter gradients nothing in the backward reads again —
// GroupNorm / LayerNorm gamma and beta, biases), deferred to the end of the pass and run COLSUM_BATCH
// per launch (blockIdx.y = job; each job one row block, the same per-column order as colsum_kernel)
constexpr int COLSUM_BATCH = 16;
struct ColsumJob {
  const float* in; float* outa; float* outb; size_t stride; int rows, C, cb;
};
struct ColsumBatch {
  ColsumJob j[COLSUM_BATCH];
};
static __global__ __launch_bounds__(256) void colsum_batch_kernel(const ColsumBatch b) {
  const ColsumJob& j = b.j[blockIdx.y];
  if ((int)blockIdx.x * 64 >= j.C) return;
  colsum_body(j.in, j.rows, j.C, j.stride, j.rows, j.outa, 0, j.outb, j.cb, blockIdx.x, 0);
}

// ---------------------------------------------------------------------------
// LayerNorm backward (nn.LayerNorm over C, eps 1e-5; kernels.h layernorm_kernel): one wave per
// token.  dx (+)= rstd (gamma dy - mean(gamma dy) - xhat mean(gamma dy xhat)); per-block
// partials of dgamma / dbeta ([blocks][2][C], summed later by colsum_kernel).
// ---------------------------------------------------------------------------
template <int CPL>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* x, const float* w, const float* dy, float* dx,
                                                     int accumulate, float* part, int M) {
  constexpr int C = CPL * 64;
  __shared__ float pg[4][C], pb[4][C];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float ag[CPL], ab[CPL];  // this lane's dgamma / dbeta partials over the wave's rows
#pragma unroll
  for (int j = 0; j < CPL; ++j) ag[j] = ab[j] = 0.f;
  for (int row = blockIdx.x * 4 + wv; row < M; row += gridDim.x * 4) {
    float v[CPL], g[CPL];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      v[j] = x[(size_t)row * C + lane + 64 * j];
      s += v[j];
    }
    const float mean = wave_sum(s) / (float)C;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const float d = v[j] - mean;
      q += d * d;
    }
    const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)C + 1e-5f);
    float a1 = 0.f, a2 = 0.f;
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const int c = lane + 64 * j;
      const float xh = (v[j] - mean) * rstd;
      g[j] = dy[(size_t)row * C + c];
      const float gd = g[j] * w[c];
      a1 += gd;
      a2 += gd * xh;
      ag[j] += g[j] * xh;
      ab[j] += g[j];
    }
    const float m1 = wave_sum(a1) / (float)C, m2 = wave_sum(a2) / (float)C;
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const int c = lane + 64 * j;
      const float xh = (v[j] - mean) * rstd;
      const float r = rstd * (g[j] * w[c] - m1 - xh * m2);
      float* o = dx + (size_t)row * C + c;
      *o = accumulate ? *o + r : r;
    }
  }
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    pg[wv][lane + 64 * j] = ag[j];
    pb[wv][lane + 64 * j] = ab[j];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    part[((size_t)blockIdx.x * 2 + 0) * C + c] = (pg[0][c] + pg[1][c]) + (pg[2][c] + pg[3][c]);
    part[((size_t)blockIdx.x * 2 + 1) * C + c] = (pb[0][c] + pb[1][c]) + (pb[2][c] + pb[3][c]);
  }
}

// ---------------------------------------------------------------------------
// Weight gradient of an implicit GEMM (conv3x3 pad 1 or Linear):
//   dW[co][k] = sum_m dY[m][co] * A[m][k],  A[m][k] = X at row m's tap (k = tap * Cin + ci)
// on fp32 MFMA (v_mfma_f32_32x32x2_f32): block tile 64 (co) x 64 (k), 4 waves 2 x 2, the rows m
// split into `splits` slabs (blockIdx.z) written to part[split][Cout][K]; wgrad_finish_kernel
// sums the slabs in split order and scatters to the torch layout [Cout][Cin][3][3] / [Cout][Cin].
// ---------------------------------------------------------------------------
struct WgradParams {
  const float* dy;   // [M][Cout]
  const float* x;    // [N][H][W][Cin] (NHWC)
  int N, H, W, Cin, Cout, taps;  // taps 9 (conv3x3) or 1 (linear)
  int M, K;          // M = N*H*W rows, K = taps * Cin
  int rows_per_split;
  float* part;       // [splits][Cout][K]
  float* bpart;      // wgrad_x3_kernel: [splits][Cout] column sums of dY (bias gradient), or null
  // wgrad_x3_kernel (the f16 matrix cores, x3 split, fp32 accumulate): dY scaled on the device by 2^ea
  // from its max (dy_nparts per-block partial maxima, absmax_part_kernel); X (tape activations, O(1))
  // split as is
  const unsigned* dy_amax;
  int dy_nparts;
};

static __global__ __launch_bounds__(256) void wgrad_kernel(const WgradParams p) {
  constexpr int MK = 16;  // rows per LDS tile
  __shared__ float dys[MK][64 + 4];
  __shared__ float xs[MK][64 + 4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wm = wv >> 1, wn = wv & 1;
  const int co0 = blockIdx.x * 64, k0 = blockIdx.y * 64;
  const int mbeg = blockIdx.z * p.rows_per_split, mend = min(p.M, mbeg + p.rows_per_split);
  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  const int HW = p.H * p.W;
  for (int m0 = mbeg; m0 < mend; m0 += MK) {
    // stage 16 rows x 64 co of dY and 16 rows x 64 k of the tapped input
    for (int i = tid; i < MK * 64; i += 256) {
      const int r = i >> 6, c = i & 63, m = m0 + r;
      const int co = co0 + c, k = k0 + c;
      dys[r][c] = (m < mend && co < p.Cout) ? p.dy[(size_t)m * p.Cout + co] : 0.f;
      float xv = 0.f;
      if (m < mend && k < p.K) {
        const int tap = k / p.Cin, ci = k - tap * p.Cin;
        const int n = m / HW, rr = m - n * HW, y = rr / p.W, xx = rr - y * p.W;
        int iy = y, ix = xx;
        if (p.taps == 9) {
          iy = y + tap / 3 - 1;
          ix = xx + tap % 3 - 1;
        }
        if (iy >= 0 && iy < p.H && ix >= 0 && ix < p.W) xv = p.x[(((size_t)n * p.H + iy) * p.W + ix) * p.Cin + ci];
      }
      xs[r][c] = xv;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < MK; s += 2) {
      const float a = dys[s + (lane >> 5)][wm * 32 + (lane & 31)];
      const float b = xs[s + (lane >> 5)][wn * 32 + (lane & 31)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    __syncthreads();
  }
  float* dst = p.part + (size_t)blockIdx.z * p.Cout * p.K;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int co = co0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    const int k = k0 + wn * 32 + (lane & 31);
    if (co < p.Cout && k < p.K) dst[(size_t)co * p.K + k] = acc[r];
  }
}

// Weight gradient on the f16 matrix cores (x3 split, fp32 accumulate): block tile CO (64 or 128) Cout x
// 128 K, 2 x 2 waves of CO/2 x 64, 32-row stages, double-buffered, with the staged rows split once into
// f16 hi / lo planes kept row-major in LDS ([m][co], [m][k]) and the MFMA operands — contraction over m,
// 8 consecutive rows per lane — read with ds_read_b64_tr_b16: per 16-lane group a 4-row x 16-column
// block, lane 4q + p addressing row q, columns 4p .. 4p + 3, lane i receiving column i (MI355X guide
// T10).  dY is multiplied by 2^ea (its max |dY| 2^ea in [2^12, 2^13): the lo parts stay f16-normal) and
// the slabs by 2^-ea.  Row pitches of CO + 32 / 160 halves (48 or 80 banks: the 4 rows of a block on 4
// disjoint 16-bank ranges) make the transposed reads conflict-free.  CO = 128 (Cout % 128 == 0) stages
// each X row once for twice the MFMA work of CO = 64 (the split and im2col VALU per product halve).
// The bias gradient (column sums of dY) is summed from the staged registers: lanes, then the 4 waves
// in a fixed order.
constexpr int WG_BM = 32;  // rows per stage
typedef __fp16 fp16x4_t __attribute__((__vector_size__(4 * sizeof(__fp16))));
DMX_DEV half4 lds_tr16(const _Float16* p) {
  return __builtin_bit_cast(half4, __builtin_amdgcn_ds_read_tr16_b64_v4f16(
                                       (__attribute__((address_space(3))) fp16x4_t*)(p)));
}
template <int CO>
static __global__ __launch_bounds__(256) void wgrad_x3_kernel(const WgradParams p) {
  constexpr int DP = CO + 32, XP = 160;  // plane row pitches (halves)
  constexpr int MT = CO / 64;            // 32-row m-tiles per wave
  constexpr int DL = CO / 4;             // lanes per dY row (one float4 each)
  constexpr int DR = 256 / DL;           // dY rows per pass
  constexpr int DI = WG_BM / DR;         // dY float4 per thread per stage
  __shared__ __attribute__((aligned(16))) _Float16 Dh[2][WG_BM][DP];
  __shared__ __attribute__((aligned(16))) _Float16 Dl[2][WG_BM][DP];
  __shared__ __attribute__((aligned(16))) _Float16 Xh[2][WG_BM][XP];
  __shared__ __attribute__((aligned(16))) _Float16 Xl[2][WG_BM][XP];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wm = wv >> 1, wn = wv & 1;
  const int co0 = blockIdx.x * CO, k0 = blockIdx.y * 128;
  const int mbeg = blockIdx.z * p.rows_per_split, mend = min(p.M, mbeg + p.rows_per_split);
  const int HW = p.H * p.W;
  const float rhw = 1.f / (float)HW, rw = 1.f / (float)p.W;
  const int dr = tid / DL, dc = (tid % DL) * 4;  // dY: rows dr + DR i (i < DI), float4 dc
  const int xr = tid >> 5, xc = (tid & 31) * 4;  // X: rows xr + 8 i (i < 4), float4 xc
  const int k = k0 + xc;
  const bool kvalid = k < p.K;
  const int tap = kvalid ? k / p.Cin : 0, ci = k - tap * p.Cin;
  const int ty = p.taps == 9 ? tap / 3 - 1 : 0, tx = p.taps == 9 ? tap % 3 - 1 : 0;
  unsigned mb = 0u;
  for (int i = lane; i < p.dy_nparts; i += 64) mb = max(mb, p.dy_amax[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mb = max(mb, (unsigned)__shfl_xor((int)mb, o, 64));
  const int ea = amax_exp(mb);
  const float a_sc = ldexpf(1.f, ea), o_sc = ldexpf(1.f, -ea);
  const bool bias = p.bpart != nullptr && blockIdx.y == 0;
  floatx4 bs = {0.f, 0.f, 0.f, 0.f};  // column sums of dY (columns dc .. dc + 3) over this thread's rows
  floatx4 rdv[2][DI], rxv[2][4];      // two register stages (the loads run two 32-row stages ahead)
  auto load = [&](int m0, int rs) {
    floatx4(&rd)[DI] = rdv[rs];
    floatx4(&rx)[4] = rxv[rs];
#pragma unroll
    for (int i = 0; i < DI; ++i) {
      const int m = m0 + dr + DR * i;
      rd[i] = m < mend ? *reinterpret_cast<const floatx4*>(p.dy + (size_t)m * p.Cout + co0 + dc)
                       : floatx4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + xr + 8 * i;
      floatx4 v = {0.f, 0.f, 0.f, 0.f};
      if (m < mend && kvalid) {
        // (division by HW and W through the float reciprocal plus one correction step: exact for the
        // M < 2^24 rows here)
        int n = (int)((float)m * rhw), rr = m - n * HW;
        if (rr < 0) { --n; rr += HW; } else if (rr >= HW) { ++n; rr -= HW; }
        int y = (int)((float)rr * rw), xx = rr - y * p.W;
        if (xx < 0) { --y; xx += p.W; } else if (xx >= p.W) { ++y; xx -= p.W; }
        const int iy = y + ty, ix = xx + tx;
        if (iy >= 0 && iy < p.H && ix >= 0 && ix < p.W)
          v = *reinterpret_cast<const floatx4*>(p.x + (((size_t)n * p.H + iy) * p.W + ix) * p.Cin + ci);
      }
      rx[i] = v;
    }
  };
  auto store = [&](int b, int rs) {
    floatx4(&rd)[DI] = rdv[rs];
    floatx4(&rx)[4] = rxv[rs];
#pragma unroll
    for (int i = 0; i < DI; ++i) {
      if (bias) bs += rd[i];
      floatx4 v = rd[i];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] *= a_sc;
      half4 h, l;
      split4(v, h, l);
      *reinterpret_cast<half4*>(&Dh[b][dr + DR * i][dc]) = h;
      *reinterpret_cast<half4*>(&Dl[b][dr + DR * i][dc]) = l;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      half4 h, l;
      split4(rx[i], h, l);
      *reinterpret_cast<half4*>(&Xh[b][xr + 8 * i][xc]) = h;
      *reinterpret_cast<half4*>(&Xl[b][xr + 8 * i][xc]) = l;
    }
  };
  floatx16 acc[MT][2];
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][j][r] = 0.f;
  // transposed-read addressing: group g = lane / 16 (rows + 8 for g >= 2, columns + 16 for odd g),
  // lane 4q + p of the group -> row q, columns 4p .. 4p + 3
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const int trow = 8 * (g >> 1) + q, tcol = 16 * (g & 1) + 4 * pp;
  const int nst = (mend - mbeg + WG_BM - 1) / WG_BM;
  auto compute = [&](int b) {
#pragma unroll
    for (int s = 0; s < WG_BM; s += 16) {
      const int r0 = s + trow;
      half8 ah[MT], al[MT];
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int cd = wm * (CO / 2) + 32 * t + tcol;
        const half4 a0 = lds_tr16(&Dh[b][r0][cd]), a1 = lds_tr16(&Dh[b][r0 + 4][cd]);
        const half4 c0 = lds_tr16(&Dl[b][r0][cd]), c1 = lds_tr16(&Dl[b][r0 + 4][cd]);
        ah[t] = half8{a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
        al[t] = half8{c0[0], c0[1], c0[2], c0[3], c1[0], c1[1], c1[2], c1[3]};
      }
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int cx = wn * 64 + 32 * n + tcol;
        const half4 b0 = lds_tr16(&Xh[b][r0][cx]), b1 = lds_tr16(&Xh[b][r0 + 4][cx]);
        const half4 d0 = lds_tr16(&Xl[b][r0][cx]), d1 = lds_tr16(&Xl[b][r0 + 4][cx]);
        const half8 bh = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
        const half8 bl = {d0[0], d0[1], d0[2], d0[3], d1[0], d1[1], d1[2], d1[3]};
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          acc[t][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[t], bh, acc[t][n], 0, 0, 0);
          acc[t][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[t], bl, acc[t][n], 0, 0, 0);
          acc[t][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[t], bh, acc[t][n], 0, 0, 0);
        }
      }
    }
  };
  // stage st lives in register set st & 1 and LDS buffer st & 1; its loads are issued two stages
  // ahead (before stage st - 2's MFMAs), its store after stage st - 1's MFMAs
  if (nst > 0) load(mbeg, 0);
  if (nst > 1) load(mbeg + WG_BM, 1);
  if (nst > 0) store(0, 0);
  __syncthreads();
  auto body = [&](int st, int rs) {  // rs = st & 1 (compile-time at both call sites)
    if (st + 2 < nst) load(mbeg + (st + 2) * WG_BM, rs);  // (set rs was stored one iteration ago)
    compute(rs);
    if (st + 1 < nst) store(rs ^ 1, rs ^ 1);
    __syncthreads();
  };
  for (int st = 0; st < nst; st += 2) {
    body(st, 0);
    if (st + 1 < nst) body(st + 1, 1);
  }
  if (bias) {  // lanes sharing columns (same tid % DL), then waves 0..3 in order through LDS
#pragma unroll
    for (int o = DL; o < 64; o <<= 1)
#pragma unroll
      for (int e = 0; e < 4; ++e) bs[e] += __shfl_xor(bs[e], o, 64);
    float* red = reinterpret_cast<float*>(&Dh[0][0][0]);  // (the stages are done: last barrier above)
    if (lane < DL) *reinterpret_cast<floatx4*>(&red[wv * CO + dc]) = bs;
    __syncthreads();
    if (tid < CO)
      p.bpart[(size_t)blockIdx.z * p.Cout + co0 + tid] = ((red[tid] + red[CO + tid]) + red[2 * CO + tid]) + red[3 * CO + tid];
  }
  float* dst = p.part + (size_t)blockIdx.z * p.Cout * p.K;
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = co0 + wm * (CO / 2) + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int kk = k0 + wn * 64 + j * 32 + (lane & 31);
        if (kk < p.K) dst[(size_t)co * p.K + kk] = acc[t][j][r] * o_sc;
      }
}

// grad (torch layout) = sum over the split slabs; k = tap * Cin + ci -> [co][ci][tap] (input channels
// >= cin_real — the zero padding of a 3-channel input — are dropped).  64 consecutive elements per
// block, the slabs split over 4 row groups (slab z to group z % 4, four independent load chains per
// thread) and the groups added in a fixed order: deterministic, and ~4x the loads in flight of one
// thread walking all slabs (which left this kernel latency-bound at Cout K / 256 blocks).
static __global__ __launch_bounds__(256) void wgrad_finish_kernel(const float* part, int splits, int Cout, int Cin,
                                                                  int cin_real, int taps, float* grad) {
  __shared__ float red[4][64];
  const int K = taps * Cin;
  const size_t total = (size_t)Cout * K;
  const int cl = threadIdx.x & 63, zg = threadIdx.x >> 6;
  const size_t i = (size_t)blockIdx.x * 64 + cl;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (i < total) {
    int z = zg;
    for (; z + 12 < splits; z += 16) {
      s0 += part[(size_t)z * total + i];
      s1 += part[(size_t)(z + 4) * total + i];
      s2 += part[(size_t)(z + 8) * total + i];
      s3 += part[(size_t)(z + 12) * total + i];
    }
    for (; z < splits; z += 4) s0 += part[(size_t)z * total + i];
  }
  red[zg][cl] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (zg == 0 && i < total) {
    const int co = (int)(i / K), k = (int)(i - (size_t)co * K), tap = k / Cin, ci = k - tap * Cin;
    if (ci < cin_real)
      grad[((size_t)co * cin_real + ci) * taps + tap] = (red[0][cl] + red[1][cl]) + (red[2][cl] + red[3][cl]);
  }
}

// ---------------------------------------------------------------------------
// Elementwise / layout helpers.
// ---------------------------------------------------------------------------
// dst (+)= src * GELU'(pre)
static __global__ void gelu_bwd_kernel(const float* d, const float* pre, float* dst, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    dst[i] = d[i] * gelu_grad(pre[i]);
}
static __global__ void gelu_fwd_kernel(const float* x, float* y, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) y[i] = gelu_exact(x[i]);
}
static __global__ void add_kernel(float* dst, const float* src, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) dst[i] += src[i];
}

// max_pool2d(2) backward (floor mode): the gradient goes to the first maximum of each window in
// (0,0), (0,1), (1,0), (1,1) order (strict >, torch's CPU kernel); uncovered rows / columns get 0.
// x: [N][Hs][Ws][C], dy: [N][Hs/2][Ws/2][C]; dx (+)= (accumulate).
static __global__ void maxpool_bwd_kernel(const float* src, const float* dy, float* dx, int N, int Hs, int Ws, int C,
                                          int accumulate) {
  const int Ho = Hs / 2, Wo = Ws / 2;
  const size_t total = (size_t)N * Hs * Ws * C;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
    const int c = (int)(i % C);
    const size_t pix = i / C;
    const int n = (int)(pix / ((size_t)Hs * Ws)), rr = (int)(pix % ((size_t)Hs * Ws)), y = rr / Ws, x = rr % Ws;
    const int oy = y >> 1, ox = x >> 1;
    float g = 0.f;
    if (oy < Ho && ox < Wo) {
      const float* b = src + (((size_t)n * Hs + 2 * oy) * Ws + 2 * ox) * C + c;
      const float v[4] = {b[0], b[C], b[(size_t)Ws * C], b[(size_t)Ws * C + C]};
      int am = 0;
      for (int k = 1; k < 4; ++k)
        if (v[k] > v[am]) am = k;
      if (am == (y & 1) * 2 + (x & 1)) g = dy[(((size_t)n * Ho + oy) * Wo + ox) * C + c];
    }
    dx[i] = accumulate ? dx[i] + g : g;
  }
}

// Up's input backward: dcat [N][H][W][C0 + C1] -> dskip (+)= dcat[..., :C0] and the low-resolution
// map's gradient (+)= bilinear-x2 (align_corners) adjoint of the un-padded dcat[..., C0:].  Gather
// form: each low-res pixel (i, j) sums w_y(oy, i) w_x(ox, j) d(oy, ox) over the output pixels whose
// interpolation touches it (same weights as source.h upsample4).
static __global__ void upcat_bwd_kernel(const float* dcat, float* dskip, float* dlow, int N, int H, int W, int C0,
                                        int C1, int Hs, int Ws, int padT, int padL, int acc_skip, int acc_low) {
  const int C = C0 + C1;
  const size_t tot_skip = (size_t)N * H * W * C0;
  const size_t tot_low = (size_t)N * Hs * Ws * C1;
  const size_t stride = (size_t)gridDim.x * 256;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < tot_skip + tot_low; i += stride) {
    if (i < tot_skip) {
      const int c = (int)(i % C0);
      const size_t pix = i / C0;
      const float g = dcat[pix * C + c];
      dskip[i] = acc_skip ? dskip[i] + g : g;
      continue;
    }
    const size_t j = i - tot_skip;
    const int c = (int)(j % C1);
    const size_t pix = j / C1;
    const int n = (int)(pix / ((size_t)Hs * Ws)), rr = (int)(pix % ((size_t)Hs * Ws)), li = rr / Ws, lj = rr % Ws;
    const int Ho = 2 * Hs, Wo = 2 * Ws;
    const float sh = Ho > 1 ? (float)(Hs - 1) / (float)(Ho - 1) : 0.f;
    const float sw = Wo > 1 ? (float)(Ws - 1) / (float)(Wo - 1) : 0.f;
    float g = 0.f;
    // output rows / columns whose interpolation can touch (li, lj): floor(sh * u) in {li - 1, li}
    const int uy0 = sh > 0.f ? max(0, (int)floorf((float)(li - 1) / sh) - 1) : 0;
    const int uy1 = sh > 0.f ? min(Ho - 1, (int)ceilf((float)(li + 1) / sh) + 1) : Ho - 1;
    const int ux0 = sw > 0.f ? max(0, (int)floorf((float)(lj - 1) / sw) - 1) : 0;
    const int ux1 = sw > 0.f ? min(Wo - 1, (int)ceilf((float)(lj + 1) / sw) + 1) : Wo - 1;
    for (int uy = uy0; uy <= uy1; ++uy) {
      const float fy = sh * (float)uy;
      const int y0 = (int)fy, y1 = y0 + (y0 < Hs - 1 ? 1 : 0);
      const float ly = fminf(fmaxf(fy - (float)y0, 0.f), 1.f), hy = 1.f - ly;
      float wy = 0.f;
      if (y0 == li) wy += hy;
      if (y1 == li) wy += ly;
      if (wy == 0.f) continue;
      const int oy = uy + padT;
      if (oy < 0 || oy >= H) continue;
      for (int ux = ux0; ux <= ux1; ++ux) {
        const float fx = sw * (float)ux;
        const int x0 = (int)fx, x1 = x0 + (x0 < Ws - 1 ? 1 : 0);
        const float lx = fminf(fmaxf(fx - (float)x0, 0.f), 1.f), hx = 1.f - lx;
        float wx = 0.f;
        if (x0 == lj) wx += hx;
        if (x1 == lj) wx += lx;
        if (wx == 0.f) continue;
        const int ox = ux + padL;
        if (ox < 0 || ox >= W) continue;
        g += wy * wx * dcat[(((size_t)n * H + oy) * W + ox) * C + C0 + c];
      }
    }
    dlow[j] = acc_low ? dlow[j] + g : g;
  }
}

// ---------------------------------------------------------------------------
// Multi-head attention core backward on the fp32 matrix cores (v_mfma_f32_16x16x4f32), per
// (sample, head):  P = softmax(Q K^T / sqrt D), O = P V;  given dO:
//   Dlt_i = sum_d dO_i O_i;  dS = P (dO V^T - Dlt);  dQ = dS K / sqrt D;  dK = dS^T Q / sqrt D;  dV = P^T dO.
// P is recomputed from Q, K and the per-query (max m_i, 1 / sum l_i); nothing L x L is stored.
//   attn_dq_mfma_kernel: 64 queries per block, 16 per wave with the query on the lane.  m_i and 1 / l_i
//     come from the training forward (kernels.h attention_kernel writes them to st), or with STATS
//     from a first pass over the keys (online); Dlt_i goes to st.  Then it streams K and V:
//     S^T = K Q^T,  dP^T = V dO^T,  dS^T = P^T (dP^T - Dlt),  dQ^T += K^T dS^T.
//   attn_dkv_mfma_kernel (after it): 64 keys per block, the key on the lane, queries streamed:
//     S = Q K^T,  dP = dO V^T,  dV^T += dO^T P,  dK^T += Q^T dS.
// The 16 x 16 accumulator of one product (lane: column lane % 16, rows 4 (lane / 16) + r) is the B
// operand of the next, contracting over its rows: step r maps k = lane / 16 to row 4 (lane / 16) + r,
// and the A operand is read from LDS with the same mapping (the forward kernel's arrangement,
// kernels.h attention_kernel).  The D-contractions map d = (lane / 16) D/4 + s (contiguous float4 LDS
// reads).  Deterministic: no atomics, fixed summation order.
// qkv: [N][L][3C] (q | k | v, head h at columns h*D), o / dO: [N][L][C]; dqkv: [N][L][3C];
// st: [N][4][L][3].
// ---------------------------------------------------------------------------
template <int D, bool STATS>
__global__ __launch_bounds__(256) void attn_dq_mfma_kernel(const float* qkv, const float* o, const float* dout,
                                                           float* st, float* dqkv, int L, int C) {
  constexpr int KC = 64, PT = D + 4, DP = D / 4, NT = D / 16;
  __shared__ __attribute__((aligned(16))) float Ks[KC][PT];
  __shared__ __attribute__((aligned(16))) float Vs[KC][PT];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, ql = lane & 15, g = lane >> 4;
  const int hd = blockIdx.y, n = blockIdx.z;
  const int qi = blockIdx.x * 64 + w * 16 + ql, qc = min(qi, L - 1);
  const size_t rs = 3 * (size_t)C;
  const float* base = qkv + (size_t)n * L * rs;
  const float sc = 1.0f / sqrtf((float)D);
  float qf[DP], gf[DP];
  float dl = 0.f;
  {
    const float* qr = base + (size_t)qc * rs + hd * D + g * DP;
    const size_t ob = ((size_t)n * L + qc) * C + hd * D + g * DP;
#pragma unroll
    for (int s = 0; s < DP; s += 4) {
      const floatx4 q4 = ld4(qr + s), g4 = ld4(dout + ob + s), o4 = ld4(o + ob + s);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        qf[s + e] = q4[e] * sc;
        gf[s + e] = g4[e];
        dl += g4[e] * o4[e];
      }
    }
  }
  dl += __shfl_xor(dl, 16, 64);
  dl += __shfl_xor(dl, 32, 64);
  auto stage = [&](int c0, bool with_v) {
    for (int i = tid; i < KC * (D / 4); i += 256) {
      const int key = i / (D / 4), d4 = (i % (D / 4)) * 4;
      floatx4 kv = {0.f, 0.f, 0.f, 0.f}, vv = {0.f, 0.f, 0.f, 0.f};
      if (c0 + key < L) {
        const float* r = base + (size_t)(c0 + key) * rs + C + hd * D + d4;
        kv = ld4(r);
        if (with_v) vv = ld4(r + C);
      }
      *reinterpret_cast<floatx4*>(&Ks[key][d4]) = kv;
      if (with_v) *reinterpret_cast<floatx4*>(&Vs[key][d4]) = vv;
    }
  };
  auto dotk = [&](const float (*X)[PT], int row, const float* f) {  // 16 x 16 tile of X Q^T-like products
    floatx4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < DP; s += 4) {
      const floatx4 x4 = *reinterpret_cast<const floatx4*>(&X[row][g * DP + s]);
#pragma unroll
      for (int e = 0; e < 4; ++e) a = __builtin_amdgcn_mfma_f32_16x16x4f32(x4[e], f[s + e], a, 0, 0, 0);
    }
    return a;
  };
  const int nch = (L + KC - 1) / KC;
  float M, il;
  float* so = st + (((size_t)n * 4 + hd) * L + qc) * 3;
  if constexpr (STATS) {
    // per-lane online max / sum over the lane's keys (4 of every 16), then across the 4 lane groups
    float m = -INFINITY, l = 0.f;
    for (int c = 0; c < nch; ++c) {
      const int c0 = c * KC;
      stage(c0, false);
      __syncthreads();
#pragma unroll
      for (int kt = 0; kt < KC / 16; ++kt) {
        if (c0 + kt * 16 >= L) break;
        const floatx4 s4 = dotk(Ks, kt * 16 + ql, qf);
        float mx = -INFINITY;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (c0 + kt * 16 + 4 * g + r < L) mx = fmaxf(mx, s4[r]);
        if (mx > -INFINITY) {
          const float mn = fmaxf(m, mx);
          float a = l * __expf(m - mn);
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (c0 + kt * 16 + 4 * g + r < L) a += __expf(s4[r] - mn);
          l = a;
          m = mn;
        }
      }
      __syncthreads();
    }
    M = fmaxf(m, __shfl_xor(m, 16, 64));
    M = fmaxf(M, __shfl_xor(M, 32, 64));
    float Ls = m > -INFINITY ? l * __expf(m - M) : 0.f;
    Ls += __shfl_xor(Ls, 16, 64);
    Ls += __shfl_xor(Ls, 32, 64);
    il = 1.0f / Ls;
    if (g == 0 && qi < L) {
      so[0] = M;
      so[1] = il;
    }
  } else {
    M = so[0];
    il = so[1];
  }
  if (g == 0 && qi < L) so[2] = dl;
  // pass 2: dQ^T (D x 16 queries per wave) += K^T dS^T over the key tiles
  floatx4 dq[NT];
#pragma unroll
  for (int dt = 0; dt < NT; ++dt) dq[dt] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int c = 0; c < nch; ++c) {
    const int c0 = c * KC;
    stage(c0, true);
    __syncthreads();
#pragma unroll
    for (int kt = 0; kt < KC / 16; ++kt) {
      if (c0 + kt * 16 >= L) break;
      const floatx4 s4 = dotk(Ks, kt * 16 + ql, qf);  // S^T: keys 4g + r, query ql
      const floatx4 p4 = dotk(Vs, kt * 16 + ql, gf);  // dP^T
      float ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float pr = c0 + kt * 16 + 4 * g + r < L ? __expf(s4[r] - M) * il : 0.f;
        ds[r] = pr * (p4[r] - dl);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int dt = 0; dt < NT; ++dt)
          dq[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(Ks[kt * 16 + 4 * g + r][dt * 16 + ql], ds[r], dq[dt], 0, 0, 0);
    }
    __syncthreads();
  }
  if (qi < L) {  // dQ^T tile dt: lane column = query ql, rows d = dt * 16 + 4g + r
    float* dst = dqkv + ((size_t)n * L + qi) * rs + hd * D;
#pragma unroll
    for (int dt = 0; dt < NT; ++dt) {
      floatx4 v = dq[dt];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] *= sc;
      *reinterpret_cast<floatx4*>(dst + dt * 16 + 4 * g) = v;
    }
  }
}

template <int D>
__global__ __launch_bounds__(256) void attn_dkv_mfma_kernel(const float* qkv, const float* dout, const float* st,
                                                            float* dqkv, int L, int C) {
  constexpr int QC = 64, PT = D + 4, DP = D / 4, NT = D / 16;
  __shared__ __attribute__((aligned(16))) float Qs[QC][PT];
  __shared__ __attribute__((aligned(16))) float Gs[QC][PT];
  __shared__ __attribute__((aligned(16))) float Sm[QC], Si[QC], Sd[QC];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, ql = lane & 15, g = lane >> 4;
  const int hd = blockIdx.y, n = blockIdx.z;
  const int kj = blockIdx.x * 64 + w * 16 + ql, kc = min(kj, L - 1);
  const size_t rs = 3 * (size_t)C;
  const float* base = qkv + (size_t)n * L * rs;
  const float* sth = st + ((size_t)n * 4 + hd) * L * 3;
  const float sc = 1.0f / sqrtf((float)D);
  float kf[DP], vf[DP];
  {
    const float* kr = base + (size_t)kc * rs + C + hd * D + g * DP;
#pragma unroll
    for (int s = 0; s < DP; s += 4) {
      const floatx4 k4 = ld4(kr + s), v4 = ld4(kr + C + s);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        kf[s + e] = k4[e];
        vf[s + e] = v4[e];
      }
    }
  }
  floatx4 dk[NT], dv[NT];
#pragma unroll
  for (int dt = 0; dt < NT; ++dt) dk[dt] = dv[dt] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int nch = (L + QC - 1) / QC;
  for (int c = 0; c < nch; ++c) {
    const int c0 = c * QC;
    // queries past L: zero Q / dO rows and 1 / l = 0, so P = dS = 0 there
    for (int i = tid; i < QC * (D / 4); i += 256) {
      const int q = i / (D / 4), d4 = (i % (D / 4)) * 4;
      floatx4 qv = {0.f, 0.f, 0.f, 0.f}, gv = {0.f, 0.f, 0.f, 0.f};
      if (c0 + q < L) {
        qv = ld4(base + (size_t)(c0 + q) * rs + hd * D + d4);
#pragma unroll
        for (int e = 0; e < 4; ++e) qv[e] *= sc;
        gv = ld4(dout + ((size_t)n * L + c0 + q) * C + hd * D + d4);
      }
      *reinterpret_cast<floatx4*>(&Qs[q][d4]) = qv;
      *reinterpret_cast<floatx4*>(&Gs[q][d4]) = gv;
    }
    if (tid < QC) {
      const bool ok = c0 + tid < L;
      Sm[tid] = ok ? sth[(size_t)(c0 + tid) * 3] : 0.f;
      Si[tid] = ok ? sth[(size_t)(c0 + tid) * 3 + 1] : 0.f;
      Sd[tid] = ok ? sth[(size_t)(c0 + tid) * 3 + 2] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int qt = 0; qt < QC / 16; ++qt) {
      if (c0 + qt * 16 >= L) break;
      floatx4 s4 = {0.f, 0.f, 0.f, 0.f}, p4 = {0.f, 0.f, 0.f, 0.f};  // S, dP: queries 4g + r, key ql
#pragma unroll
      for (int s = 0; s < DP; s += 4) {
        const floatx4 q4 = *reinterpret_cast<const floatx4*>(&Qs[qt * 16 + ql][g * DP + s]);
        const floatx4 g4 = *reinterpret_cast<const floatx4*>(&Gs[qt * 16 + ql][g * DP + s]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s4 = __builtin_amdgcn_mfma_f32_16x16x4f32(q4[e], kf[s + e], s4, 0, 0, 0);
          p4 = __builtin_amdgcn_mfma_f32_16x16x4f32(g4[e], vf[s + e], p4, 0, 0, 0);
        }
      }
      const int q0 = qt * 16 + 4 * g;
      const floatx4 mq = *reinterpret_cast<const floatx4*>(&Sm[q0]);
      const floatx4 iq = *reinterpret_cast<const floatx4*>(&Si[q0]);
      const floatx4 dq = *reinterpret_cast<const floatx4*>(&Sd[q0]);
      float pr[4], ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pr[r] = __expf(s4[r] - mq[r]) * iq[r];
        ds[r] = pr[r] * (p4[r] - dq[r]);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int dt = 0; dt < NT; ++dt) {
          dv[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(Gs[q0 + r][dt * 16 + ql], pr[r], dv[dt], 0, 0, 0);
          dk[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(Qs[q0 + r][dt * 16 + ql], ds[r], dk[dt], 0, 0, 0);
        }
    }
    __syncthreads();
  }
  if (kj < L) {  // dK^T / dV^T tile dt: lane column = key ql, rows d = dt * 16 + 4g + r (Qs carries 1/sqrt D)
    float* dst = dqkv + ((size_t)n * L + kj) * rs + hd * D;
#pragma unroll
    for (int dt = 0; dt < NT; ++dt) {
      *reinterpret_cast<floatx4*>(dst + C + dt * 16 + 4 * g) = dk[dt];
      *reinterpret_cast<floatx4*>(dst + 2 * C + dt * 16 + 4 * g) = dv[dt];
    }
  }
}

// ---------------------------------------------------------------------------
// Small dense layers (embedding MLPs, emb heads, GeomHead; R = the batch, a few hundred rows at most):
//   forward y = x W^T + b over [R][K] -> [R][O]; backward dW = dY^T X, db = sum_r dY, dX = dY W.
// All three are one strided small GEMM  C[i][j] = sum_l A(i, l) B(l, j),  A(i, l) = a[i sai + l sal],
// B(l, j) = b[l sbl + j sbj]: 32 x 32 output tiles per 256-thread block (4 outputs per thread), the l
// range in 32-deep chunks staged through LDS, split over grid.z where the output tiles alone leave the
// chip empty (the emb heads' dX: 8 tiles, l = 1024 deep); each split writes its own partial slab and
// small_gemm_finish_kernel adds the slabs in split order (+ bias, + accumulate).  Every output is a
// fixed-order fp32 sum: deterministic.  (The previous one-thread-per-output kernels ran 32-block grids
// with stride-K weight reads: 46 us per emb-head dX.)
// ---------------------------------------------------------------------------
struct SmallGemm {
  const float* a;
  const float* b;
  long sai, sal, sbl, sbj;
  int I, J, L, lsplit;  // lsplit: l per split (grid.z splits)
  float* c;             // splits == 1: output [I][ldc] (+ bias, accumulate); else partial [z][I][J]
  int ldc;
  const float* bias;    // [J] or null
  int accumulate;
};
static __global__ __launch_bounds__(256) void small_gemm_kernel(const SmallGemm g) {
  __shared__ float As[32][33], Bs[32][33];  // [l][i], [l][j]
  const int tid = threadIdx.x, tj = tid & 31, ti = tid >> 5;  // outputs (4 ti + q, tj)
  const int i0 = blockIdx.y * 32, j0 = blockIdx.x * 32;
  const int lb = blockIdx.z * g.lsplit, le = min(g.L, lb + g.lsplit);
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int l0 = lb; l0 < le; l0 += 32) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = tid + 256 * q;
      // A tile: consecutive threads along whichever of i / l is contiguous in memory
      const int ai = g.sai == 1 ? (e & 31) : (e >> 5), al = g.sai == 1 ? (e >> 5) : (e & 31);
      const bool aok = i0 + ai < g.I && l0 + al < le;
      As[al][ai] = aok ? g.a[(long)(i0 + ai) * g.sai + (long)(l0 + al) * g.sal] : 0.f;
      const int bj = g.sbj == 1 ? (e & 31) : (e >> 5), bl = g.sbj == 1 ? (e >> 5) : (e & 31);
      const bool bok = j0 + bj < g.J && l0 + bl < le;
      Bs[bl][bj] = bok ? g.b[(long)(l0 + bl) * g.sbl + (long)(j0 + bj) * g.sbj] : 0.f;
    }
    __syncthreads();
#pragma unroll 8
    for (int l = 0; l < 32; ++l) {
      const float bv = Bs[l][tj];
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = fmaf(As[l][4 * ti + q], bv, acc[q]);
    }
    __syncthreads();
  }
  const int j = j0 + tj;
  if (j >= g.J) return;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int i = i0 + 4 * ti + q;
    if (i >= g.I) continue;
    if (gridDim.z > 1) {
      g.c[((size_t)blockIdx.z * g.I + i) * g.J + j] = acc[q];
    } else {
      float v = acc[q] + (g.bias != nullptr ? g.bias[j] : 0.f);
      float* d = g.c + (size_t)i * g.ldc + j;
      *d = g.accumulate ? *d + v : v;
    }
  }
}
static __global__ void small_gemm_finish_kernel(const float* part, int splits, int I, int J, const float* bias,
                                                float* c, int ldc, int accumulate) {
  for (size_t e = (size_t)blockIdx.x * 256 + threadIdx.x; e < (size_t)I * J; e += (size_t)gridDim.x * 256) {
    const int i = (int)(e / J), j = (int)(e % J);
    float v = 0.f;
    for (int z = 0; z < splits; ++z) v += part[(size_t)z * I * J + e];
    v += bias != nullptr ? bias[j] : 0.f;
    float* d = c + (size_t)i * ldc + j;
    *d = accumulate ? *d + v : v;
  }
}
// db[o] = sum_r dY[r][o] (rows in order)
static __global__ void dense_db_kernel(const float* dy, int ldy, int R, int O, float* db) {
  const int o = blockIdx.x * 256 + threadIdx.x;
  if (o >= O) return;
  float s = 0.f;
  for (int r = 0; r < R; ++r) s += dy[(size_t)r * ldy + o];
  db[o] = s;
}
static __global__ void silu_fwd_kernel(const float* x, float* y, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) y[i] = silu(x[i]);
}
static __global__ void silu_bwd_kernel(const float* d, const float* pre, float* dst, size_t n, int accumulate) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const float g = d[i] * silu_grad(pre[i]);
    dst[i] = accumulate ? dst[i] + g : g;
  }
}

// Layout helpers: NCHW <-> NHWC (channels padded to Cp with zeros), [vals | mask] concat.
static __global__ void nchw_to_nhwc_kernel(const float* src, float* dst, int N, int C, int Cp, int HW) {
  const size_t total = (size_t)N * HW * Cp;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
    const int c = (int)(i % Cp);
    const size_t pix = i / Cp;
    const int n = (int)(pix / HW), hw = (int)(pix % HW);
    dst[i] = c < C ? src[((size_t)n * C + c) * HW + hw] : 0.f;
  }
}
static __global__ void cat24_kernel(const float* vals, const float* mask, float* out, int N) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= N * 24) return;
  const int n = i / 24, k = i % 24;
  out[i] = k < 12 ? vals[n * 12 + k] : mask[n * 12 + k - 12];
}

// GAP (mean over HW) of feat [N][HW][64] -> g [N][64]; and its backward dfeat[n][hw][k] += dg[n][k] / HW.
static __global__ void gap_fwd_kernel(const float* feat, int HW, float* g) {
  const int n = blockIdx.x, k = threadIdx.x & 63, sl = threadIdx.x >> 6;
  __shared__ float part[4][64];
  float s = 0.f;
  for (int pix = sl; pix < HW; pix += 4) s += feat[((size_t)n * HW + pix) * 64 + k];
  part[sl][k] = s;
  __syncthreads();
  if (threadIdx.x < 64) g[n * 64 + threadIdx.x] = (part[0][threadIdx.x] + part[1][threadIdx.x] +
                                                   part[2][threadIdx.x] + part[3][threadIdx.x]) / (float)HW;
}
static __global__ void gap_bwd_kernel(const float* dg, int N, int HW, float* dfeat) {
  const size_t total = (size_t)N * HW * 64;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
    const int k = (int)(i % 64), n = (int)(i / ((size_t)HW * 64));
    dfeat[i] += dg[n * 64 + k] / (float)HW;
  }
}

// Embedding (models/unet_cond.py:155-167): emb[n] = pos(t_n) + class_emb[y_n] (+ cond, added by the
// host sequence); dclass[c][k] = sum over samples with y_n == c of demb[n][k] (sample order).
static __global__ void embed_base_kernel(const int64_t* t, const int64_t* y, const float* pos_table, int tmax,
                                         const float* class_emb, int ncls, float* emb) {
  const int n = blockIdx.x, k = threadIdx.x;
  int64_t tt = t[n];
  tt = tt < 1 ? 1 : (tt > tmax ? tmax : tt);
  float v = pos_table[(size_t)(tt - 1) * 256 + k];
  if (y != nullptr) {
    int64_t yy = y[n];
    yy = yy < 0 ? 0 : (yy >= ncls ? ncls - 1 : yy);
    v += class_emb[yy * 256 + k];
  }
  emb[n * 256 + k] = v;
}
static __global__ void class_emb_bwd_kernel(const float* demb, const int64_t* y, int N, int ncls, float* dclass) {
  const int c = blockIdx.x, k = threadIdx.x;
  float s = 0.f;
  for (int n = 0; n < N; ++n)
    if (y[n] == c) s += demb[n * 256 + k];
  dclass[c * 256 + k] = s;
}

}  // namespace dmx
