// dmx — fused per-token kernels of AttenionBlock (models/unet_cond.py:32-52), gfx950.
//
// The block is   xl = LN1(x);  av = MHA(xl) + xl;  out = FF(LN2(av)) + av
// with FF = Linear -> GELU -> Linear.  Everything except the attention core is row-local
// (one token = one row of C channels), so two kernels cover it with K = C resident:
//
//   tok_ln_qkv_kernel     qkv = LN1(x) Wqkv^T + b                      (TA)
//   tok_attn_out_kernel   av  = ao Wo^T + bo + LN1(x)                   (TB, one kernel)
//                         f   = GELU(LN2(av) W1^T + b1)
//                         out = f W2^T + b2 + av
//
// replacing 2 LayerNorm + 4 GEMM launches and five (M, C) intermediates per block.
//
// Layout: one block = TM (64 | 32) tokens x all C channels (TA: x NB output columns),
// 4 waves; the activation tile lives in LDS as f16 hi / lo planes [TM][C + 8] (row
// stride ≡ 4 dwords mod 64 for C = 128/256 and 36 for C = 64: conflict-free ds_read_b128).  Weights are the
// x3 B layout [Npad][Kpad] (scaled hi / lo), small and L2-resident, read straight into
// MFMA B fragments (16 B per lane) with a rolling register prefetch — no LDS, no barrier.
// Products are the x3 split (ah*bh + ah*bl + al*bh, fp32 accumulate) as in igemm_x3.h.
#pragma once
#include "common.h"
#include "igemm_x3.h"

namespace dmx {

constexpr int TOK_PD = 8;  // k16 steps of B fragments in flight in tok_gemm (L2 latency cover)

struct TokW {                 // one Linear in the x3 B layout
  const _Float16* h;          // [Npad][Kpad] hi (scaled by 1/inv_scale)
  const _Float16* l;          //               lo
  const float* bias;          // [N]
  float inv_scale;
  int kpad;
  const _Float16* fh;         // the same planes in MFMA-fragment order (igemm_halo.h
  const _Float16* fl;         // frag_planes_kernel), or null
};

struct TokParams {
  const float* x;             // block input tokens [M][C] (NHWC rows)
  const float* ao;            // TB: attention core output [M][C]
  float* out;                 // TA: qkv [M][3C]; TB: block output [M][C]
  const float* l1w;           // LN1 (AttenionBlock.ln)
  const float* l1b;
  const float* l2w;           // LN2 (ff_self[0])
  const float* l2b;
  TokW w0, w1, w2;            // TA: w0 = in_proj; TB: w0 = out_proj, w1 = ff_self[1], w2 = ff_self[3]
  int M;
};

enum { ROWS_SPLIT = 0, ROWS_LN = 1, ROWS_STATS = 2, ROWS_LNF = 3 };

// DPP lane exchange (no LDS round trip): quad_perm / row_half_mirror / row_mirror.
template <int CTRL>
DMX_DEV float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
// Sum over aligned groups of G lanes (G = 4, 8, 16); every lane of a group gets the same bits.
template <int G>
DMX_DEV float group_sum(float s) {
  s += dpp_f<0xB1>(s);                          // quad_perm [1,0,3,2]
  s += dpp_f<0x4E>(s);                          // quad_perm [2,3,0,1]
  if constexpr (G >= 8) s += dpp_f<0x141>(s);   // row_half_mirror
  if constexpr (G >= 16) s += dpp_f<0x140>(s);  // row_mirror
  return s;
}

// TM rows (m0 .. m0+TM-1, zero past M) of an fp32 [.][ld] source -> A planes, either split
// as-is (ROWS_SPLIT), LayerNorm'd then split (ROWS_LN), or only the LN statistics recorded
// (ROWS_STATS).  A row is owned by G = C/16 lanes, 4 float4 each (columns 4g + 4Gj, so one
// load instruction covers 16G contiguous bytes of a row); every load of the pass is issued
// before any is used.  LN = nn.LayerNorm: two-pass mean / biased variance, eps 1e-5, the
// same per-element expression as layernorm_kernel.
// The loaded rows of one tok_rows pass (tok_rows_load), consumed by tok_rows_put: split so a
// multi-tile block can load tile t + 1 under tile t's GEMMs.
template <int C, int TM, int NW>
struct TokRowsV {
  static constexpr int G = C / 16, RP = 64 / G, RW = TM / NW, NP = RW / RP;
  static_assert(G == 4 || G == 8 || G == 16, "C");
  static_assert(NP >= 1 && RW % RP == 0, "rows per wave");
  floatx4 v[NP][4];
};
template <int C, int TM, int NW = 4>
DMX_DEV void tok_rows_load(const float* src, int ld, int m0, int M, TokRowsV<C, TM, NW>& rv) {
  using R = TokRowsV<C, TM, NW>;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int rr = lane / R::G, c0 = 4 * (lane % R::G);
#pragma unroll
  for (int p = 0; p < R::NP; ++p) {
    const int m = min(m0 + wid * R::RW + p * R::RP + rr, M - 1);
#pragma unroll
    for (int j = 0; j < 4; ++j) rv.v[p][j] = ld4(src + (size_t)m * ld + c0 + 4 * R::G * j);
  }
}
template <int C, int TM, int MODE, int NW = 4>
DMX_DEV void tok_rows_put(TokRowsV<C, TM, NW>& rv, int m0, int M, const float* g, const float* b,
                          _Float16 (*Ah)[C + 8], _Float16 (*Al)[C + 8], float* mu, float* rs, float* o32 = nullptr,
                          int ldo = 0) {
  using R = TokRowsV<C, TM, NW>;
  constexpr int G = R::G, RP = R::RP, RW = R::RW, NP = R::NP;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int rr = lane / G, c0 = 4 * (lane % G);
  auto& v = rv.v;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int row = wid * RW + p * RP + rr;
    if (m0 + row >= M) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[p][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    if constexpr (MODE == ROWS_SPLIT) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        half4 h, l;
        split4(v[p][j], h, l);
        *reinterpret_cast<half4*>(&Ah[row][c0 + 4 * G * j]) = h;
        *reinterpret_cast<half4*>(&Al[row][c0 + 4 * G * j]) = l;
      }
    } else {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) s += (v[p][j][0] + v[p][j][1]) + (v[p][j][2] + v[p][j][3]);
      const float mean = group_sum<G>(s) / (float)C;
      float q = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = v[p][j][e] - mean;
          q += d * d;
        }
      const float rstd = 1.0f / sqrtf(group_sum<G>(q) / (float)C + 1e-5f);
      if constexpr (MODE == ROWS_STATS) {
        if (lane % G == 0) {
          mu[row] = mean;
          rs[row] = rstd;
        }
      } else if constexpr (MODE == ROWS_LNF) {  // LN'd rows kept fp32 in LDS (o32[row][c], stride ldo)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = c0 + 4 * G * j;
          const floatx4 gw = ld4(g + c), bw = ld4(b + c);
          floatx4 y;
#pragma unroll
          for (int e = 0; e < 4; ++e) y[e] = (v[p][j][e] - mean) * rstd * gw[e] + bw[e];
          *reinterpret_cast<floatx4*>(o32 + row * ldo + c) = y;
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = c0 + 4 * G * j;
          const floatx4 gw = ld4(g + c), bw = ld4(b + c);
          floatx4 y;
#pragma unroll
          for (int e = 0; e < 4; ++e) y[e] = (v[p][j][e] - mean) * rstd * gw[e] + bw[e];
          half4 h, l;
          split4(y, h, l);
          *reinterpret_cast<half4*>(&Ah[row][c]) = h;
          *reinterpret_cast<half4*>(&Al[row][c]) = l;
        }
      }
    }
  }
}

template <int C, int TM, int MODE, int NW = 4>
DMX_DEV void tok_rows(const float* src, int ld, int m0, int M, const float* g, const float* b,
                      _Float16 (*Ah)[C + 8], _Float16 (*Al)[C + 8], float* mu, float* rs, float* o32 = nullptr,
                      int ldo = 0) {
  TokRowsV<C, TM, NW> rv;
  tok_rows_load<C, TM, NW>(src, ld, m0, M, rv);
  tok_rows_put<C, TM, MODE, NW>(rv, m0, M, g, b, Ah, Al, mu, rs, o32, ldo);
}

// B fragments of one token GEMM in flight: the first PD k16 steps, requested by tok_prime before
// the GEMM's A operand exists (under the LayerNorm / epilogue phases and their barriers), so the
// L2 round trip of the weights is off the critical path; tok_gemm_primed consumes them and keeps
// PD steps in flight (rolling register prefetch).
template <int C, int NT, int PDM = TOK_PD>
struct TokB {
  static constexpr int S = C / 16, PD = S < PDM ? S : PDM;
  half8 h[PD][NT], l[PD][NT];
};

// fragment-ordered planes: fragment (column block nb, k16 step s) is 1 KB contiguous, lane-major
// (one coalesced load per wave); otherwise 32 rows x 32 bytes of the [Npad][Kpad] planes
struct TokBPtr {
  const _Float16 *wh, *wl;
  size_t jstride;
  int sstride;
};
DMX_DEV TokBPtr tok_bptr(const TokW& w, int nw, int fr, int fh) {
  const bool frag = w.fh != nullptr;
  const int lane = 32 * fh + fr;
  TokBPtr p;
  p.wh = frag ? w.fh + (size_t)(nw >> 5) * (w.kpad / 16) * 512 + lane * 8 : w.h + (size_t)(nw + fr) * w.kpad + 8 * fh;
  p.wl = frag ? w.fl + (size_t)(nw >> 5) * (w.kpad / 16) * 512 + lane * 8 : w.l + (size_t)(nw + fr) * w.kpad + 8 * fh;
  p.jstride = frag ? (size_t)(w.kpad / 16) * 512 : (size_t)32 * w.kpad;
  p.sstride = frag ? 512 : 16;
  return p;
}
template <int NT, int X1>
DMX_DEV void tok_loadb(const TokBPtr& p, int s, half8* h, half8* l) {
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    h[j] = *reinterpret_cast<const half8*>(p.wh + j * p.jstride + p.sstride * s);
    if constexpr (!X1) l[j] = *reinterpret_cast<const half8*>(p.wl + j * p.jstride + p.sstride * s);
  }
}
template <int C, int NT, int X1 = 0, int PDM = TOK_PD>
DMX_DEV void tok_prime(const TokW& w, int nw, int fr, int fh, TokB<C, NT, PDM>& b) {
  const TokBPtr p = tok_bptr(w, nw, fr, fh);
#pragma unroll
  for (int s = 0; s < TokB<C, NT, PDM>::PD; ++s) tok_loadb<NT, X1>(p, s, b.h[s], b.l[s]);
}

// acc[j] = A[arow0 .. +32][0, C) . W[nw + 32j .. +32][0, C)^T  (x3 sum, still scaled by 2^e),
// B fragments primed by tok_prime (same w, nw).
template <int C, int NT, int X1 = 0, int PDM = TOK_PD>
DMX_DEV void tok_gemm_primed(const _Float16 (*Ah)[C + 8], const _Float16 (*Al)[C + 8], const TokW& w, int nw,
                             TokB<C, NT, PDM>& b, floatx16 (&acc)[NT], int arow0, int fr, int fh) {
  constexpr int S = C / 16, PD = TokB<C, NT, PDM>::PD;
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  const TokBPtr p = tok_bptr(w, nw, fr, fh);
  const int arow = arow0 + fr;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const half8 ah = *reinterpret_cast<const half8*>(&Ah[arow][16 * s + 8 * fh]);
    half8 al;
    if constexpr (!X1) al = *reinterpret_cast<const half8*>(&Al[arow][16 * s + 8 * fh]);
    half8 ch[NT], cl[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      ch[j] = b.h[s % PD][j];
      cl[j] = b.l[s % PD][j];
    }
    if (s + PD < S) tok_loadb<NT, X1>(p, s + PD, b.h[s % PD], b.l[s % PD]);
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      if constexpr (!X1) {
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, ch[j], acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, cl[j], acc[j], 0, 0, 0);
      }
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, ch[j], acc[j], 0, 0, 0);
    }
  }
}

// Unprimed form: B fragments straight from global memory (L2-resident weights), PD steps ahead.
template <int C, int NT, int X1 = 0>
DMX_DEV void tok_gemm(const _Float16 (*Ah)[C + 8], const _Float16 (*Al)[C + 8], const TokW& w, int nw,
                      floatx16 (&acc)[NT], int arow0, int fr, int fh) {
  TokB<C, NT> b;
  tok_prime<C, NT, X1>(w, nw, fr, fh, b);
  tok_gemm_primed<C, NT, X1>(Ah, Al, w, nw, b, acc, arow0, fr, fh);
}

// Row of accumulator register r inside a wave's 32-row tile (v_mfma_f32_32x32x16 layout).
DMX_DEV int tok_r(int fh, int r) { return (r & 3) + 8 * (r >> 2) + 4 * fh; }

// TA: qkv = LN1(x) Wqkv^T + b_in (nn.MultiheadAttention in_proj on the LN1 output).
// Block = 64 tokens x NB of the 3C output columns (grid.y = 3C / NB); waves 2 x 2.
template <int C, int NB, int X1 = 0>
__global__ __launch_bounds__(256) void tok_ln_qkv_kernel(const TokParams P) {
  constexpr int NT = NB / 64;
  __shared__ __attribute__((aligned(16))) _Float16 Ah[64][C + 8];
  __shared__ __attribute__((aligned(16))) _Float16 Al[64][C + 8];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, fr = lane & 31, fh = lane >> 5;
  const int wm = wid >> 1, wn = wid & 1, m0 = blockIdx.x * 64;
  const int nw = blockIdx.y * NB + wn * (NB / 2);
  TokB<C, NT> b;
  tok_prime<C, NT, X1>(P.w0, nw, fr, fh, b);  // weights in flight with the token loads
  tok_rows<C, 64, ROWS_LN>(P.x, C, m0, P.M, P.l1w, P.l1b, Ah, Al, nullptr, nullptr);
  __syncthreads();
  floatx16 acc[NT];
  tok_gemm_primed<C, NT, X1>(Ah, Al, P.w0, nw, b, acc, wm * 32, fr, fh);
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int col = nw + 32 * j + fr;
    const float bias = P.w0.bias[col];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + wm * 32 + tok_r(fh, r);
      if (m < P.M) P.out[(size_t)m * 3 * C + col] = acc[j][r] * P.w0.inv_scale + bias;
    }
  }
}

// TA for wide C (256): NW = 8 waves as 2 (32-token halves) x 4 (column quarters), 64 tokens x NB
// of the 3C columns per block (grid.y = 3C / NB), each wave 32 x NB/4 (NT = NB / 128 tiles) with PD
// k16 steps of B fragments in flight.  The LayerNorm of a token tile runs 3C / NB times instead of
// 3C / 64 times (tok_ln_qkv_kernel<256, 64>: twelve), and the grid is one round of blocks.
template <int C, int NB, int NW, int PD, int X1 = 0>
__global__ __launch_bounds__(NW * 64) void tok_ln_qkv_w_kernel(const TokParams P) {
  constexpr int WN = NW / 2, NT = NB / WN / 32;
  static_assert(NT >= 1 && NB % (WN * 32) == 0, "tile");
  __shared__ __attribute__((aligned(16))) _Float16 Ah[64][C + 8];
  __shared__ __attribute__((aligned(16))) _Float16 Al[64][C + 8];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, fr = lane & 31, fh = lane >> 5;
  const int wm = wid / WN, wn = wid % WN, m0 = blockIdx.x * 64;
  const int nw = blockIdx.y * NB + wn * (NB / WN);
  TokB<C, NT, PD> b;
  tok_prime<C, NT, X1, PD>(P.w0, nw, fr, fh, b);  // weights in flight with the token loads
  tok_rows<C, 64, ROWS_LN, NW>(P.x, C, m0, P.M, P.l1w, P.l1b, Ah, Al, nullptr, nullptr);
  __syncthreads();
  floatx16 acc[NT];
  tok_gemm_primed<C, NT, X1, PD>(Ah, Al, P.w0, nw, b, acc, wm * 32, fr, fh);
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int col = nw + 32 * j + fr;
    const float bias = P.w0.bias[col];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + wm * 32 + tok_r(fh, r);
      if (m < P.M) P.out[(size_t)m * 3 * C + col] = acc[j][r] * P.w0.inv_scale + bias;
    }
  }
}

// acc[j] = A[arow0 .. +32][0, C) . W[nw + 32j .. +32][0, C)^T with W staged in LDS planes
// ([rows][C + 8], the A planes' conflict-free stride).
template <int C, int NT, int X1 = 0>
DMX_DEV void tok_gemm_lds(const _Float16 (*Ah)[C + 8], const _Float16 (*Al)[C + 8], const _Float16 (*Wh)[C + 8],
                          const _Float16 (*Wl)[C + 8], int nw, floatx16 (&acc)[NT], int arow0, int fr, int fh) {
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  const int arow = arow0 + fr;
#pragma unroll
  for (int s = 0; s < C / 16; ++s) {
    const half8 ah = *reinterpret_cast<const half8*>(&Ah[arow][16 * s + 8 * fh]);
    half8 al;
    if constexpr (!X1) al = *reinterpret_cast<const half8*>(&Al[arow][16 * s + 8 * fh]);
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const half8 bh = *reinterpret_cast<const half8*>(&Wh[nw + 32 * j + fr][16 * s + 8 * fh]);
      if constexpr (!X1) {
        const half8 bl = *reinterpret_cast<const half8*>(&Wl[nw + 32 * j + fr][16 * s + 8 * fh]);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc[j], 0, 0, 0);
      }
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc[j], 0, 0, 0);
    }
  }
}

// TA with the weight slice resident in LDS: the block stages rows [blockIdx.y * NB, +NB) of
// the in_proj hi / lo planes once, then runs TPB consecutive 64-token tiles (LN1 -> planes ->
// GEMM -> store).  Per 64 tokens the B-fragment reads of tok_ln_qkv_kernel (NB x C x 4 bytes
// from L2, 3x the activation bytes at C = 64) become LDS reads.
template <int C, int NB, int TPB, int X1 = 0>
__global__ __launch_bounds__(256) void tok_ln_qkv_lds_kernel(const TokParams P) {
  constexpr int NT = NB / 64;
  __shared__ __attribute__((aligned(16))) _Float16 Wh[NB][C + 8];
  __shared__ __attribute__((aligned(16))) _Float16 Wl[X1 ? 1 : NB][C + 8];
  __shared__ __attribute__((aligned(16))) _Float16 Ah[64][C + 8];
  __shared__ __attribute__((aligned(16))) _Float16 Al[64][C + 8];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, fr = lane & 31, fh = lane >> 5;
  const int wm = wid >> 1, wn = wid & 1;
  const int nb0 = blockIdx.y * NB;
  constexpr int CPR = C / 8;  // 16-byte chunks per weight row
  for (int i = tid; i < NB * CPR; i += 256) {
    const int r = i / CPR, q = i % CPR;
    const size_t o = (size_t)(nb0 + r) * P.w0.kpad + q * 8;
    *reinterpret_cast<half8*>(&Wh[r][q * 8]) = *reinterpret_cast<const half8*>(P.w0.h + o);
    if constexpr (!X1) *reinterpret_cast<half8*>(&Wl[r][q * 8]) = *reinterpret_cast<const half8*>(P.w0.l + o);
  }
  const int nwl = wn * (NB / 2);  // this wave's first column inside the slice
  float bias[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) bias[j] = P.w0.bias[nb0 + nwl + 32 * j + fr];
  TokRowsV<C, 64, 4> rv;  // token rows of the next tile, loaded under this tile's GEMM
  if (blockIdx.x * TPB * 64 < P.M) tok_rows_load<C, 64>(P.x, C, blockIdx.x * TPB * 64, P.M, rv);
  for (int t = 0; t < TPB; ++t) {
    const int m0 = (blockIdx.x * TPB + t) * 64;
    if (m0 >= P.M) break;
    tok_rows_put<C, 64, ROWS_LN>(rv, m0, P.M, P.l1w, P.l1b, Ah, Al, nullptr, nullptr);
    __syncthreads();
    if (t + 1 < TPB && m0 + 64 < P.M) tok_rows_load<C, 64>(P.x, C, m0 + 64, P.M, rv);
    floatx16 acc[NT];
    tok_gemm_lds<C, NT, X1>(Ah, Al, Wh, Wl, nwl, acc, wm * 32, fr, fh);
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int col = nb0 + nwl + 32 * j + fr;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 32 + tok_r(fh, r);
        if (m < P.M) P.out[(size_t)m * 3 * C + col] = acc[j][r] * P.w0.inv_scale + bias[j];
      }
    }
    __syncthreads();  // every wave is done with this tile's planes
  }
}

// TB: out-proj + residual, LN2, FF1 + GELU, FF2 + residual for TM tokens x all C channels.
// NW waves: TM = 64: 2 (rows) x NW/2 (cols); TM = 32: 1 x NW (more blocks for small M / wide C);
// TM = 128: 4 x NW/4.  WLDS = 1: the three C x C weights (hi / lo planes) are staged in LDS
// once per block and the block runs TPB consecutive token tiles (C = 64: the weights are 3x
// the tile's activation bytes, re-read from L2 per tile otherwise).
template <int C, int TM, int X1 = 0, int NW = 4, int WLDS = 0, int TPB = 1>
__global__ __launch_bounds__(NW * 64) void tok_attn_out_kernel(const TokParams P) {
  constexpr int WR = TM / 32, WC = NW / WR, CW = C / WC, NT = CW / 32, VS = C + 4;
  static_assert(NT >= 1, "tile");
  constexpr int NWS = WLDS ? 3 : 1, WRW = WLDS ? C : 1, WRL = (WLDS && !X1) ? C : 1;
  __shared__ __attribute__((aligned(16))) _Float16 Ah[TM][C + 8];
  __shared__ __attribute__((aligned(16))) _Float16 Al[TM][C + 8];
  __shared__ __attribute__((aligned(16))) float Av[TM][VS];
  __shared__ __attribute__((aligned(16))) _Float16 Wh[NWS][WRW][C + 8];
  __shared__ __attribute__((aligned(16))) _Float16 Wl[NWS][WRL][C + 8];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, fr = lane & 31, fh = lane >> 5;
  const int wm = wid / WC, wn = wid % WC;
  const int M = P.M, nw = wn * CW, arow0 = wm * 32;
  if constexpr (WLDS) {
    constexpr int CPR = C / 8;
    for (int i = threadIdx.x; i < 3 * C * CPR; i += NW * 64) {
      const int w = i / (C * CPR), r = (i / CPR) % C, q = i % CPR;
      const TokW& tw = w == 0 ? P.w0 : w == 1 ? P.w1 : P.w2;
      const size_t o = (size_t)r * tw.kpad + q * 8;
      *reinterpret_cast<half8*>(&Wh[w][r][q * 8]) = *reinterpret_cast<const half8*>(tw.h + o);
      if constexpr (!X1) *reinterpret_cast<half8*>(&Wl[w][r][q * 8]) = *reinterpret_cast<const half8*>(tw.l + o);
    }
  }
  // non-WLDS: the next GEMM's first B fragments are requested as soon as the current GEMM has
  // consumed its own (tok_prime), i.e. before the epilogue / LayerNorm phases and their barriers
  TokB<C, NT> bf;
  const TokW* const tws[3] = {&P.w0, &P.w1, &P.w2};
  auto gemm = [&](int w, const TokW& tw, floatx16(&acc)[NT]) {
    if constexpr (WLDS) {
      tok_gemm_lds<C, NT, X1>(Ah, Al, Wh[w], Wl[X1 ? 0 : w], nw, acc, arow0, fr, fh);
    } else {
      tok_gemm_primed<C, NT, X1>(Ah, Al, tw, nw, bf, acc, arow0, fr, fh);
      if (w < 2) tok_prime<C, NT, X1>(*tws[w + 1], nw, fr, fh, bf);
    }
  };
  if constexpr (!WLDS) tok_prime<C, NT, X1>(P.w0, nw, fr, fh, bf);

  // ao -> A planes; LN1(x) -> Av (fp32, the residual of the out-projection): both loads in flight
  // together, no second read of x later; with several tiles per block the next tile's rows are
  // loaded under this tile's GEMMs
  TokRowsV<C, TM, NW> rao, rx;
  if (blockIdx.x * TPB * TM < M) {
    tok_rows_load<C, TM, NW>(P.ao, C, blockIdx.x * TPB * TM, M, rao);
    tok_rows_load<C, TM, NW>(P.x, C, blockIdx.x * TPB * TM, M, rx);
  }
  for (int t = 0; t < TPB; ++t) {
    const int m0 = (blockIdx.x * TPB + t) * TM;
    if (m0 >= M) break;
    tok_rows_put<C, TM, ROWS_SPLIT, NW>(rao, m0, M, nullptr, nullptr, Ah, Al, nullptr, nullptr);
    tok_rows_put<C, TM, ROWS_LNF, NW>(rx, m0, M, P.l1w, P.l1b, Ah, Al, nullptr, nullptr, &Av[0][0], VS);
    __syncthreads();
    if (TPB > 1 && t + 1 < TPB && m0 + TM < M) {
      tok_rows_load<C, TM, NW>(P.ao, C, m0 + TM, M, rao);
      tok_rows_load<C, TM, NW>(P.x, C, m0 + TM, M, rx);
    }

    floatx16 acc[NT];
    // av = ao Wo^T + bo + LN1(x)   (models/unet_cond.py:49-50); each Av element is read and
    // rewritten by the same lane
    gemm(0, P.w0, acc);
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int col = nw + 32 * j + fr;
      const float bo = P.w0.bias[col];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = arow0 + tok_r(fh, r);
        Av[row][col] = (acc[j][r] * P.w0.inv_scale + bo) + Av[row][col];
      }
    }
    __syncthreads();
    // LN2(av) -> A planes (ff_self[0])
    tok_rows<C, TM, ROWS_LN, NW>(&Av[0][0], VS, 0, TM, P.l2w, P.l2b, Ah, Al, nullptr, nullptr);
    __syncthreads();
    // f = GELU(LN2(av) W1^T + b1)  (ff_self[1:3])
    gemm(1, P.w1, acc);
    __syncthreads();  // every wave is done reading the LN2 planes
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int col = nw + 32 * j + fr;
      const float b = P.w1.bias[col];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = arow0 + tok_r(fh, r);
        const float f = gelu(acc[j][r] * P.w1.inv_scale + b);
        const _Float16 h = (_Float16)f;
        Ah[row][col] = h;
        Al[row][col] = (_Float16)(f - (float)h);
      }
    }
    __syncthreads();
    // out = f W2^T + b2 + av  (ff_self[3] + residual, models/unet_cond.py:51)
    gemm(2, P.w2, acc);
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int col = nw + 32 * j + fr;
      const float b = P.w2.bias[col];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = arow0 + tok_r(fh, r), m = m0 + row;
        if (m < M) P.out[(size_t)m * C + col] = (acc[j][r] * P.w2.inv_scale + b) + Av[row][col];
      }
    }
    if (TPB > 1) {
      if constexpr (!WLDS) {
        if ((blockIdx.x * TPB + t + 1) * TM < M) tok_prime<C, NT, X1>(P.w0, nw, fr, fh, bf);
      }
      __syncthreads();  // the next tile overwrites the planes and Av
    }
  }
}

}  // namespace dmx
