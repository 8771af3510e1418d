// dmx — split-precision implicit GEMM: fp32 operands as fp16 (hi + lo) pairs on the
// fp16 matrix cores (v_mfma_f32_32x32x16_f16, fp32 accumulate), gfx950.
//
//   a = ah + al,  ah = f16(a), al = f16(a - ah)       (|a - ah - al| <= 2^-22 |a|, normal range)
//   C = sum_k ah*bh + ah*bl + al*bh                     (al*bl ~ 2^-22, dropped)
//
// Three MFMAs per product at 16x the fp32-MFMA rate => ~5.3x the fp32 ceiling with an error
// of a few 1e-7 relative (the f16 products are exact in the fp32 accumulator).  B (weights) is
// split once at load time, pre-scaled by 2^e so its lo parts stay f16-normal; the epilogue
// multiplies by 2^-e (exact).  A (activations, plain NHWC fp32) is split while staging to LDS.
//
// Tiling: 256 threads = 2x2 waves, block BM x BN, K-step 32 (two k16 MFMA steps), separate
// hi / lo LDS planes with 80-byte rows (conflict-free ds_read_b128), double-buffered; lane
// (r, h) reads k = 16s + 8h .. +7 of row r.  Epilogues identical to igemm.h.
#pragma once
#include "common.h"
#include "igemm.h"

namespace dmx {


// 16 readable zero bytes: the load target of masked (padding) A pieces.
static __device__ __attribute__((aligned(16))) float g_zero16[4] = {0.f, 0.f, 0.f, 0.f};

constexpr int X3_BK = 32;
constexpr int X3_STRIDE = 40;  // f16 per LDS row (32 + 8 pad) = 80 bytes

struct X3Params {
  IgemmParams g;           // geometry / epilogue (g.Bw unused)
  const _Float16* Ash;     // SPLIT_A: activation hi / lo planes [N][H][W][C] (else g.src.src0 fp32)
  const _Float16* Asl;
  const _Float16* Bh;      // [phases][Npad][Kpad] scaled hi
  const _Float16* Bl;      //                      scaled lo
  float inv_scale;         // 2^-e
  unsigned a_bytes;        // bytes of the A source (one plane) — buffer-load range
  unsigned b_bytes;        // bytes of one phase of one B plane ([Npad][Kpad] f16)
  const _Float16* Fh;      // the B planes in MFMA-fragment order (igemm_halo.h), or null
  const _Float16* Fl;
  // GroupNorm(1, C) + GELU applied to the raw fp32 source while staging (igemm_halo.h GNA):
  const float2* gn_rowpart;  // [N][gn_cnt] (sum, sum of squares) partials of the producing conv
  int gn_cnt;
  const float* gn_gamma;
  const float* gn_beta;
  const float* gn_res;       // GNA = 2: GELU(res + GroupNorm(src)) (a residual ResBlock's output)
  // Winograd F(2x2, 3x3) weights (igemm_wino.h): U = G g Gᵀ split hi / lo, fragment order
  const _Float16* Uh;
  const _Float16* Ul;
  unsigned u_bytes;          // bytes of one U plane (16 * Cout * Cin f16)
  int dslot;                 // diagnostic builds (DMX_DIAG): stamp slot of this launch, else unused
  // Device-side operand scales (igemm_x3_kernel, fp32 A source; the training data gradients, whose dY
  // and refreshed weights have no host-known range): a_amax = bits of max|A| — A is multiplied by
  // 2^ea (max|A| 2^ea in [2^12, 2^13)) before its hi / lo split, so the lo parts stay f16-normal;
  // w_inv = the weights' 2^-e written by split_batch_kernel.  The accumulators are multiplied
  // by w_inv 2^-ea (exact: powers of two).  Null: host inv_scale, unscaled A.
  const unsigned* a_amax;     // (a_nparts > 0: a_amax holds that many per-block partial maxima)
  int a_nparts;
  const float* w_inv;
};




// Buffer-resource loads (32-bit offsets, descriptor in SGPRs): an offset at or past the range
// returns zeros, which is how padding taps / rows past M are masked.
constexpr int kOOB = 0x7ffffff0;
DMX_DEV __amdgpu_buffer_rsrc_t rsrc_of(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
DMX_DEV half8 bload_h8(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
DMX_DEV floatx4 bload_f4(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}

// (attention outputs: plain stores — the token kernel reads them back from L2; the non-temporal
// hint measured neutral, round 4)
DMX_DEV void att_st4(float* a, floatx4 v) { *reinterpret_cast<floatx4*>(a) = v; }

// hi/lo split of two fp32 values as packed f16 pairs (common.h split2u: 3 VALU ops per pair).
DMX_DEV void split2(f32x2 v, unsigned& h, unsigned& l) { split2u(v.x, v.y, h, l); }

// X1 = 1: config-4 fp16 arithmetic — operands rounded to f16 (hi planes only), ONE MFMA per
// product (ah*bh), fp32 accumulate; the lo planes are neither loaded nor stored.
// NW = 4: 2 x 2 waves of (BM/2) x (BN/2); NW = 8: 2 x 4 waves of (BM/2) x (BN/4) (twice the waves
// in flight per block for the latency-bound split-K launches at 8x8 / 4x4).
// PF = 2 (NBUF = 1 only): two register stages, K-tile k + 2 is loaded while tile k computes (two
// MFMA phases of latency cover instead of one, for the memory-latency-bound split-K launches).
template <int BM, int BN, int EPI, int BK = 32, int NBUF = 2, int SPLIT_A = 0, int X1 = 0, int NW = 4, int PF = 1>
__global__ __launch_bounds__(64 * NW) void igemm_x3_kernel(const X3Params P) {
  const IgemmParams& p = P.g;
  constexpr int NTH = 64 * NW, NWN = NW / 2;
  constexpr int WM = BM / 2, WN = BN / NWN, TM = WM / 32, TN = WN / 32;
  constexpr int RS = BK + 8;                 // f16 per LDS row (16-byte pad)
  constexpr int APR = SPLIT_A ? BK / 8 : BK / 4;  // A pieces per row (8 f16 per plane | 4 fp32)
  constexpr int BPR = BK / 8;                // 16-byte chunks per B row per plane
  constexpr int AP = BM * APR / NTH;
  constexpr int BP = BN * BPR / NTH;
  constexpr int ARS = NTH / APR, BRS = NTH / BPR;  // rows covered per pass
  static_assert(TM >= 1 && TN >= 1 && AP >= 1 && BP >= 1, "tile");

  constexpr int LA = X1 ? 1 : BM, LB = X1 ? 1 : BN;  // lo planes (unused with X1)
  __shared__ __attribute__((aligned(16))) _Float16 Ah[NBUF][BM][RS];
  __shared__ __attribute__((aligned(16))) _Float16 Al[NBUF][LA][RS];
  __shared__ __attribute__((aligned(16))) _Float16 Bhs[NBUF][BN][RS];
  __shared__ __attribute__((aligned(16))) _Float16 Bls[NBUF][LB][RS];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / NWN, wn = wid % NWN;
  int mt, nt, bz;
  xcd_tile(mt, nt, bz);
  const int phase = EPI == EPI_PARTIAL ? 0 : bz;
  const int m0 = mt * BM, n0 = nt * BN;
  const int qa = tid % APR, ra = tid / APR;
  constexpr int PW = SPLIT_A ? 8 : 4;  // channels per A piece
  const int qb = tid % BPR, rb = tid / BPR;
  const size_t boff = (size_t)phase * p.Npad * p.Kpad;
  const _Float16* Bh = P.Bh + boff;
  const _Float16* Bl = P.Bl + boff;
  const int HW = p.H * p.W;
  const int C = p.src.C;

  // Per staged row: its pixel index (GEMM rows are input-grid pixels) and a bitmask of the
  // taps whose input pixel is inside the map (zero padding / row validity).
  int rpix[AP];
  unsigned tmask[AP];
#pragma unroll
  for (int i = 0; i < AP; ++i) {
    const int m = m0 + ra + i * ARS;
    rpix[i] = m < p.M ? row_anchor(p.geom, m, p.H, p.W, p.Hin, p.Win) : 0;
    tmask[i] = tap_mask(p.geom, phase, p.taps, m, p.M, p.H, p.W, p.Hin, p.Win);
  }

  static_assert(PF == 1 || NBUF == 1, "two register stages only with one LDS buffer");
  floatx4 ra4[PF][SPLIT_A ? 1 : AP];
  half8 rah[PF][SPLIT_A ? AP : 1], ral[PF][SPLIT_A ? AP : 1];
  half8 rbh[PF][BP], rbl[PF][BP];
  // (tap, channel) of this thread's A piece, advanced incrementally (C >= BK on this path)
  int ltap = 0, lc = 0;
  auto seek = [&](int kt) {
    const int k = kt * BK + qa * PW;
    ltap = k / C;
    lc = k - ltap * C;
  };
  const float* __restrict__ asrc = p.src.src0;
  float a_sc = 1.f, o_sc = P.inv_scale;  // device-side scales (X3Params::a_amax / w_inv)
  const bool ascale = !SPLIT_A && P.a_amax != nullptr;
  if (P.w_inv != nullptr) o_sc = *P.w_inv;
  if (!SPLIT_A && P.a_amax != nullptr) {
    unsigned mb = P.a_nparts > 0 ? 0u : *P.a_amax;
    for (int i = lane; i < P.a_nparts; i += 64) mb = max(mb, P.a_amax[i]);  // (non-negative floats order as uints)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mb = max(mb, (unsigned)__shfl_xor((int)mb, o, 64));
    const int ea = amax_exp(mb);
    a_sc = ldexpf(1.f, ea);
    o_sc = o_sc * ldexpf(1.f, -ea);
  }
  // Buffer-resource addressing: 32-bit byte offsets; a masked piece gets an out-of-range offset
  // and reads zeros (no 64-bit address math / selects per piece); B offsets are per-thread
  // constants plus a wave-uniform K-tile offset.
  constexpr int AES = SPLIT_A ? 2 : 4;  // bytes per A element
  const __amdgpu_buffer_rsrc_t rAh = rsrc_of(SPLIT_A ? (const void*)P.Ash : (const void*)asrc, P.a_bytes);
  const __amdgpu_buffer_rsrc_t rAl = rsrc_of(SPLIT_A ? (const void*)P.Asl : (const void*)asrc, P.a_bytes);
  const __amdgpu_buffer_rsrc_t rBh = rsrc_of(Bh, P.b_bytes), rBl = rsrc_of(Bl, P.b_bytes);
  int boffs[BP];
#pragma unroll
  for (int i = 0; i < BP; ++i) boffs[i] = ((n0 + rb + i * BRS) * p.Kpad + qb * 8) * 2;
  auto load_tile = [&](int kt, int st) {  // st: register stage (compile-time constant at every call)
    int ddy, ddx;
    tap_offset(p.geom, phase, ltap, ddy, ddx);
    const int delta = ddy * p.Win + ddx;
    const int tap = ltap, c = lc;
    lc += BK;
    if (lc >= C) {
      lc -= C;
      ++ltap;
    }
#pragma unroll
    for (int i = 0; i < AP; ++i) {
      // Padding taps / rows past M read zeros: the select is on the ADDRESS, so nothing
      // consumes the loaded data before store_tile and the loads stay in flight across
      // compute() (a select on the data forced a vmcnt wait before the MFMAs).
      const bool ok = (tmask[i] >> tap) & 1u;
      const int off = (rpix[i] + delta) * C + c;
      const int boff_a = ok ? off * AES : kOOB;
      if constexpr (SPLIT_A) {
        rah[st][i] = bload_h8(rAh, boff_a, 0);
        if constexpr (!X1) ral[st][i] = bload_h8(rAl, boff_a, 0);
      } else {
        ra4[st][i] = bload_f4(rAh, boff_a, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < BP; ++i) {
      rbh[st][i] = bload_h8(rBh, boffs[i], kt * BK * 2);
      if constexpr (!X1) rbl[st][i] = bload_h8(rBl, boffs[i], kt * BK * 2);
    }
  };
  auto store_tile = [&](int buf, int st) {
#pragma unroll
    for (int i = 0; i < AP; ++i) {
      if constexpr (SPLIT_A) {
        *reinterpret_cast<half8*>(&Ah[buf][ra + i * ARS][qa * 8]) = rah[st][i];
        if constexpr (!X1) *reinterpret_cast<half8*>(&Al[buf][ra + i * ARS][qa * 8]) = ral[st][i];
      } else if constexpr (X1) {
        *reinterpret_cast<half4*>(&Ah[buf][ra + i * ARS][qa * 4]) = __builtin_convertvector(ra4[st][i], half4);
      } else {
        half4 h, l;
        floatx4 v = ra4[st][i];
        if (ascale) {  // (uniform: training data gradients only)
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] *= a_sc;
        }
        split4(v, h, l);
        *reinterpret_cast<half4*>(&Ah[buf][ra + i * ARS][qa * 4]) = h;
        *reinterpret_cast<half4*>(&Al[buf][ra + i * ARS][qa * 4]) = l;
      }
    }
#pragma unroll
    for (int i = 0; i < BP; ++i) {
      *reinterpret_cast<half8*>(&Bhs[buf][rb + i * BRS][qb * 8]) = rbh[st][i];
      if constexpr (!X1) *reinterpret_cast<half8*>(&Bls[buf][rb + i * BRS][qb * 8]) = rbl[st][i];
    }
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int fr = lane & 31, fh = lane >> 5;
  // Fragments of k16-step s+1 are read from LDS while step s's MFMAs issue (double-buffered
  // fragment registers, interleave pinned with sched_group_barrier), so only the first step of
  // a K-tile waits on LDS latency.
  auto compute = [&](int buf) {
    constexpr int S = BK / 16, NR = (X1 ? 1 : 2) * (TM + TN), NM = (X1 ? 1 : 3) * TM * TN;
    half8 ah[2][TM], al[2][TM], bh[2][TN], bl[2][TN];
    auto ldf = [&](int s, int d) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WM + i * 32 + fr;
        ah[d][i] = *reinterpret_cast<const half8*>(&Ah[buf][row][16 * s + 8 * fh]);
        if constexpr (!X1) al[d][i] = *reinterpret_cast<const half8*>(&Al[buf][row][16 * s + 8 * fh]);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * WN + j * 32 + fr;
        bh[d][j] = *reinterpret_cast<const half8*>(&Bhs[buf][row][16 * s + 8 * fh]);
        if constexpr (!X1) bl[d][j] = *reinterpret_cast<const half8*>(&Bls[buf][row][16 * s + 8 * fh]);
      }
    };
    ldf(0, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);  // step 0's reads first
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int d = s & 1;
      if (s + 1 < S) ldf(s + 1, d ^ 1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if constexpr (!X1) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[d][i], bh[d][j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[d][i], bl[d][j], acc[i][j], 0, 0, 0);
          }
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[d][i], bh[d][j], acc[i][j], 0, 0, 0);
        }
      if (s + 1 < S) {
#pragma unroll
        for (int r = 0; r < NR; ++r) {  // one next-step read after each of the first NR MFMAs
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, NM - NR, 0);
      } else {
        __builtin_amdgcn_sched_group_barrier(0x008, NM, 0);
      }
    }
  };
  int kbeg = 0, nK = p.Kpad / BK;
  if constexpr (EPI == EPI_PARTIAL) {
    kbeg = blockIdx.z * p.ksplit;
    nK = min(nK - kbeg, p.ksplit);
  }
  seek(kbeg);
  if constexpr (NBUF == 2) {
    load_tile(kbeg, 0);
    store_tile(0, 0);
    __syncthreads();
    for (int kt = 0; kt < nK; ++kt) {
      const int buf = kt & 1;
      if (kt + 1 < nK) load_tile(kbeg + kt + 1, 0);
      compute(buf);
      if (kt + 1 < nK) store_tile(buf ^ 1, 0);
      __syncthreads();
    }
  } else if constexpr (PF == 2) {
    load_tile(kbeg, 0);
    if (nK > 1) load_tile(kbeg + 1, 1);
    auto body = [&](int kt, int st) {
      store_tile(0, st);
      __syncthreads();
      if (kt + 2 < nK) load_tile(kbeg + kt + 2, st);  // the stage just written is free again
      compute(0);
      __syncthreads();
    };
    for (int kt = 0; kt < nK; kt += 2) {
      body(kt, 0);
      if (kt + 1 < nK) body(kt + 1, 1);
    }
  } else {
    load_tile(kbeg, 0);
    for (int kt = 0; kt < nK; ++kt) {
      store_tile(0, 0);
      __syncthreads();
      if (kt + 1 < nK) load_tile(kbeg + kt + 1, 0);  // in flight during the MFMAs
      compute(0);
      __syncthreads();
    }
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] *= o_sc;

  // the shared epilogue's 2 x 2 wave grid: column pairs of waves as separate BN / (NW / 2) halves
  igemm_epilogue<BM, 2 * WN, EPI>(p, acc, phase, m0, n0 + (wn >> 1) * 2 * WN, wm, wn & 1, fr, fh);
}

static __global__ void split_weights_kernel(const float* src, _Float16* hi, _Float16* lo, size_t n, float scale) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float v = src[i] * scale;
    const _Float16 h = (_Float16)v;
    hi[i] = h;
    lo[i] = (_Float16)(v - (float)h);
  }
}

// Per-block partial maxima (no atomics, no zeroed slot): part[blockIdx.x] = bits of max|src| over
// the block's grid-stride share; consumers reduce the gridDim.x partials (X3Params::a_nparts).
DMX_DEV void absmax_part_body(const float* src, size_t n, unsigned* part, unsigned bx, unsigned gx) {
  float m = 0.f;
  const size_t n4 = n / 4;
  for (size_t i = (size_t)bx * 256 + threadIdx.x; i < n4; i += (size_t)gx * 256) {
    const floatx4 v = reinterpret_cast<const floatx4*>(src)[i];
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
  }
  for (size_t i = n4 * 4 + (size_t)bx * 256 + threadIdx.x; i < n; i += (size_t)gx * 256) m = fmaxf(m, fabsf(src[i]));
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  __shared__ float wm[4];
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) part[bx] = __float_as_uint(fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3])));
}
static __global__ __launch_bounds__(256) void absmax_part_kernel(const float* src, size_t n, unsigned* part) {
  absmax_part_body(src, n, part, blockIdx.x, gridDim.x);
}

// Split with a device-side scale: max|w| 2^e in [2^12, 2^13) from the nparts partial maxima at amax,
// 2^-e to *inv (the training data-gradient weights, re-split on the device after every parameter
// refresh).  Batched over the model's weights (blockIdx.y = job): absmax_batch_kernel writes
// SPLIT_PARTS partial maxima per job, split_batch_kernel reads them and writes hi / lo.
constexpr int SPLIT_PARTS = 64;
struct SplitJob {
  const float* src; _Float16* hi; _Float16* lo; unsigned* amax; float* inv; size_t n;
};
static __global__ __launch_bounds__(256) void absmax_batch_kernel(const SplitJob* jobs) {
  const SplitJob j = jobs[blockIdx.y];
  absmax_part_body(j.src, j.n, j.amax, blockIdx.x, gridDim.x);
}
// blockIdx.x = chunk of SPLIT_CHUNK elements (chunks[] = {job, first}, built on the host)
constexpr unsigned SPLIT_CHUNK = 8192;
static __global__ __launch_bounds__(256) void split_batch_kernel(const SplitJob* jobs, const uint2* chunks) {
  const uint2 c = chunks[blockIdx.x];
  const SplitJob j = jobs[c.x];
  unsigned mb = 0u;
  for (int i = 0; i < SPLIT_PARTS; ++i) mb = max(mb, j.amax[i]);
  const int e = amax_exp(mb);
  const float scale = ldexpf(1.f, e);
  if (c.y == 0 && threadIdx.x == 0) *j.inv = ldexpf(1.f, -e);
  const size_t end = min(j.n, (size_t)c.y + SPLIT_CHUNK);
  for (size_t i = (size_t)c.y + threadIdx.x; i < end; i += 256) {
    const float v = j.src[i] * scale;
    const _Float16 h = (_Float16)v;
    j.hi[i] = h;
    j.lo[i] = (_Float16)(v - (float)h);
  }
}

static __global__ void absmax_kernel(const float* src, size_t n, unsigned* out) {
  float m = 0.f;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    m = fmaxf(m, fabsf(src[i]));
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) atomicMax(out, __float_as_uint(m));  // non-negative floats order as uints
}

}  // namespace dmx

namespace dmx {

// ---------------------------------------------------------------------------
// K5 multi-head attention core in split precision (fp32 values as fp16 hi+lo,
// v_mfma_f32_32x32x16_f16, fp32 accumulate) — nn.MultiheadAttention(C, 4) inner product
// softmax(q k^T / sqrt(D)) v (models/unet_cond.py:36,49).
//
// One wave = 32 queries; 64-key chunks staged in LDS (K as [key][d] hi/lo planes,
// V transposed as [d][key] planes).  S^T = K Q^T (keys on rows, the wave's 32 queries on
// lanes); softmax in the log2 domain (Q pre-scaled by log2(e)/sqrt(D)); then
// O^T += V^T P^T where the S^T accumulator registers 8s..8s+7 are directly the B operand
// of k-step s (row 16s + 8(j>>2) + 4h + (j&3) of the tile), and V^T is read with the same
// key permutation.  D = 16 pads V^T to 32 rows (zero).
// ---------------------------------------------------------------------------
// X1 = 1: config-4 fp16 arithmetic (Q, K, V, P rounded to f16, one MFMA per product).
template <int D, int WPE = 1, int X1 = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void attention_x3_kernel(
    const float* qkv, float* out, int L, int C, float* stats) {
  constexpr int KC = 64, KS = D + 8, VR = D < 32 ? 32 : D, VS = KC + 4, NKS = D / 16, NDT = VR / 32;
  __shared__ __attribute__((aligned(16))) _Float16 Kh[KC][KS];
  __shared__ __attribute__((aligned(16))) _Float16 Kl[X1 ? 1 : KC][KS];
  __shared__ __attribute__((aligned(16))) _Float16 Vh[VR][VS];
  __shared__ __attribute__((aligned(16))) _Float16 Vl[X1 ? 1 : VR][VS];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int hd = blockIdx.y, n = blockIdx.z;
  const int fr = lane & 31, fh = lane >> 5;
  const size_t rs = (size_t)3 * C;
  const float* base = qkv + (size_t)n * L * rs;
  const float qscale = 1.4426950408889634f / sqrtf((float)D);
  const int q = blockIdx.x * 128 + wid * 32 + fr;

  // Q^T fragments (B operand): lane (q, h) holds Q[q][16ks + 8h + j]
  half8 qh[NKS], ql[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    floatx4 a = {0.f, 0.f, 0.f, 0.f}, b = {0.f, 0.f, 0.f, 0.f};
    if (q < L) {
      const float* r = base + (size_t)q * rs + hd * D + 16 * ks + 8 * fh;
      a = ld4(r);
      b = ld4(r + 4);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float va = a[j] * qscale, vb = b[j] * qscale;
      const _Float16 ha = (_Float16)va, hb = (_Float16)vb;
      qh[ks][j] = ha;
      ql[ks][j] = (_Float16)(va - (float)ha);
      qh[ks][j + 4] = hb;
      ql[ks][j + 4] = (_Float16)(vb - (float)hb);
    }
  }
  // D < 32: V^T is padded to 32 rows; row D holds ones so O^T row D accumulates the
  // softmax denominator on the matrix cores (rescaled by alpha with the rest of O).
  constexpr bool ONES = VR > D;
  if constexpr (ONES) {
    for (int i = tid; i < (VR - D) * VS; i += 256) {
      const int r = D + i / VS;
      Vh[r][i % VS] = (_Float16)(r == D ? 1.f : 0.f);
      if constexpr (!X1) Vl[r][i % VS] = (_Float16)0.f;
    }
  }
  floatx16 o[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
  float mrun = -INFINITY, lrun = 0.f;

  // K/V chunk staging, software-pipelined: chunk c+1 is loaded into registers while chunk c
  // is computed, then split into the LDS planes after the barrier.
  constexpr int IT = KC * (D / 4) / 256;  // float4 of K (and of V) per thread per chunk
  static_assert(IT >= 1 && KC * (D / 4) % 256 == 0, "staging");
  floatx4 kr[IT], vr[IT];
  auto load_kv = [&](int c0) {
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int i = tid + 256 * it, key = i / (D / 4), d4 = (i % (D / 4)) * 4;
      const float* r = base + (size_t)min(c0 + key, L - 1) * rs + hd * D + d4;  // clamped: finite
      kr[it] = ld4(r + C);
      vr[it] = ld4(r + 2 * C);
    }
  };
  load_kv(0);
  for (int c0 = 0; c0 < L; c0 += KC) {
    __syncthreads();  // previous chunk fully consumed
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int i = tid + 256 * it, key = i / (D / 4), d4 = (i % (D / 4)) * 4;
      const bool kvalid = c0 + key < L;  // keys past L: zero K / V (their scores are masked)
      const floatx4 z = {0.f, 0.f, 0.f, 0.f};
      half4 h, l;
      if constexpr (X1) {
        *reinterpret_cast<half4*>(&Kh[key][d4]) = __builtin_convertvector(kvalid ? kr[it] : z, half4);
        h = __builtin_convertvector(kvalid ? vr[it] : z, half4);
#pragma unroll
        for (int j = 0; j < 4; ++j) Vh[d4 + j][key] = h[j];
        continue;
      }
      split4(kvalid ? kr[it] : z, h, l);
      *reinterpret_cast<half4*>(&Kh[key][d4]) = h;
      *reinterpret_cast<half4*>(&Kl[key][d4]) = l;
      split4(kvalid ? vr[it] : z, h, l);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        Vh[d4 + j][key] = h[j];
        Vl[d4 + j][key] = l[j];
      }
    }
    __syncthreads();
    if (c0 + KC < L) load_kv(c0 + KC);  // in flight during this chunk's MFMAs
    // S^T for the two 32-key tiles of the chunk
    floatx16 sc[2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
      for (int r = 0; r < 16; ++r) sc[kt][r] = 0.f;
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const half8 kh = *reinterpret_cast<const half8*>(&Kh[kt * 32 + fr][16 * ks + 8 * fh]);
        if constexpr (!X1) {
          const half8 kl = *reinterpret_cast<const half8*>(&Kl[kt * 32 + fr][16 * ks + 8 * fh]);
          sc[kt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kl, qh[ks], sc[kt], 0, 0, 0);
          sc[kt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kh, ql[ks], sc[kt], 0, 0, 0);
        }
        sc[kt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kh, qh[ks], sc[kt], 0, 0, 0);
      }
    }
    // online softmax (log2 domain); lane holds keys (r&3)+8(r>>2)+4h of each tile
    const int nvalid = L - c0;
    if (nvalid < KC) {  // ragged last chunk only (uniform branch)
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
          if (key >= nvalid) sc[kt][r] = -INFINITY;
        }
    }
    float mx = sc[0][0];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sc[kt][r]);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mnew = fmaxf(mrun, mx);
    const float alpha = __builtin_amdgcn_exp2f(mrun - mnew);  // exp2(-inf) = 0 on the first chunk
    mrun = mnew;
    const f32x2 mn2 = {mnew, mnew}, al2 = {alpha, alpha};
    f32x2 ls2 = {0.f, 0.f};
    u32x4 phu[2][2], plu[2][2];  // P^T hi/lo fragments per (key tile, 16-key step)
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int jp = 0; jp < 4; ++jp) {
          f32x2 v = {sc[kt][8 * s + 2 * jp], sc[kt][8 * s + 2 * jp + 1]};
          v -= mn2;
          v.x = __builtin_amdgcn_exp2f(v.x);
          v.y = __builtin_amdgcn_exp2f(v.y);
          if constexpr (!ONES) ls2 += v;
          unsigned h, l;
          if constexpr (X1) {
            h = __builtin_bit_cast(unsigned, __builtin_convertvector(v, half2v));
            l = 0u;
          } else {
            split2(v, h, l);
          }
          phu[kt][s][jp] = h;
          plu[kt][s][jp] = l;
        }
    if constexpr (!ONES) lrun = lrun * alpha + (ls2.x + ls2.y);
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        f32x2 v = {o[dt][r], o[dt][r + 1]};
        v *= al2;
        o[dt][r] = v.x;
        o[dt][r + 1] = v.y;
      }
    // O^T += V^T P^T
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const half8 ph = __builtin_bit_cast(half8, phu[kt][s]);
        const half8 pl = __builtin_bit_cast(half8, plu[kt][s]);
        const int k0 = kt * 32 + 16 * s + 4 * fh;
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          const int d = dt * 32 + fr;
          half8 vh, vl;
          const half4 a0 = *reinterpret_cast<const half4*>(&Vh[d][k0]);
          const half4 a1 = *reinterpret_cast<const half4*>(&Vh[d][k0 + 8]);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            vh[j] = a0[j];
            vh[j + 4] = a1[j];
          }
          if constexpr (!X1) {
            const half4 b0 = *reinterpret_cast<const half4*>(&Vl[d][k0]);
            const half4 b1 = *reinterpret_cast<const half4*>(&Vl[d][k0 + 8]);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              vl[j] = b0[j];
              vl[j + 4] = b1[j];
            }
            o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vl, ph, o[dt], 0, 0, 0);
            o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vh, pl, o[dt], 0, 0, 0);
          }
          o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vh, ph, o[dt], 0, 0, 0);
        }
      }
  }
  if constexpr (ONES) {
    lrun = __shfl(o[0][8], fr, 64);  // O^T row D = 16 lives in reg 8 of the h = 0 lane
  } else {
    lrun += __shfl_xor(lrun, 32, 64);
  }
  const float inv = 1.0f / lrun;
  if (stats != nullptr && fh == 0 && q < L) {  // training forward: (row max, 1 / sum) in natural units
    float* so = stats + (((size_t)n * 4 + hd) * L + q) * 3;
    so[0] = mrun * 0.6931471805599453f;
    so[1] = inv;
  }
  if (q < L) {
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = dt * 32 + 8 * g + 4 * fh;  // rows (r&3) + 8(r>>2) + 4h for r = 4g..4g+3
        if (d < D) {
          floatx4 v;
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = o[dt][4 * g + j] * inv;
          att_st4(out + ((size_t)n * L + q) * C + hd * D + d, v);
        }
      }
  }
}

// ---------------------------------------------------------------------------
// D = 16 attention core with the whole head resident in LDS (sa5 / sa6: C = 64, L = 256 / 784 /
// 1024).  Same arithmetic and operation order as attention_x3_kernel<16> (S^T = K Q^T on
// 32x32x16 MFMAs, log2-domain online softmax over 64-key chunks, O^T += V^T P^T with V^T padded
// to 32 rows whose row 16 is ones, so the denominator comes off the matrix cores), but one
// block per (sample, head) stages that head's K and V^T once — f16 hi / lo planes, L x 16 and
// 16 x L — and then every wave sweeps all keys for its query tiles with no further barrier.
// The per-chunk staging of the 128-query kernel (two barriers per 64 keys, K / V re-read and
// re-split by every query block of the head, 2-byte transposed V stores) is gone.
//
// LDS (dynamic, Lp = L rounded up to 64): Kh, Kl [Lp][16]; Vh [18][Lp + 4] (rows 0-15 V^T,
// 16 ones, 17 zeros); Vl [17][Lp + 4] (row 16 zeros).  The V^T row pitch is 2 mod 32 dwords: the
// 16 rows a ds_read2_b64 lane group reads (banks (a/4) mod 32) cover the 32 banks exactly once.  Lanes 16-31 of a V^T fragment read the
// constant rows instead of holding padding in LDS.  Keys in [L, Lp) are zero and masked.
// ---------------------------------------------------------------------------
__host__ __device__ inline int att16_lp(int L) { return (L + 63) / 64 * 64; }
__host__ __device__ inline size_t att16_lds_bytes(int L, int x1) {
  const size_t lp = (size_t)att16_lp(L), vs = lp + 4;
  return 2 * ((x1 ? 1 : 2) * lp * 16 + (x1 ? 18 : 35) * vs);
}

// Cross-half (lanes l and l ^ 32) max with v_permlane32_swap (a VALU op; __shfl_xor(v, 32) is a
// ds_bpermute round trip through the LDS pipe on the softmax's critical path).
DMX_DEV float max_halves(float v) {
  const unsigned u = __builtin_bit_cast(unsigned, v);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return fmaxf(__builtin_bit_cast(float, (unsigned)r[0]), __builtin_bit_cast(float, (unsigned)r[1]));
}

// v_mfma_f32_32x32x16_f16 with its accumulator input (the loop-invariant -mref) in other registers
// than its result: the builtin's tied form copies negm into the result registers every chunk
// (eight v_mov_b64 on the VALU issue port this kernel is bound by).
DMX_DEV floatx16 mfma_untied(half8 a, half8 b, floatx16 c) {
  floatx16 d;
  asm("v_mfma_f32_32x32x16_f16 %0, %1, %2, %3" : "=&v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}

template <int NW, int X1 = 0>
__global__ __launch_bounds__(NW * 64) void attention16_kernel(const float* qkv, float* out, int L, int C,
                                                              float* stats) {
  constexpr int D = 16;
  extern __shared__ __attribute__((aligned(16))) _Float16 att_lds[];
  const int Lp = att16_lp(L), VS = Lp + 4;
  _Float16* Kh = att_lds;
  _Float16* Kl = Kh + Lp * D;
  _Float16* Vh = Kl + (X1 ? 0 : Lp * D);
  _Float16* Vl = Vh + 18 * VS;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int hd = blockIdx.y, n = blockIdx.z;
  const int fr = lane & 31, fh = lane >> 5;
  const size_t rs = (size_t)3 * C;
  const float* base = qkv + (size_t)n * L * rs + hd * D;

  // stage: a unit = 4 consecutive keys x 4 dims (K rows as half4 stores, V^T rows as half4 stores)
  for (int u = tid; u < Lp; u += NW * 64) {
    const int k0 = (u >> 2) * 4, d4 = (u & 3) * 4;
    floatx4 kv[4], vv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool ok = k0 + j < L;
      const float* r = base + (size_t)(ok ? k0 + j : 0) * rs + d4;
      kv[j] = ok ? ld4(r + C) : floatx4{0.f, 0.f, 0.f, 0.f};
      vv[j] = ok ? ld4(r + 2 * C) : floatx4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      half4 h, l;
      // K row r keeps its two 8-dim halves swapped when bit 3 of r is set: the QK^T fragment reads
      // (lane fr: row c0 + fr, half fh) then hit 16 distinct 16-byte bank slots per ds_read_b128 lane
      // group instead of 2-way conflicts on the plain 32-byte rows
      const int kd = (((d4 >> 3) ^ (((k0 + j) >> 3) & 1)) << 3) | (d4 & 7);
      if constexpr (X1) {
        h = __builtin_convertvector(kv[j], half4);
      } else {
        split4(kv[j], h, l);
        *reinterpret_cast<half4*>(&Kl[(k0 + j) * D + kd]) = l;
      }
      *reinterpret_cast<half4*>(&Kh[(k0 + j) * D + kd]) = h;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const floatx4 t = {vv[0][e], vv[1][e], vv[2][e], vv[3][e]};
      half4 h, l;
      if constexpr (X1) {
        h = __builtin_convertvector(t, half4);
      } else {
        split4(t, h, l);
        *reinterpret_cast<half4*>(&Vl[(d4 + e) * VS + k0]) = l;
      }
      *reinterpret_cast<half4*>(&Vh[(d4 + e) * VS + k0]) = h;
    }
  }
  for (int i = tid; i < VS; i += NW * 64) {
    Vh[16 * VS + i] = (_Float16)1.f;
    Vh[17 * VS + i] = (_Float16)0.f;
    if constexpr (!X1) Vl[16 * VS + i] = (_Float16)0.f;
  }
  __syncthreads();

  const float qscale = 1.4426950408889634f / sqrtf((float)D);
  const _Float16* vrh = Vh + (fr < 16 ? fr : fr == 16 ? 16 : 17) * VS;  // this lane's V^T row (hi)
  const _Float16* vrl = Vl + (fr < 16 ? fr : 16) * VS;                  // (lo)
  const int nqt = (L + 31) / 32;
  for (int qt = wid; qt < nqt; qt += NW) {
    const int q = qt * 32 + fr;
    half8 qh, ql;
    {
      floatx4 a = {0.f, 0.f, 0.f, 0.f}, b = {0.f, 0.f, 0.f, 0.f};
      if (q < L) {
        const float* r = base + (size_t)q * rs + 8 * fh;
        a = ld4(r);
        b = ld4(r + 4);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float va = a[j] * qscale, vb = b[j] * qscale;
        const _Float16 ha = (_Float16)va, hb = (_Float16)vb;
        qh[j] = ha;
        ql[j] = (_Float16)(va - (float)ha);
        qh[j + 4] = hb;
        ql[j + 4] = (_Float16)(vb - (float)hb);
      }
    }
    // Lazily rescaled online softmax: the first S^T MFMA of a tile takes C = -mref, so scores
    // leave the matrix cores already shifted by the running reference max (no per-score
    // subtract), and P = exp2(s - mref).  The reference moves — rescaling O, whose ones row is
    // the denominator — only on a tile's first chunk or when a chunk's max exceeds it by more
    // than TAU (P <= 2^TAU in between: exact in fp32 and in the f16 hi / lo split).  O / l does
    // not depend on the reference.
    constexpr float TAU = 8.f;
    floatx16 o, negm;
#pragma unroll
    for (int r = 0; r < 16; ++r) o[r] = negm[r] = 0.f;
    float mref = 0.f;
    for (int c0 = 0; c0 < L; c0 += 32) {  // 32-key chunks: one S^T tile live (register budget)
      floatx16 sc;
      {
        const int krow = (c0 + fr) * D + 8 * (fh ^ ((fr >> 3) & 1));  // (swizzled halves, c0 % 32 == 0)
        const half8 kh = *reinterpret_cast<const half8*>(&Kh[krow]);
        if constexpr (!X1) {
          const half8 kl = *reinterpret_cast<const half8*>(&Kl[krow]);
          sc = mfma_untied(kl, qh, negm);
          sc = __builtin_amdgcn_mfma_f32_32x32x16_f16(kh, ql, sc, 0, 0, 0);
          sc = __builtin_amdgcn_mfma_f32_32x32x16_f16(kh, qh, sc, 0, 0, 0);
        } else {
          sc = mfma_untied(kh, qh, negm);
        }
      }
      const int nvalid = L - c0;
      if (nvalid < 32) {  // ragged last chunk only (uniform branch)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if ((r & 3) + 8 * (r >> 2) + 4 * fh >= nvalid) sc[r] = -INFINITY;
      }
      float mx = sc[0];
#pragma unroll
      for (int r = 1; r < 16; ++r) mx = fmaxf(mx, sc[r]);
      mx = max_halves(mx);
      if (c0 == 0 || mx > TAU) {  // move the reference to this chunk's max (rare after the first)
        const float alpha = __builtin_amdgcn_exp2f(-mx);
#pragma unroll
        for (int r = 0; r < 16; ++r) o[r] *= alpha;
#pragma unroll
        for (int r = 0; r < 16; ++r) sc[r] -= mx;
        mref += mx;
#pragma unroll
        for (int r = 0; r < 16; ++r) negm[r] = -mref;
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        u32x4 phu, plu;
#pragma unroll
        for (int jp = 0; jp < 4; ++jp) {
          f32x2 v;
          v.x = __builtin_amdgcn_exp2f(sc[8 * s + 2 * jp]);
          v.y = __builtin_amdgcn_exp2f(sc[8 * s + 2 * jp + 1]);
          unsigned h, l;
          if constexpr (X1) {
            h = __builtin_bit_cast(unsigned, __builtin_convertvector(v, half2v));
            l = 0u;
          } else {
            split2(v, h, l);
          }
          phu[jp] = h;
          plu[jp] = l;
        }
        const half8 ph = __builtin_bit_cast(half8, phu);
        const half8 pl = __builtin_bit_cast(half8, plu);
        const int k0 = c0 + 16 * s + 4 * fh;
        half8 vh, vl;
        const half4 a0 = *reinterpret_cast<const half4*>(vrh + k0);
        const half4 a1 = *reinterpret_cast<const half4*>(vrh + k0 + 8);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          vh[j] = a0[j];
          vh[j + 4] = a1[j];
        }
        if constexpr (!X1) {
          const half4 b0 = *reinterpret_cast<const half4*>(vrl + k0);
          const half4 b1 = *reinterpret_cast<const half4*>(vrl + k0 + 8);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            vl[j] = b0[j];
            vl[j + 4] = b1[j];
          }
          o = __builtin_amdgcn_mfma_f32_32x32x16_f16(vl, ph, o, 0, 0, 0);
          o = __builtin_amdgcn_mfma_f32_32x32x16_f16(vh, pl, o, 0, 0, 0);
        }
        o = __builtin_amdgcn_mfma_f32_32x32x16_f16(vh, ph, o, 0, 0, 0);
      }
    }
    const float inv = 1.0f / __shfl(o[8], fr, 64);  // O^T row 16 (the ones row) = the denominator
    if (stats != nullptr && fh == 0 && q < L) {  // training forward: (reference, 1 / sum) in natural units —
      float* so = stats + (((size_t)n * 4 + hd) * L + q) * 3;  // P = exp(s - ref) / sum for any reference
      so[0] = mref * 0.6931471805599453f;
      so[1] = inv;
    }
    if (q < L) {
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        const int d = 8 * g + 4 * fh;
        floatx4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = o[4 * g + j] * inv;
        att_st4(out + ((size_t)n * L + q) * C + hd * D + d, v);
      }
    }
  }
}

}  // namespace dmx

