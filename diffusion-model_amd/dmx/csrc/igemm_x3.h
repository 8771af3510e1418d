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

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));

constexpr int X3_BK = 32;
constexpr int X3_STRIDE = 40;  // f16 per LDS row (32 + 8 pad) = 80 bytes

struct X3Params {
  IgemmParams g;           // geometry / epilogue (g.Bw unused)
  const _Float16* Bh;      // [phases][Npad][Kpad] scaled hi
  const _Float16* Bl;      //                      scaled lo
  float inv_scale;         // 2^-e
};

DMX_DEV void split4(floatx4 v, half4& h, half4& l) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const _Float16 hi = (_Float16)v[j];
    h[j] = hi;
    l[j] = (_Float16)(v[j] - (float)hi);
  }
}

template <int BM, int BN, int EPI>
__global__ __launch_bounds__(256) void igemm_x3_kernel(const X3Params P) {
  const IgemmParams& p = P.g;
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 32, TN = WN / 32;
  constexpr int AP = BM * 8 / 256;   // float4 pieces of A per thread per K-step (8 per row)
  constexpr int BP = BN * 4 / 256;   // 16-byte chunks of B per plane per thread (4 per row)
  static_assert(TM >= 1 && TN >= 1 && AP >= 1 && BP >= 1, "tile");

  __shared__ __attribute__((aligned(16))) _Float16 Ah[2][BM][X3_STRIDE];
  __shared__ __attribute__((aligned(16))) _Float16 Al[2][BM][X3_STRIDE];
  __shared__ __attribute__((aligned(16))) _Float16 Bhs[2][BN][X3_STRIDE];
  __shared__ __attribute__((aligned(16))) _Float16 Bls[2][BN][X3_STRIDE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int phase = EPI == EPI_PARTIAL ? 0 : blockIdx.z;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int qa = tid & 7, ra = tid >> 3;   // A: piece 0..7 of a row, row (+ i*32)
  const int qb = tid & 3, rb = tid >> 2;   // B: chunk 0..3 of a row, row (+ i*64)
  const size_t boff = (size_t)phase * p.Npad * p.Kpad;
  const _Float16* Bh = P.Bh + boff;
  const _Float16* Bl = P.Bl + boff;
  const int HW = p.H * p.W;
  const int C = p.src.C;

  int an[AP], ay[AP], ax[AP];
  bool av[AP];
#pragma unroll
  for (int i = 0; i < AP; ++i) {
    const int m = m0 + ra + i * 32;
    av[i] = m < p.M;
    const int mm = av[i] ? m : 0;
    an[i] = mm / HW;
    const int r = mm - an[i] * HW;
    ay[i] = r / p.W;
    ax[i] = r - ay[i] * p.W;
  }

  floatx4 ra4[AP];
  half8 rbh[BP], rbl[BP];
  auto load_tile = [&](int kt) {
    const int k = kt * X3_BK + qa * 4;
    const bool kv = k < p.Kreal;
    const int tap = kv ? k / C : 0;
    const int c = k - tap * C;
    const int ddy = p.dy[phase][tap], ddx = p.dx[phase][tap];
#pragma unroll
    for (int i = 0; i < AP; ++i) {
      const int iy = ay[i] + ddy, ix = ax[i] + ddx;
      const bool ok = kv && av[i] && iy >= 0 && ix >= 0 && iy < p.H && ix < p.W;
      ra4[i] = ok ? ld4(p.src.src0 + (((size_t)an[i] * p.H + iy) * p.W + ix) * C + c) : floatx4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < BP; ++i) {
      const size_t o = (size_t)(n0 + rb + i * 64) * p.Kpad + kt * X3_BK + qb * 8;
      rbh[i] = *reinterpret_cast<const half8*>(Bh + o);
      rbl[i] = *reinterpret_cast<const half8*>(Bl + o);
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int i = 0; i < AP; ++i) {
      half4 h, l;
      split4(ra4[i], h, l);
      *reinterpret_cast<half4*>(&Ah[buf][ra + i * 32][qa * 4]) = h;
      *reinterpret_cast<half4*>(&Al[buf][ra + i * 32][qa * 4]) = l;
    }
#pragma unroll
    for (int i = 0; i < BP; ++i) {
      *reinterpret_cast<half8*>(&Bhs[buf][rb + i * 64][qb * 8]) = rbh[i];
      *reinterpret_cast<half8*>(&Bls[buf][rb + i * 64][qb * 8]) = rbl[i];
    }
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  int kbeg = 0, nK = p.Kpad / X3_BK;
  if constexpr (EPI == EPI_PARTIAL) {
    kbeg = blockIdx.z * p.ksplit;
    nK = min(nK - kbeg, p.ksplit);
  }
  load_tile(kbeg);
  store_tile(0);
  __syncthreads();

  const int fr = lane & 31, fh = lane >> 5;
  for (int kt = 0; kt < nK; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nK) load_tile(kbeg + kt + 1);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      half8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WM + i * 32 + fr;
        ah[i] = *reinterpret_cast<const half8*>(&Ah[buf][row][16 * s + 8 * fh]);
        al[i] = *reinterpret_cast<const half8*>(&Al[buf][row][16 * s + 8 * fh]);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * WN + j * 32 + fr;
        bh[j] = *reinterpret_cast<const half8*>(&Bhs[buf][row][16 * s + 8 * fh]);
        bl[j] = *reinterpret_cast<const half8*>(&Bls[buf][row][16 * s + 8 * fh]);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
        }
    }
    if (kt + 1 < nK) store_tile(buf ^ 1);
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] *= P.inv_scale;

  igemm_epilogue<BM, BN, EPI>(p, acc, phase, m0, n0, wm, wn, fr, fh);
}

// Split fp32 weights (already in the B layout) into scaled f16 hi / lo planes.
__global__ void split_weights_kernel(const float* src, _Float16* hi, _Float16* lo, size_t n, float scale) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float v = src[i] * scale;
    const _Float16 h = (_Float16)v;
    hi[i] = h;
    lo[i] = (_Float16)(v - (float)h);
  }
}

__global__ void absmax_kernel(const float* src, size_t n, unsigned* out) {
  float m = 0.f;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    m = fmaxf(m, fabsf(src[i]));
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) atomicMax(out, __float_as_uint(m));  // non-negative floats order as uints
}

}  // namespace dmx
