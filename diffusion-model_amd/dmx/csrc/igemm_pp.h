// dmx — split-precision implicit GEMM, "ping-pong" schedule for the large convolutions (gfx950).
//
// Same arithmetic, operand layouts, geometries and epilogues as igemm_x3_kernel (igemm_x3.h):
// fp32 operands as fp16 hi + lo, three v_mfma_f32_32x32x16_f16 per product, fp32 accumulate.
// What differs is the schedule.  The register-staged kernel runs two independent 4-wave
// blocks per CU whose load / barrier phases tend to line up, so each SIMD's matrix pipe idles
// while both of its waves stage (measured ≈50 % of the attainable MFMA rate on the big convs).
// Here ONE 512-thread block per CU owns a 256 x BN tile as two 4-wave groups (G0 = rows
// 0..127, G1 = rows 128..255; every SIMD hosts one wave of each) that take turns, one
// barrier per phase:
//
//   phase 2k+1:  G0 computes K-tile k        | G1 stores K-tile k+1 (regs -> LDS), loads k+2
//   phase 2k+2:  G1 computes K-tile k        | G0 stores K-tile k+1,               loads k+2
//
// so while one wave of a SIMD issues its 24 MFMAs, its partner does the ds_writes, the
// address arithmetic and the global loads — the MFMA pipe is fed from alternating waves.
// LDS: two buffers of (256 A rows + BN B rows) x 32 k, hi / lo planes, 80-byte rows
// (conflict-free ds_read_b128) = 120 KB at BN = 128.  Each group stages its own 128 A rows
// and half of the B rows; a group's loads land two phases (one group-compute) after issue.
//
// Buffer hazards (k = compute tile): store(k+1) writes buffer (k+1)&1 == (k-1)&1, whose last
// readers (G0 compute(k-1), phase 2k-1; G1 compute(k-1), phase 2k) finished before the
// barriers that precede the stores (phases 2k+1, 2k+2); compute(k) reads buffer k&1, complete
// after phase 2k (G1's half in 2k-1, G0's half in 2k).
#pragma once
#include "common.h"
#include "igemm.h"
#include "igemm_x3.h"

namespace dmx {

template <int BN, int EPI, int SPLIT_A = 0, int X1 = 0>
__global__ __launch_bounds__(512) void igemm_pp_kernel(const X3Params P) {
  const IgemmParams& p = P.g;
  constexpr int BM = 256, GM = 128, BK = 32, RS = BK + 8;
  constexpr int WM = GM / 2, WN = BN / 2, TM = WM / 32, TN = WN / 32;
  constexpr int APR = SPLIT_A ? BK / 8 : BK / 4;  // A pieces per row (8 f16 per plane | 4 fp32)
  constexpr int AP = GM * APR / 256;               // A pieces per group thread
  constexpr int ARS = 256 / APR;                   // rows covered per pass
  constexpr int BPR = BK / 8;                      // 16-byte chunks per B row per plane
  constexpr int BCH = (BN / 2) * BPR;              // B chunks per group (half the B rows)
  static_assert(TM >= 1 && TN >= 1 && AP >= 1 && BCH <= 256, "tile");

  constexpr int LA = X1 ? 1 : BM, LB = X1 ? 1 : BN;
  __shared__ __attribute__((aligned(16))) _Float16 Ah[2][BM][RS];
  __shared__ __attribute__((aligned(16))) _Float16 Al[2][LA][RS];
  __shared__ __attribute__((aligned(16))) _Float16 Bhs[2][BN][RS];
  __shared__ __attribute__((aligned(16))) _Float16 Bls[2][LB][RS];

  const int tid = threadIdx.x, lane = tid & 63;
  const int g = tid >> 8, t = tid & 255, wg = t >> 6;  // group, thread / wave within the group
  const int wm = wg >> 1, wn = wg & 1;
  int mt, nt, bz;
  xcd_tile(mt, nt, bz);
  const int phase = EPI == EPI_PARTIAL ? 0 : bz;
  const int m0 = mt * BM, n0 = nt * BN;
  const int gr0 = g * GM;                                   // this group's first A row in the tile
  const int qa = t % APR, ra = t / APR;
  constexpr int PW = SPLIT_A ? 8 : 4;
  const bool bact = t < BCH;                                // this thread stages a B chunk
  const int qb = t % BPR, rb = g * (BN / 2) + t / BPR;      // B row (within the tile) of that chunk
  const size_t boff = (size_t)phase * p.Npad * p.Kpad;
  const _Float16* Bh = P.Bh + boff;
  const _Float16* Bl = P.Bl + boff;
  const int C = p.src.C;

  int rpix[AP];
  unsigned tmask[AP];
#pragma unroll
  for (int i = 0; i < AP; ++i) {
    const int m = m0 + gr0 + ra + i * ARS;
    rpix[i] = m < p.M ? row_anchor(p.geom, m, p.H, p.W, p.Hin, p.Win) : 0;
    tmask[i] = tap_mask(p.geom, phase, p.taps, m, p.M, p.H, p.W, p.Hin, p.Win);
  }

  // register stage of one K-tile (this thread's A pieces and B chunk); two stages keep two
  // K-tiles in flight per group (loads land four phases after issue)
  struct Stage {
    floatx4 ra4[SPLIT_A ? 1 : AP];
    half8 rah[SPLIT_A ? AP : 1], ral[SPLIT_A ? AP : 1];
    half8 rbh, rbl;
  };
  Stage S0, S1;
  int ltap = 0, lc = 0;
  auto seek = [&](int kt) {
    const int k = kt * BK + qa * PW;
    ltap = k / C;
    lc = k - ltap * C;
  };
  const float* __restrict__ asrc = p.src.src0;
  // buffer-resource addressing as in igemm_x3_kernel (out-of-range offset = zero padding)
  constexpr int AES = SPLIT_A ? 2 : 4;
  const __amdgpu_buffer_rsrc_t rAh = rsrc_of(SPLIT_A ? (const void*)P.Ash : (const void*)asrc, P.a_bytes);
  const __amdgpu_buffer_rsrc_t rAl = rsrc_of(SPLIT_A ? (const void*)P.Asl : (const void*)asrc, P.a_bytes);
  const __amdgpu_buffer_rsrc_t rBh = rsrc_of(Bh, P.b_bytes), rBl = rsrc_of(Bl, P.b_bytes);
  const int boffs = ((n0 + rb) * p.Kpad + qb * 8) * 2;
  // K-tiles must be loaded in order (incremental tap / channel tracking)
  auto load_tile = [&](int kt, Stage& st) {
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
      const bool ok = (tmask[i] >> tap) & 1u;  // padding taps / rows past M read zeros
      const int boff_a = ok ? ((rpix[i] + delta) * C + c) * AES : kOOB;
      if constexpr (SPLIT_A) {
        st.rah[i] = bload_h8(rAh, boff_a, 0);
        if constexpr (!X1) st.ral[i] = bload_h8(rAl, boff_a, 0);
      } else {
        st.ra4[i] = bload_f4(rAh, boff_a, 0);
      }
    }
    if (bact) {
      st.rbh = bload_h8(rBh, boffs, kt * BK * 2);
      if constexpr (!X1) st.rbl = bload_h8(rBl, boffs, kt * BK * 2);
    }
  };
  auto store_tile = [&](int buf, const Stage& st) {
#pragma unroll
    for (int i = 0; i < AP; ++i) {
      const int row = gr0 + ra + i * ARS;
      if constexpr (SPLIT_A) {
        *reinterpret_cast<half8*>(&Ah[buf][row][qa * 8]) = st.rah[i];
        if constexpr (!X1) *reinterpret_cast<half8*>(&Al[buf][row][qa * 8]) = st.ral[i];
      } else if constexpr (X1) {
        *reinterpret_cast<half4*>(&Ah[buf][row][qa * 4]) = __builtin_convertvector(st.ra4[i], half4);
      } else {
        half4 h, l;
        split4(st.ra4[i], h, l);
        *reinterpret_cast<half4*>(&Ah[buf][row][qa * 4]) = h;
        *reinterpret_cast<half4*>(&Al[buf][row][qa * 4]) = l;
      }
    }
    if (bact) {
      *reinterpret_cast<half8*>(&Bhs[buf][rb][qb * 8]) = st.rbh;
      if constexpr (!X1) *reinterpret_cast<half8*>(&Bls[buf][rb][qb * 8]) = st.rbl;
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
  // next k16-step's fragments read while this step's MFMAs issue (as igemm_x3_kernel)
  auto compute = [&](int buf) {
    constexpr int S = BK / 16, NR = (X1 ? 1 : 2) * (TM + TN), NM = (X1 ? 1 : 3) * TM * TN;
    half8 ah[2][TM], al[2][TM], bh[2][TN], bl[2][TN];
    auto ldf = [&](int s, int d) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = gr0 + wm * WM + i * 32 + fr;
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
    __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
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
        for (int r = 0; r < NR; ++r) {
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
  // prologue: K-tile 0 staged into buffer 0 by both groups; K-tiles 1, 2 in flight (S1, S0)
  load_tile(kbeg, S0);
  store_tile(0, S0);
  if (nK > 1) load_tile(kbeg + 1, S1);
  if (nK > 2) load_tile(kbeg + 2, S0);
  __syncthreads();
  // phases 2k+1 (G0 computes k, G1 stores k+1) and 2k+2 (G1 computes k, G0 stores k+1);
  // `st` holds K-tile k+1 and is refilled with K-tile k+3 after its store
  auto phase_pair = [&](int k, Stage& st) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (g == h) {
        compute(k & 1);
      } else if (k + 1 < nK) {
        store_tile((k + 1) & 1, st);
        if (k + 3 < nK) load_tile(kbeg + k + 3, st);
      }
      __syncthreads();
    }
  };
  for (int k = 0; k < nK; k += 2) {
    phase_pair(k, S1);
    if (k + 1 < nK) phase_pair(k + 1, S0);
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] *= P.inv_scale;

  igemm_epilogue<GM, BN, EPI>(p, acc, phase, m0 + gr0, n0, wm, wn, fr, fh);
}

}  // namespace dmx
