// dmx — split-precision implicit GEMM with A fragments loaded straight into registers (gfx950).
//
// Same arithmetic, operand layouts, geometries and epilogues as igemm_x3_kernel (igemm_x3.h):
// fp32 operands as fp16 hi + lo, three v_mfma_f32_32x32x16_f16 per product, fp32 accumulate.
//
// Why: in the LDS-staged kernels every A element (hi + lo, 4 B) is written to LDS once per
// block, and LDS stores run at ≈79 B/clk/CU (ds_write_b128, MI355X_MICROARCH.md §LDS) against
// 256 B/clk for ds_read_b128.  At 128 x 128 x 64 tiles the stores alone take ≈830 LDS cycles
// per K-tile, the fragment reads ≈510, the block's MFMAs 1536 per SIMD — with two blocks per
// CU the LDS array is ≈87 % busy at full MFMA rate, so any non-overlap shows directly.
//
// Here a wave owns WR = 32·TMW whole GEMM rows and all BN columns of its block, so its A
// fragments are not shared with any other wave: lane (r, h) loads the 8 consecutive channels
// k = 16s + 8h .. +7 of its row r for k16 step s straight from the NHWC source (buffer loads,
// out-of-range offset = zero padding), one K-tile ahead, and feeds them to the MFMAs (fp32
// sources are split to hi / lo in registers).  Only B (BN x 32 k, hi / lo) goes through LDS,
// double-buffered, one barrier per K-tile; per wave and k16 step that is TN·2 fragment reads
// for TMW·TN·3 MFMAs.
#pragma once
#include "common.h"
#include "igemm.h"
#include "igemm_x3.h"

namespace dmx {

template <int TMW, int BN, int EPI, int SPLIT_A = 0, int X1 = 0, int NWV = 4>
__global__ __launch_bounds__(NWV * 64) void igemm_ad_kernel(const X3Params P) {
  const IgemmParams& p = P.g;
  constexpr int NT = NWV * 64;
  constexpr int WR = 32 * TMW, BM = NWV * WR, TN = BN / 32;
  constexpr int BK = 32, RS = BK + 8, NS = BK / 16;  // K-tile, LDS row (f16), k16 steps per tile
  constexpr int BPR = BK / 8;                        // 16-byte B chunks per row per plane
  constexpr int BP = BN * BPR / NT;                  // B chunks per thread per plane
  constexpr int BRS = NT / BPR;                      // B rows covered per pass
  static_assert(TN >= 1 && BP >= 1 && (BN * BPR) % NT == 0, "tile");
  constexpr int LB = X1 ? 1 : BN;
  __shared__ __attribute__((aligned(16))) _Float16 Bhs[2][BN][RS];
  __shared__ __attribute__((aligned(16))) _Float16 Bls[2][LB][RS];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int fr = lane & 31, fh = lane >> 5;
  int mt, nt, bz;
  xcd_tile(mt, nt, bz);
  const int phase = EPI == EPI_PARTIAL ? 0 : bz;
  const int m0 = mt * BM + w * WR, n0 = nt * BN;  // this wave's first row
  const int qb = tid % BPR, rb = tid / BPR;
  const size_t boff = (size_t)phase * p.Npad * p.Kpad;
  const int C = p.src.C;

  int rpix[TMW];
  unsigned tmask[TMW];
#pragma unroll
  for (int i = 0; i < TMW; ++i) {
    const int m = m0 + i * 32 + fr;
    rpix[i] = m < p.M ? row_anchor(p.geom, m, p.H, p.W, p.Hin, p.Win) : 0;
    tmask[i] = tap_mask(p.geom, phase, p.taps, m, p.M, p.H, p.W, p.Hin, p.Win);
  }

  constexpr int AES = SPLIT_A ? 2 : 4;  // bytes per A element
  const __amdgpu_buffer_rsrc_t rAh = rsrc_of(SPLIT_A ? (const void*)P.Ash : (const void*)p.src.src0, P.a_bytes);
  const __amdgpu_buffer_rsrc_t rAl = rsrc_of(SPLIT_A ? (const void*)P.Asl : (const void*)p.src.src0, P.a_bytes);
  const __amdgpu_buffer_rsrc_t rBh = rsrc_of(P.Bh + boff, P.b_bytes), rBl = rsrc_of(P.Bl + boff, P.b_bytes);
  int boffs[BP];
#pragma unroll
  for (int i = 0; i < BP; ++i) boffs[i] = ((n0 + rb + i * BRS) * p.Kpad + qb * 8) * 2;

  // one K-tile of this lane's A fragments (split planes, or 8 fp32 per fragment)
  struct AStage {
    half8 h[SPLIT_A ? NS : 1][TMW], l[SPLIT_A ? NS : 1][TMW];
    floatx4 f[SPLIT_A ? 1 : NS][TMW][2];
  };
  half8 rbh[BP], rbl[BP];
  int ltap = 0, lc = 0;  // wave-uniform (tap, channel) of the next A K-tile (C % BK == 0)
  auto seek = [&](int kt) {
    const int k = kt * BK;
    ltap = k / C;
    lc = k - ltap * C;
  };
  // K-tiles must be loaded in order (incremental tap / channel tracking)
  auto load_a = [&](AStage& st) {
    int ddy, ddx;
    tap_offset(p.geom, phase, ltap, ddy, ddx);
    const int delta = ddy * p.Win + ddx;
    const int tap = ltap, c = lc + 8 * fh;
    lc += BK;
    if (lc >= C) {
      lc -= C;
      ++ltap;
    }
#pragma unroll
    for (int i = 0; i < TMW; ++i) {
      const bool ok = (tmask[i] >> tap) & 1u;  // padding taps / rows past M read zeros
      const int off = ((rpix[i] + delta) * C + c) * AES;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        if constexpr (SPLIT_A) {
          const int o = ok ? off + s * 16 * AES : kOOB;
          st.h[s][i] = bload_h8(rAh, o, 0);
          if constexpr (!X1) st.l[s][i] = bload_h8(rAl, o, 0);
        } else {
          st.f[s][i][0] = bload_f4(rAh, ok ? off + s * 16 * AES : kOOB, 0);
          st.f[s][i][1] = bload_f4(rAh, ok ? off + s * 16 * AES + 16 : kOOB, 0);
        }
      }
    }
  };
  auto load_b = [&](int kt) {
#pragma unroll
    for (int i = 0; i < BP; ++i) {
      rbh[i] = bload_h8(rBh, boffs[i], kt * BK * 2);
      if constexpr (!X1) rbl[i] = bload_h8(rBl, boffs[i], kt * BK * 2);
    }
  };
  auto store_b = [&](int buf) {
#pragma unroll
    for (int i = 0; i < BP; ++i) {
      *reinterpret_cast<half8*>(&Bhs[buf][rb + i * BRS][qb * 8]) = rbh[i];
      if constexpr (!X1) *reinterpret_cast<half8*>(&Bls[buf][rb + i * BRS][qb * 8]) = rbl[i];
    }
  };

  floatx16 acc[TMW][TN];
#pragma unroll
  for (int i = 0; i < TMW; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto compute = [&](int buf, const AStage& st) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      half8 ah[TMW], al[TMW];
#pragma unroll
      for (int i = 0; i < TMW; ++i) {
        if constexpr (SPLIT_A) {
          ah[i] = st.h[s][i];
          if constexpr (!X1) al[i] = st.l[s][i];
        } else if constexpr (X1) {
          const half4 h0 = __builtin_convertvector(st.f[s][i][0], half4);
          const half4 h1 = __builtin_convertvector(st.f[s][i][1], half4);
          ah[i] = __builtin_shufflevector(h0, h1, 0, 1, 2, 3, 4, 5, 6, 7);
        } else {
          half4 h0, l0, h1, l1;
          split4(st.f[s][i][0], h0, l0);
          split4(st.f[s][i][1], h1, l1);
          ah[i] = __builtin_shufflevector(h0, h1, 0, 1, 2, 3, 4, 5, 6, 7);
          al[i] = __builtin_shufflevector(l0, l1, 0, 1, 2, 3, 4, 5, 6, 7);
        }
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = j * 32 + fr;
        const half8 bh = *reinterpret_cast<const half8*>(&Bhs[buf][row][16 * s + 8 * fh]);
        half8 bl;
        if constexpr (!X1) bl = *reinterpret_cast<const half8*>(&Bls[buf][row][16 * s + 8 * fh]);
#pragma unroll
        for (int i = 0; i < TMW; ++i) {
          if constexpr (!X1) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh, acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl, acc[i][j], 0, 0, 0);
          }
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh, acc[i][j], 0, 0, 0);
        }
      }
    }
  };

  int kbeg = 0, nK = p.Kpad / BK;
  if constexpr (EPI == EPI_PARTIAL) {
    kbeg = blockIdx.z * p.ksplit;
    nK = min(nK - kbeg, p.ksplit);
  }
  seek(kbeg);
  AStage A0, A1;
  // prologue: B tile 0 in LDS buffer 0, B tile 1 in registers; A tiles 0 and 1 in flight
  load_b(kbeg);
  load_a(A0);
  store_b(0);
  if (nK > 1) {
    load_b(kbeg + 1);
    load_a(A1);
  }
  __syncthreads();
  // iteration k: MFMAs of tile k (A from `cur`, B from LDS buffer k&1); then B tile k+1 to
  // LDS buffer (k+1)&1 (last read by tile k-1, before the previous barrier); refill `cur`
  // and the B registers with tile k+2.
  auto iter = [&](int k, AStage& cur) {
    compute(k & 1, cur);
    if (k + 1 < nK) store_b((k + 1) & 1);
    if (k + 2 < nK) {
      load_b(kbeg + k + 2);
      load_a(cur);
    }
    __syncthreads();
  };
  for (int k = 0; k < nK; k += 2) {
    iter(k, A0);
    if (k + 1 < nK) iter(k + 1, A1);
  }
#pragma unroll
  for (int i = 0; i < TMW; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] *= P.inv_scale;

  // each 32-row slice of the wave's accumulators in the shared epilogue's (2x2-wave) indexing:
  // a 64 x (2·BN) tile seen from wave (0, 0) has exactly 1 x TN 32x32 blocks at (m, n0)
  // (written out: a loop over the slices is not unrolled and spills the accumulators)
  static_assert(TMW == 1 || TMW == 2, "TMW");
  igemm_epilogue<64, 2 * BN, EPI>(p, reinterpret_cast<floatx16(&)[1][TN]>(acc[0]), phase, m0, n0, 0, 0, fr, fh);
  if constexpr (TMW == 2)
    igemm_epilogue<64, 2 * BN, EPI>(p, reinterpret_cast<floatx16(&)[1][TN]>(acc[1]), phase, m0 + 32, n0, 0, 0, fr,
                                    fh);
}

}  // namespace dmx
