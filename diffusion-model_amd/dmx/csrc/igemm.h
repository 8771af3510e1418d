// dmx — implicit GEMM on fp32 MFMA (v_mfma_f32_32x32x2_f32) for gfx950.
//
//   C[m, n] = sum_k A[m, k] * B[n, k]      m: output pixel/token, n: out channel
//
// One kernel serves conv3x3 (9 taps), each phase of ConvTranspose 4x4/s2
// (4 taps per phase, blockIdx.z = phase) and token Linear layers (1 tap).
// A is gathered on the fly from a fused source (source.h: plain NHWC,
// GroupNorm+GELU of a raw conv output, 2x2 max-pool, bilinear-x2+pad+concat,
// NCHW input); B is the repacked weight [phase][Npad][Kpad] (k contiguous,
// k = tap * C + c).  fp32 in / fp32 accumulate: each MFMA is bit-for-bit an
// fmaf chain, so no precision is traded for the matrix cores.
//
// Tiling: 256 threads = 4 waves in a 2x2 grid; block tile BM x BN, K-step 16,
// LDS double buffer (rows padded to 20 floats => conflict-free ds_read_b128),
// register-staged global loads for tile k+1 issued before the MFMAs of tile k.
// Inside a K-step lane (r, h) feeds k = 8h + s to MFMA s, so every fragment is
// two contiguous ds_read_b128 (the k order inside an MFMA is free as long as A
// and B agree).
#pragma once
#include "common.h"
#include "source.h"

namespace dmx {

struct IgemmParams {
  SrcDesc src;
  int H, W;           // GEMM row grid (input grid of the conv / token grid)
  int M;              // rows = N * H * W
  int taps;
  int geom;           // 0: linear (1 tap), 1: conv3x3 pad 1, 2: ConvTranspose 4x4/s2 phase (4 taps),
                      // 3: Conv2d 4x4 / stride 2 / pad 1 (16 taps; rows = output pixels)
  int Hin, Win;       // source map (== H, W except geom 3: 2H, 2W)
  int Kreal, Kpad;
  int Cout, Npad;
  int osy, osx;       // output stride (2 for ConvT phases)
  int Hout, Wout;
  const float* Bw;    // [phases][Npad][Kpad]
  const float* bias;  // [Cout] or null
  float* out;         // NHWC [N][Hout][Wout][Cout]
  const float* res;   // EPI_BIAS_RES residual, same layout as out
  float2* rowpart;    // EPI_STATS: GroupNorm partials, see stats_row()
  int seg;            // columns per GroupNorm partial (power of two, <= 32)
  int rgrp;           // rows per partial: 32 (needs H*W % 32 == 0) or 1
  int nphase;         // phases of this GEMM (1, or 4 for ConvT)
  int ksplit;         // EPI_PARTIAL: K-tiles per split (blockIdx.z = split; phases must be 1)
  float* partial;     // EPI_PARTIAL: [splits][M][Cout]
  int gexact;         // EPI_BIAS_GELU: 1 = erf-form GELU (exact-fp32 mode)
};

constexpr int IG_BK = 16;

// Input offset of `tap` (no memory lookups: a runtime-indexed kernarg table costs a global load
// + vmcnt(0) per K-step, which drains the software pipeline).
DMX_DEV void tap_offset(int geom, int phase, int tap, int& dy, int& dx) {
  if (geom == 1) {
    const int ty = (tap * 11) >> 5;  // tap / 3 for tap in [0, 8]
    dy = ty - 1;
    dx = tap - 3 * ty - 1;
  } else if (geom == 2) {  // ConvT 4x4/s2/p1, output parity (py, px) = phase bits
    const int jy = tap >> 1, jx = tap & 1;
    dy = (phase >> 1) ? 1 - jy : -jy;
    dx = (phase & 1) ? 1 - jx : -jx;
  } else if (geom == 3) {  // tap = ky * 4 + kx; input (2y + ky - 1, 2x + kx - 1)
    dy = (tap >> 2) - 1;
    dx = (tap & 3) - 1;
  } else {
    dy = dx = 0;
  }
}

// Source-map pixel index of GEMM row m's tap origin (geom 3: the stride-2 anchor (2y, 2x) in
// the Hin x Win input; otherwise the row's own pixel).
DMX_DEV int row_anchor(int geom, int m, int H, int W, int Hin, int Win) {
  if (geom != 3) return m;
  const int HW = H * W, n = m / HW, r = m - n * HW, y = r / W, x = r - y * W;
  return (n * Hin + 2 * y) * Win + 2 * x;
}

// XCD-aware tile order (cdna_hip_programming.md T1): hardware deals consecutive block ids
// round-robin over the 8 XCDs; remap so every XCD walks a contiguous range of logical tiles
// with the N tile fastest — the N tiles and the spatially neighbouring M tiles that re-read
// the same input rows (3x3 taps) then share one L2.  Bijective for any grid size.
// Bitmask of the taps whose input pixel of output row m is inside the H x W map
// (bit t = tap t of the GEMM geometry; 0 for m >= M).
DMX_DEV unsigned tap_mask(int geom, int phase, int taps, int m, int M, int H, int W, int Hin = 0, int Win = 0) {
  if (m >= M) return 0u;
  if (geom == 0) return 1u;
  const int HW = H * W, n = m / HW, r = m - n * HW, y = r / W, x = r - y * W;
  if (geom == 3) {  // 4x4 / s2 / p1: rows and columns 2y-1 .. 2y+2 of the Hin x Win input
    unsigned ry = 0u, cx = 0u;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      ry |= (2 * y + k - 1 >= 0 && 2 * y + k - 1 < Hin) ? 1u << k : 0u;
      cx |= (2 * x + k - 1 >= 0 && 2 * x + k - 1 < Win) ? 1u << k : 0u;
    }
    unsigned mk = 0u;
#pragma unroll
    for (int k = 0; k < 4; ++k) mk |= ((ry >> k) & 1u) ? cx << (4 * k) : 0u;
    return mk;
  }
  if (geom == 1) {  // 3x3, pad 1: outer product of row / column validity
    const unsigned ry = (y > 0 ? 1u : 0u) | 2u | (y < H - 1 ? 4u : 0u);
    const unsigned cx = (x > 0 ? 1u : 0u) | 2u | (x < W - 1 ? 4u : 0u);
    return ((ry & 1u) ? cx : 0u) | ((ry & 2u) ? cx << 3 : 0u) | ((ry & 4u) ? cx << 6 : 0u);
  }
  unsigned mk = 0;
  for (int t = 0; t < taps; ++t) {
    int dy, dx;
    tap_offset(geom, phase, t, dy, dx);
    if (y + dy >= 0 && y + dy < H && x + dx >= 0 && x + dx < W) mk |= 1u << t;
  }
  return mk;
}

DMX_DEV void xcd_tile(int& mt, int& nt, int& z) {
  const int nm = gridDim.x, nn = gridDim.y;
  const int total = nm * nn;
  const int b = blockIdx.y * nm + blockIdx.x;  // dispatch order (x fastest)
  const int xcd = b & 7, q = total >> 3, r = total & 7;
  const int t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  mt = t / nn;
  nt = t - mt * nn;
  z = blockIdx.z;
}
constexpr int IG_LDS_STRIDE = 20;  // floats per LDS row (16 + 4 pad)

// Shared epilogue of the implicit GEMMs: accumulators (C/D layout of the 32x32 MFMA:
// col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5)) -> split-K slab | output (+bias,
// GELU, residual) and GroupNorm partials.
// RPERM = 1: the A operand's fragment rows 16..31 were read in the rotated order of
// igemm_halo_kernel<W = 16> (fragment row i >= 16 holds tile row 16 + ((i - 18) & 15)).
template <int BM, int BN, int EPI, int RPERM = 0>
DMX_DEV void igemm_epilogue(const IgemmParams& p, floatx16 (&acc)[BM / 64][BN / 64], int phase, int m0, int n0,
                            int wm, int wn, int fr, int fh) {
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 32, TN = WN / 32;
  // RPERM: tile row of fragment row i = (r & 3) + 8 (r >> 2) + 4 fh is i + adj, adj = 14 for
  // i = 16, 17 (r = 8, 9 with fh = 0), -2 for the other i >= 16 (r >= 8), 0 below
#define rperm_adj(r) ((RPERM && (r) >= 8) ? (((r) <= 9 && fh == 0) ? 14 : -2) : 0)
  const int HW = p.H * p.W;
  if constexpr (EPI == EPI_PARTIAL) {
    float* dst = p.partial + (size_t)blockIdx.z * p.M * p.Cout;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh + rperm_adj(r);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = n0 + wn * WN + j * 32 + fr;
          if (m < p.M && col < p.Cout) {
            dst[(size_t)m * p.Cout + col] = acc[i][j][r];
          }
        }
      }
    return;
  }
  const int nseg = EPI == EPI_STATS ? p.Cout / p.seg : 1;
  const bool strided = p.geom == 2;  // ConvT phases scatter rows; otherwise output row = m
  float bj[TN];                      // bias of this lane's columns, loaded once
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn * WN + j * 32 + fr;
    bj[j] = (p.bias != nullptr && col < p.Cout) ? p.bias[col] : 0.f;
  }
  if (!strided && (EPI != EPI_STATS || p.rgrp == 32)) {
    // common case: output row = m, GroupNorm partials per 32-row group (no index divisions)
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      float s1[TN], s2[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) s1[j] = s2[j] = 0.f;
      const int mb = m0 + wm * WM + i * 32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = mb + (r & 3) + 8 * (r >> 2) + 4 * fh + rperm_adj(r);
        const bool mv = m < p.M;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = n0 + wn * WN + j * 32 + fr;
          const bool v = mv && col < p.Cout;
          float val = acc[i][j][r] + bj[j];
          if constexpr (EPI == EPI_BIAS_GELU) val = p.gexact ? gelu_exact(val) : gelu(val);
          if constexpr (EPI == EPI_BIAS_RES) {
            if (v) val += p.res[(size_t)m * p.Cout + col];
          }
          if (v) p.out[(size_t)m * p.Cout + col] = val;
          if constexpr (EPI == EPI_STATS) {
            const float a1 = v ? val : 0.f;
            s1[j] += a1;
            s2[j] += a1 * a1;
          }
        }
      }
      if constexpr (EPI == EPI_STATS) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          float t1 = s1[j], t2 = s2[j];
          for (int o = 1; o < p.seg; o <<= 1) {
            t1 += __shfl_xor(t1, o, 64);
            t2 += __shfl_xor(t2, o, 64);
          }
          t1 += __shfl_xor(t1, 32, 64);
          t2 += __shfl_xor(t2, 32, 64);
          const int col = n0 + wn * WN + j * 32 + fr;
          if (mb < p.M && col < p.Cout && fh == 0 && (fr & (p.seg - 1)) == 0) {
            const int nn = mb / HW, lg = (mb - nn * HW) / 32;
            const size_t er = ((size_t)nn * p.nphase + phase) * (HW / 32) + lg;
            p.rowpart[er * nseg + col / p.seg] = make_float2(t1, t2);
          }
        }
      }
    }
    return;
  }
  // general case: ConvT phase scatter and / or per-row GroupNorm partials
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    float s1[TN], s2[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) s1[j] = s2[j] = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * fh;
      const int m = m0 + wm * WM + i * 32 + row + rperm_adj(r);
      const bool mv = m < p.M;
      size_t oidx = (size_t)m;
      int nn = 0, rr = 0;
      if (mv && (strided || (EPI == EPI_STATS && p.rgrp != 32))) {
        nn = m / HW;
        rr = m - nn * HW;
        if (strided) {
          const int y = rr / p.W, x = rr - y * p.W;
          const int py = phase >> 1, px = phase & 1;
          oidx = ((size_t)nn * p.Hout + (y * p.osy + py)) * p.Wout + (x * p.osx + px);
        }
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = n0 + wn * WN + j * 32 + fr;
        const bool v = mv && col < p.Cout;
        float val = acc[i][j][r] + bj[j];
        if constexpr (EPI == EPI_BIAS_GELU) val = p.gexact ? gelu_exact(val) : gelu(val);
        if constexpr (EPI == EPI_BIAS_RES) {
          if (v) val += p.res[oidx * p.Cout + col];
        }
        if (v) p.out[oidx * p.Cout + col] = val;
        if constexpr (EPI == EPI_STATS) {
          const float a1 = v ? val : 0.f;
          if (p.rgrp == 32) {  // accumulate the lane's 16 rows, reduce across lanes below
            s1[j] += a1;
            s2[j] += a1 * a1;
          } else {
            float t1 = a1, t2 = a1 * a1;
            for (int o = 1; o < p.seg; o <<= 1) {
              t1 += __shfl_xor(t1, o, 64);
              t2 += __shfl_xor(t2, o, 64);
            }
            const size_t er = ((size_t)nn * p.nphase + phase) * HW + rr;
            if (v && (fr & (p.seg - 1)) == 0) p.rowpart[er * nseg + col / p.seg] = make_float2(t1, t2);
          }
        }
      }
    }
    if constexpr (EPI == EPI_STATS) {
      if (p.rgrp == 32) {
        const int mb = m0 + wm * WM + i * 32;  // 32-row group, within one sample (HW % 32 == 0)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          float t1 = s1[j], t2 = s2[j];
          for (int o = 1; o < p.seg; o <<= 1) {
            t1 += __shfl_xor(t1, o, 64);
            t2 += __shfl_xor(t2, o, 64);
          }
          t1 += __shfl_xor(t1, 32, 64);
          t2 += __shfl_xor(t2, 32, 64);
          const int col = n0 + wn * WN + j * 32 + fr;
          if (mb < p.M && col < p.Cout && fh == 0 && (fr & (p.seg - 1)) == 0) {
            const int nn = mb / HW, lg = (mb - nn * HW) / 32;
            const size_t er = ((size_t)nn * p.nphase + phase) * (HW / 32) + lg;
            p.rowpart[er * nseg + col / p.seg] = make_float2(t1, t2);
          }
        }
      }
    }
  }
#undef rperm_adj
}

template <int BM, int BN, int SRC, int EPI>
__global__ __launch_bounds__(256) void igemm_f32_kernel(const IgemmParams p) {
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 32, TN = WN / 32;
  constexpr int AP = BM * 4 / 256, BP = BN * 4 / 256;
  static_assert(TM >= 1 && TN >= 1 && AP >= 1 && BP >= 1, "tile");

  __shared__ __attribute__((aligned(16))) float As[2][BM][IG_LDS_STRIDE];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN][IG_LDS_STRIDE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  int mt, nt, bz;
  xcd_tile(mt, nt, bz);
  const int phase = EPI == EPI_PARTIAL ? 0 : bz;
  const int m0 = mt * BM, n0 = nt * BN;
  const int q = tid & 3;          // float4 piece within a 16-wide K slice
  const int rbase = tid >> 2;     // staging row (+ i * 64)
  const float* Bw = p.Bw + (size_t)phase * p.Npad * p.Kpad;
  const int HW = p.H * p.W;
  const int C = p.src.C;

  // per staged A row: decode m -> (n, y, x) once
  int an[AP], ay[AP], ax[AP];
  bool av[AP];
#pragma unroll
  for (int i = 0; i < AP; ++i) {
    const int m = m0 + rbase + i * 64;
    av[i] = m < p.M;
    const int mm = av[i] ? m : 0;
    an[i] = mm / HW;
    const int r = mm - an[i] * HW;
    ay[i] = r / p.W;
    ax[i] = r - ay[i] * p.W;
    if (p.geom == 3) {  // stride-2 anchor in the source map
      ay[i] *= 2;
      ax[i] *= 2;
    }
  }

  floatx4 ra[AP], rb[BP];
  auto load_tile = [&](int kt) {
    const int k = kt * IG_BK + q * 4;
    const bool kv = k < p.Kreal;
    const int tap = kv ? k / C : 0;
    const int c = k - tap * C;
    int ddy, ddx;
    tap_offset(p.geom, phase, tap, ddy, ddx);
#pragma unroll
    for (int i = 0; i < AP; ++i) {
      const int iy = ay[i] + ddy, ix = ax[i] + ddx;
      const bool ok = kv && av[i] && iy >= 0 && ix >= 0 && iy < p.Hin && ix < p.Win;
      ra[i] = ok ? load_src4<SRC>(p.src, an[i], iy, ix, c, p.Hin, p.Win) : floatx4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < BP; ++i)
      rb[i] = ld4(Bw + (size_t)(n0 + rbase + i * 64) * p.Kpad + kt * IG_BK + q * 4);
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int i = 0; i < AP; ++i) *reinterpret_cast<floatx4*>(&As[buf][rbase + i * 64][q * 4]) = ra[i];
#pragma unroll
    for (int i = 0; i < BP; ++i) *reinterpret_cast<floatx4*>(&Bs[buf][rbase + i * 64][q * 4]) = rb[i];
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  int kbeg = 0, nK = p.Kpad / IG_BK;
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
    floatx4 a[TM][2], b[TN][2];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const float* ap = &As[buf][wm * WM + i * 32 + fr][8 * fh];
      a[i][0] = ld4(ap);
      a[i][1] = ld4(ap + 4);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const float* bp = &Bs[buf][wn * WN + j * 32 + fr][8 * fh];
      b[j][0] = ld4(bp);
      b[j][1] = ld4(bp + 4);
    }
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][s >> 2][s & 3], b[j][s >> 2][s & 3], acc[i][j], 0, 0, 0);
    if (kt + 1 < nK) store_tile(buf ^ 1);
    __syncthreads();
  }

  igemm_epilogue<BM, BN, EPI>(p, acc, phase, m0, n0, wm, wn, fr, fh);
}

// Split-K reduction + the epilogue the GEMM would have applied (deterministic:
// slabs summed in split order).  One thread per 4 columns of a row; a 32-column
// GroupNorm segment is 8 consecutive threads.
struct SplitkParams {
  const float* partial; int splits; int M, Cout;
  const float* bias; const float* res; float* out; float2* rowpart; int seg; int epi;
  int gexact;  // EPI_BIAS_GELU: erf-form GELU
};

static __global__ __launch_bounds__(256) void splitk_reduce_kernel(const SplitkParams p) {
  const int C4 = p.Cout / 4;
  const size_t total = (size_t)p.M * C4;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const bool valid = i < total;
  const size_t m = valid ? i / C4 : 0;
  const int c = valid ? (int)(i % C4) * 4 : 0;
  floatx4 v = {0.f, 0.f, 0.f, 0.f};
  if (valid) {
    for (int s = 0; s < p.splits; ++s) {
      const floatx4 a = ld4(p.partial + ((size_t)s * p.M + m) * p.Cout + c);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] += a[j];
    }
    if (p.bias != nullptr) {
      const floatx4 b = ld4(p.bias + c);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] += b[j];
    }
    if (p.epi == EPI_BIAS_GELU) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = p.gexact ? gelu_exact(v[j]) : gelu(v[j]);
    } else if (p.epi == EPI_BIAS_RES) {
      const floatx4 r = ld4(p.res + m * p.Cout + c);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] += r[j];
    }
    *reinterpret_cast<floatx4*>(p.out + m * p.Cout + c) = v;
  }
  if (p.epi == EPI_STATS) {
    // lanes of one segment are consecutive (seg/4 threads; Cout % seg == 0)
    float s1 = valid ? v[0] + v[1] + v[2] + v[3] : 0.f;
    float s2 = valid ? v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3] : 0.f;
    for (int o = 1; o < p.seg / 4; o <<= 1) {
      s1 += __shfl_xor(s1, o, 64);
      s2 += __shfl_xor(s2, o, 64);
    }
    if (valid && (c % p.seg) == 0) p.rowpart[m * (p.Cout / p.seg) + c / p.seg] = make_float2(s1, s2);
  }
}

}  // namespace dmx
