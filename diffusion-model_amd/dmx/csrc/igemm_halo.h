// dmx — split-precision 3x3 convolution with the input halo staged once per channel chunk
// ("halo conv"), gfx950.
//
// Same arithmetic as igemm_x3_kernel (igemm_x3.h): fp32 operands as fp16 hi + lo, three
// v_mfma_f32_32x32x16_f16 per product (al*bh, ah*bl, ah*bh), fp32 accumulate, weights pre-split
// and pre-scaled.  What differs is how A reaches LDS.  The implicit GEMMs stage A per K-tile =
// (tap, channel slice), so every input pixel is loaded, (split,) and written to LDS nine times.
// Here a 512-thread block owns 256 output pixels (TR whole image rows of one sample, W = 16 or
// 32) x BN output channels and walks K as (32-channel chunk) x (9 taps): the chunk's input halo
// — (TR + 2) x (W + 2) pixels, zero outside the image — is staged ONCE as f16 hi / lo planes, and
// the nine taps read their A fragments from it at a per-tap pixel offset (row r of a fragment is
// output pixel (y, x) of the tile; tap (dy, dx) reads halo pixel (y + 1 + dy, x + 1 + dx)).
// A staging falls from 9 to (TR + 2)(W + 2) / (TR W) = 1.33 (W = 32) / 1.27 (W = 16) loads per
// input element; only the B (weight) slice is staged per step.
//
// K order (sum order of every output element): chunk-major, taps 0..8 inside a chunk, k16 steps
// inside a tap — a fixed function of (C, tap geometry), independent of the grid.
//
// Schedule: one barrier per (chunk, tap) step.  Step s computes from A buffer (chunk & 1) and B
// buffer (s & 1); the B slice of step s + 1 is loaded into registers at the start of step s and
// written to B buffer (s + 1) & 1 after the step's MFMAs (that buffer's readers, step s - 1, passed
// the barrier ending step s - 1); the next chunk's halo is loaded at the chunk's tap 0 and written
// to the other A buffer after tap 1 (its readers, the previous chunk, finished before tap 0).
// LDS (80-byte rows, conflict-free ds_read_b128 as in igemm_x3): A 2 x HP x 40 f16 x 2 planes
// (108.8 KB at W = 32), B 2 x BN x 40 f16 x 2 planes (41 KB at BN = 128): one block per CU, two
// waves per SIMD.  Waves: 4 (rows) x 2 (columns), 64 x BN/2 each.
//
// Low resolution (W = 8, 4; square maps): a 256-pixel tile is 256 / W² WHOLE samples.  Their halos
// are stacked in one LDS image with the zero borders shared: row pitch W + 1 (the zero column right
// of image row y is the zero column left of row y + 1), one zero row before every sample and after
// the last, i.e. sample s row y sits in halo row 1 + s (W + 1) + y.  Every tap (dy, dx) of every
// output pixel then reads halo slot base + dy (W + 1) + dx, zero exactly where the reference pads.
// Halo pixels per output pixel: 1.30 (W = 8) / 1.59 (W = 4) instead of the implicit GEMM's 9.
// The last tile may hold fewer samples (batch not a multiple of 256 / W²): the missing ones stage
// as zeros and the epilogue drops their rows.
// Those convs are too small to fill 256 CUs with whole-K tiles, so they split K over channel chunks
// (EPI_PARTIAL: split z owns chunks [z P.g.ksplit, (z + 1) P.g.ksplit), its partial sums go to slab
// z, reduced in split order by reduce_norm_kernel / splitk_reduce_kernel like the implicit GEMMs').
#pragma once
#include "common.h"
#include "igemm.h"
#include "igemm_x3.h"

namespace dmx {

// GNA = 1: the source is a raw conv output (fp32, SA = 0) whose GroupNorm(1, C) + GELU is applied
// while the halo is staged (P.gn_*: the producing conv's (sum, sum of squares) partials of each
// sample, gamma, beta) — the ResBlock's mid norm_kernel launch and its hi / lo planes disappear.
// GNA = 2: GELU(P.gn_res + GroupNorm(source)) — the output of a residual ResBlock (models/
// unet_cond.py:25-26) consumed by the next ResBlock's conv1, its final norm_kernel folded in here.
// Statistics are reduced exactly as norm_kernel reduces them and the affine (+ residual) + GELU is
// the same expression, so the staged operand is bit-identical to what norm_kernel would write.
template <int BN, int EPI, int SA, int X1, int W, int GNA = 0, int NWN = 2, int NWM = 4>
__global__ __launch_bounds__(64 * NWM * NWN) void igemm_halo_kernel(const X3Params P) {
  constexpr int NTH = 64 * NWM * NWN;              // threads: NWM (rows) x NWN (columns) waves
  const IgemmParams& p = P.g;
  constexpr bool MS = W <= 8;                      // multi-sample tiles (H == W), stacked halos
  constexpr int TR = 256 / W;                      // output image rows per tile (MS: over the samples)
  constexpr int SPT = MS ? 256 / (W * W) : 1;      // samples per tile
  constexpr int HWD = MS ? W + 1 : W + 2;          // halo row pitch
  constexpr int HP = MS ? (1 + SPT * (W + 1)) * HWD + 1 : (TR + 2) * HWD;  // halo pixels
  constexpr int CK = 32, RS = CK + 8;              // channels per chunk, f16 per LDS row
  static_assert(!MS || (W == 4 || W == 8), "multi-sample halo tiles: W = 4 or 8");
  static_assert(!(MS && GNA), "GroupNorm-on-load needs whole-row tiles of one sample");
  static_assert(EPI == EPI_STATS || EPI == EPI_PARTIAL, "halo epilogues");
  constexpr int WM = 256 / NWM, WN = BN / NWN, TM = WM / 32, TN = WN / 32;
  constexpr int PW = SA ? 8 : 4;                   // channels per staged A piece (16 bytes)
  constexpr int PPR = CK / PW;                     // pieces per halo pixel per plane
  constexpr int NPI = (HP * PPR + NTH - 1) / NTH;  // halo pieces per thread
  constexpr int BCH = BN * (CK / 8);               // B chunks (16 bytes) per plane per step
  static_assert(TM >= 1 && TN >= 1 && BCH <= NTH, "tile");

  constexpr int LA = X1 ? 1 : HP, LB = X1 ? 1 : BN;
  __shared__ __attribute__((aligned(16))) _Float16 Ah[2][HP][RS];
  __shared__ __attribute__((aligned(16))) _Float16 Al[2][LA][RS];
  __shared__ __attribute__((aligned(16))) _Float16 Bhs[2][BN][RS];
  __shared__ __attribute__((aligned(16))) _Float16 Bls[2][LB][RS];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / NWN, wn = wid % NWN;
  int mt, nt, bz;
  xcd_tile(mt, nt, bz);
  const int m0 = mt * 256, n0 = nt * BN;
  const int HW = p.H * W;
  const int C = p.src.C;
  const int nsmp = m0 / HW, y0 = (m0 - nsmp * HW) / W;  // tile = rows y0 .. y0 + TR - 1 of sample nsmp
  constexpr int AES = SA ? 2 : 4;
  // channel chunks of this block: all of them, or split bz's range (EPI_PARTIAL)
  const int nch_all = C / CK;
  const int cbeg = EPI == EPI_PARTIAL ? bz * p.ksplit : 0;
  const int nch = EPI == EPI_PARTIAL ? min(p.ksplit, nch_all - cbeg) : nch_all;

  // halo pieces of this thread: element offset of channel 0 of the piece (chunk 0), or -1 (zero)
  int hoff[NPI];
  short hpix[NPI], hq[NPI];
#pragma unroll
  for (int i = 0; i < NPI; ++i) {
    const int e = tid + NTH * i;
    const int h = e / PPR, q = e - h * PPR;
    hpix[i] = (short)h;
    hq[i] = (short)q;
    const int hy = h / HWD, hx = h - hy * HWD;
    bool ok;
    int pix;
    if constexpr (MS) {  // halo row hy = 1 + s (W + 1) + y (y = W: the zero row after sample s)
      const int s = (hy - 1) / (W + 1), y = hy - 1 - s * (W + 1), x = hx - 1;
      ok = e < HP * PPR && hy >= 1 && hy < 1 + SPT * (W + 1) && y < W && x >= 0 && nsmp + s < p.M / HW;
      pix = ((nsmp + s) * W + y) * W + x;
    } else {
      const int y = y0 + hy - 1, x = hx - 1;
      ok = e < HP * PPR && y >= 0 && y < p.H && x >= 0 && x < W;
      pix = (nsmp * p.H + y) * W + x;
    }
    hoff[i] = ok ? (pix * C + (cbeg * CK + q * PW)) : -1;
  }
  const __amdgpu_buffer_rsrc_t rAh = rsrc_of(SA ? (const void*)P.Ash : (const void*)p.src.src0, P.a_bytes);
  const __amdgpu_buffer_rsrc_t rAl = rsrc_of(SA ? (const void*)P.Asl : (const void*)p.src.src0, P.a_bytes);
  const __amdgpu_buffer_rsrc_t rBh = rsrc_of(P.Bh, P.b_bytes), rBl = rsrc_of(P.Bl, P.b_bytes);
  const bool bact = tid < BCH;
  const int brow = tid / (CK / 8), bq = tid - brow * (CK / 8);
  const int boffs = ((n0 + brow) * p.Kpad + bq * 8) * 2;

  static_assert(!GNA || !SA, "GroupNorm-on-load reads the fp32 raw source");
  // GroupNorm(1, C) statistics of sample nsmp, reduced as norm_kernel does (threads 0..255 sum
  // strided partials in double, wave shuffle tree, ((w0 + w1) + (w2 + w3)))
  float2 gst = make_float2(0.f, 0.f);
  if constexpr (GNA) {
    __shared__ double gr1[4], gr2[4];
    __shared__ float2 gst_s;
    if (tid < 256) {
      const float2* rp = P.gn_rowpart + (size_t)nsmp * P.gn_cnt;
      double s1 = 0.0, s2 = 0.0;
      for (int i = tid; i < P.gn_cnt; i += 256) {
        const float2 q = rp[i];
        s1 += (double)q.x;
        s2 += (double)q.y;
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        s1 += __shfl_xor(s1, o, 64);
        s2 += __shfl_xor(s2, o, 64);
      }
      if ((tid & 63) == 0) {
        gr1[tid >> 6] = s1;
        gr2[tid >> 6] = s2;
      }
    }
    __syncthreads();
    if (tid == 0) {
      const double cntd = (double)HW * (double)C;
      const double mean = ((gr1[0] + gr1[1]) + (gr1[2] + gr1[3])) / cntd;
      double var = ((gr2[0] + gr2[1]) + (gr2[2] + gr2[3])) / cntd - mean * mean;
      var = var < 0.0 ? 0.0 : var;
      gst_s = make_float2((float)mean, (float)(1.0 / sqrt(var + 1e-5)));
    }
    __syncthreads();
    gst = gst_s;
  }
  // register stages (B: two sets, a step's slice is loaded two steps before it is read)
  floatx4 ha4[SA ? 1 : NPI];
  floatx4 hr4[GNA == 2 ? NPI : 1];  // residual pieces (GNA = 2)
  half8 hah[SA ? NPI : 1], hal[SA ? NPI : 1];
  const __amdgpu_buffer_rsrc_t rRes = rsrc_of(GNA == 2 ? (const void*)P.gn_res : (const void*)p.src.src0, P.a_bytes);
  half8 rbh[2], rbl[2];
  // GNA: every piece of this thread has the same 4 channels of a chunk (NTH is a multiple of PPR), so
  // the GroupNorm affine of the chunk is 2 float4, loaded with the chunk's halo (not at store time)
  // (not for GNA = 2 at BN = 128: its 8 extra registers would spill at the 128-VGPR cap)
  static_assert(NTH % PPR == 0, "piece channel");
  constexpr bool GPRE = GNA == 1 || (GNA == 2 && BN == 64);
  floatx4 ggam = {0.f, 0.f, 0.f, 0.f}, gbet = {0.f, 0.f, 0.f, 0.f};
  auto load_halo = [&](int c) {
    if constexpr (GPRE) {
      const int ch = (cbeg + c) * CK + (tid % PPR) * PW;
      ggam = ld4(P.gn_gamma + ch);
      gbet = ld4(P.gn_beta + ch);
    }
#pragma unroll
    for (int i = 0; i < NPI; ++i) {
      const int off = hoff[i] >= 0 ? (hoff[i] + c * CK) * AES : kOOB;
      if constexpr (SA) {
        hah[i] = bload_h8(rAh, off, 0);
        if constexpr (!X1) hal[i] = bload_h8(rAl, off, 0);
      } else {
        ha4[i] = bload_f4(rAh, off, 0);
        if constexpr (GNA == 2) hr4[i] = bload_f4(rRes, off, 0);
      }
    }
  };
  // pieces [i0, i1) of the staged halo to LDS buffer `buf` (chunk cc)
  auto store_halo = [&](int buf, int cc, int i0, int i1) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NPI; ++i) {
      if (i < i0 || i >= i1) continue;
      if (tid + NTH * i >= HP * PPR) continue;  // only the last piece index can be partial
      const int h = hpix[i], q = hq[i];
      if constexpr (SA) {
        *reinterpret_cast<half8*>(&Ah[buf][h][q * 8]) = hah[i];
        if constexpr (!X1) *reinterpret_cast<half8*>(&Al[buf][h][q * 8]) = hal[i];
      } else {
        floatx4 v = ha4[i];
        if constexpr (GNA) {  // GroupNorm (+ residual) + GELU of the raw source; zero padding stays zero
          if constexpr (GPRE) {
            v = gn_apply4v(v, gst, ggam, gbet, GNA == 1 ? 1 : 0);
          } else {
            const int ch = (cbeg + cc) * CK + q * 4;
            v = gn_apply4v(v, gst, ld4(P.gn_gamma + ch), ld4(P.gn_beta + ch), GNA == 1 ? 1 : 0);
          }
          if constexpr (GNA == 2) {
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = gelu(hr4[i][j] + v[j]);
          }
          if (hoff[i] < 0) v = floatx4{0.f, 0.f, 0.f, 0.f};
        }
        if constexpr (X1) {
          *reinterpret_cast<half4*>(&Ah[buf][h][q * 4]) = __builtin_convertvector(v, half4);
        } else {
          half4 hh, ll;
          split4(v, hh, ll);
          *reinterpret_cast<half4*>(&Ah[buf][h][q * 4]) = hh;
          *reinterpret_cast<half4*>(&Al[buf][h][q * 4]) = ll;
        }
      }
    }
  };
  // B slice of step s = 9 c + t (c: chunk of this block): k = t * C + (cbeg + c) * CK .. + CK of the
  // [Npad][Kpad] planes
  auto load_b = [&](int s, int set) {
    if (bact) {
      const int c = s / 9, t = s - 9 * c;
      const int soff = (t * C + (cbeg + c) * CK) * 2;
      rbh[set] = bload_h8(rBh, boffs, soff);
      if constexpr (!X1) rbl[set] = bload_h8(rBl, boffs, soff);
    }
  };
  auto store_b = [&](int buf, int set) {
    if (bact) {
      *reinterpret_cast<half8*>(&Bhs[buf][brow][bq * 8]) = rbh[set];
      if constexpr (!X1) *reinterpret_cast<half8*>(&Bls[buf][brow][bq * 8]) = rbl[set];
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
  // halo pixel of each A fragment row for tap (0, 0): output pixel r = wm*64 + i*32 + fp of the
  // tile.  W = 16: a fragment spans two image rows, whose halo rows lie 18 LDS rows apart; lanes
  // 16..31 take the second row rotated by two pixels (fp = 16 + ((fr - 18) & 15)) so that every
  // 16-lane group of ds_read_b128 (lanes {0-3,12-15,20-27}, {4-11,16-19,28-31}) reads 16 LDS rows
  // distinct mod 16 — distinct 16-byte slots of the 80-byte-row layout, no bank conflict.  The
  // epilogue writes accumulator rows back through the same rotation (igemm_epilogue RPERM).
  constexpr int RPERM = W == 16 ? 1 : 0;
  const int fp = (RPERM && fr >= 16) ? 16 + ((fr - 18) & 15) : fr;
  int abase[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int r = wm * WM + i * 32 + fp;
    if constexpr (MS) {  // tile pixel r = sample r / W², row ly, column lx
      const int s = r / (W * W), ly = (r - s * W * W) / W, lx = r % W;
      abase[i] = (1 + s * (W + 1) + ly) * HWD + lx + 1;
    } else {
      const int ly = r / W, lx = r - ly * W;
      abase[i] = (ly + 1) * HWD + lx + 1;
    }
  }
  auto compute = [&](int abuf, int bbuf, int tap) {
    const int ty = (tap * 11) >> 5;  // tap / 3 for tap in [0, 8]
    const int delta = (ty - 1) * HWD + (tap - 3 * ty - 1);
    constexpr int S = CK / 16, NR = (X1 ? 1 : 2) * (TM + TN), NM = (X1 ? 1 : 3) * TM * TN;
    half8 ah[2][TM], al[2][TM], bh[2][TN], bl[2][TN];
    auto ldf = [&](int s, int d) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = abase[i] + delta;
        ah[d][i] = *reinterpret_cast<const half8*>(&Ah[abuf][row][16 * s + 8 * fh]);
        if constexpr (!X1) al[d][i] = *reinterpret_cast<const half8*>(&Al[abuf][row][16 * s + 8 * fh]);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * WN + j * 32 + fr;
        bh[d][j] = *reinterpret_cast<const half8*>(&Bhs[bbuf][row][16 * s + 8 * fh]);
        if constexpr (!X1) bl[d][j] = *reinterpret_cast<const half8*>(&Bls[bbuf][row][16 * s + 8 * fh]);
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

  const int S = nch * 9;
  // The B slice of step s is loaded at the start of step s - 2 (register set s & 1) and written to
  // LDS after the MFMAs of step s - 1; the next chunk's halo is loaded at tap 0 and written after
  // tap HST — the global loads get two (B) / HST + 1 (halo) steps of MFMAs to land.
  // The halo is written in NRD rounds at taps HST .. HST + NRD - 1 (PRD pieces each), which spreads
  // the GroupNorm + GELU VALU work of GNA over several steps' MFMAs.
  constexpr int HST = 4, NRD = 4, PRD = (NPI + NRD - 1) / NRD;
  // prologue: chunk 0's halo and step 0's B slice in LDS, step 1's B slice in flight
  load_b(0, 0);
  load_halo(0);
  store_b(0, 0);
  store_halo(0, 0, 0, NPI);
  if (S > 1) load_b(1, 1);
  __syncthreads();
  auto step = [&](int s, int set) {  // set = (s + 1) & 1: holds B(s + 1); B(s + 2) goes to the other
    const int c = s / 9, t = s - 9 * c;
    if (s + 2 < S) load_b(s + 2, set ^ 1);
    if (t == 0 && c + 1 < nch) load_halo(c + 1);
    compute(c & 1, s & 1, t);
    if (t >= HST && t < HST + NRD && c + 1 < nch) store_halo((c + 1) & 1, c + 1, (t - HST) * PRD, (t - HST + 1) * PRD);
    if (s + 1 < S) store_b((s + 1) & 1, set);
    __syncthreads();
  };
  for (int s = 0; s < S; s += 2) {
    step(s, 1);
    if (s + 1 < S) step(s + 1, 0);
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] *= P.inv_scale;

  // rows of wave (wm, wn): m0 + wm * 64 + ...; the shared epilogue's 2 x 2 wave grid over 128 rows
  igemm_epilogue<2 * WM, 2 * WN, EPI, RPERM>(p, acc, 0, m0 + (wm >> 1) * 2 * WM, n0 + (wn >> 1) * 2 * WN, wm & 1,
                                             wn & 1, fr, fh);
}


// ---------------------------------------------------------------------------
// Low-resolution halo conv, chunk-staged (W = 8 / 4, BN = 64, 16 waves of 32 x 32).  The 4 x 4 and
// 8 x 8 convs give a block only one to four 32-channel chunks (split-K), i.e. 9 - 36 (chunk, tap)
// steps whose MFMAs (6 per wave) are far shorter than a global-load round trip: with one barrier and
// a two-step-ahead B load per tap (igemm_halo_kernel) the launch is a chain of load latencies.  Here
// the B slice of ALL nine taps of a chunk (9 x 64 x 32 f16 per plane, 92 KB for both) sits in LDS
// beside the chunk's stacked halo (one buffer each): a chunk is one global round trip, issued while
// the previous chunk's 54 MFMAs per wave run, then barrier, LDS store, barrier.  Same K order (chunk,
// tap, k16) and MFMA order as igemm_halo_kernel, so the sums are bit-identical to it.
// ---------------------------------------------------------------------------
template <int EPI, int SA, int X1, int W>
__global__ __launch_bounds__(1024) void igemm_halo_cs_kernel(const X3Params P) {
  constexpr int BN = 64, NTH = 1024;
  constexpr int SPT = 256 / (W * W), HWD = W + 1, HP = (1 + SPT * (W + 1)) * HWD + 1;
  constexpr int CK = 32, RS = CK + 8;
  constexpr int PW = SA ? 8 : 4, PPR = CK / PW, NPI = (HP * PPR + NTH - 1) / NTH;
  constexpr int BPT = BN * (CK / 8);              // 16-byte B pieces per plane per tap
  constexpr int NPB = (9 * BPT + NTH - 1) / NTH;  // B pieces per thread per plane per chunk
  constexpr int AES = SA ? 2 : 4;
  static_assert(W == 4 || W == 8, "low-resolution maps only");
  static_assert(EPI == EPI_STATS || EPI == EPI_PARTIAL, "halo epilogues");
  constexpr int LA = X1 ? 1 : HP, LB = X1 ? 1 : 9 * BN;
  __shared__ __attribute__((aligned(16))) _Float16 Ah[HP][RS];
  __shared__ __attribute__((aligned(16))) _Float16 Al[LA][RS];
  __shared__ __attribute__((aligned(16))) _Float16 Bhs[9 * BN][RS];
  __shared__ __attribute__((aligned(16))) _Float16 Bls[LB][RS];

  const IgemmParams& p = P.g;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  int mt, nt, bz;
  xcd_tile(mt, nt, bz);
  const int m0 = mt * 256, n0 = nt * BN;
  const int HW = W * W, C = p.src.C;
  const int nsmp = m0 / HW, nsamp = p.M / HW;
  const int nch_all = C / CK;
  const int cbeg = EPI == EPI_PARTIAL ? bz * p.ksplit : 0;
  const int nch = EPI == EPI_PARTIAL ? min(p.ksplit, nch_all - cbeg) : nch_all;

  // halo pieces (stacked samples, as igemm_halo_kernel MS): element offset of the piece's first
  // channel in chunk 0 of this block, or -1 (zero)
  int hoff[NPI];
  short hpix[NPI], hq[NPI];
#pragma unroll
  for (int i = 0; i < NPI; ++i) {
    const int e = tid + NTH * i;
    const int h = e / PPR, q = e - h * PPR;
    hpix[i] = (short)h;
    hq[i] = (short)q;
    const int hy = h / HWD, hx = h - hy * HWD;
    const int s = (hy - 1) / (W + 1), y = hy - 1 - s * (W + 1), x = hx - 1;
    const bool ok = e < HP * PPR && hy >= 1 && hy < 1 + SPT * (W + 1) && y < W && x >= 0 && nsmp + s < nsamp;
    hoff[i] = ok ? ((((nsmp + s) * W + y) * W + x) * C + cbeg * CK + q * PW) : -1;
  }
  // B pieces: e -> tap t = e / BPT, column row (e % BPT) / 4, 8-channel quarter e % 4
  int boff[NPB];
  short bsl[NPB];  // LDS row t * BN + row (quarter in the low 2 bits), -1: none
#pragma unroll
  for (int i = 0; i < NPB; ++i) {
    const int e = tid + NTH * i;
    const int t = e / BPT, r = e - t * BPT, row = r >> 2, q = r & 3;
    const bool ok = e < 9 * BPT;
    boff[i] = ok ? ((n0 + row) * p.Kpad + t * C + cbeg * CK + q * 8) * 2 : kOOB;
    bsl[i] = ok ? (short)(((t * BN + row) << 2) | q) : (short)-1;
  }
  const __amdgpu_buffer_rsrc_t rAh = rsrc_of(SA ? (const void*)P.Ash : (const void*)p.src.src0, P.a_bytes);
  const __amdgpu_buffer_rsrc_t rAl = rsrc_of(SA ? (const void*)P.Asl : (const void*)p.src.src0, P.a_bytes);
  const __amdgpu_buffer_rsrc_t rBh = rsrc_of(P.Bh, P.b_bytes), rBl = rsrc_of(P.Bl, P.b_bytes);

  floatx4 ha4[SA ? 1 : NPI];
  half8 hah[SA ? NPI : 1], hal[SA ? NPI : 1];
  half8 rbh[NPB], rbl[NPB];
  auto load_chunk = [&](int c) {  // c: chunk of this block
#pragma unroll
    for (int i = 0; i < NPB; ++i) {
      rbh[i] = bload_h8(rBh, boff[i], c * CK * 2);
      if constexpr (!X1) rbl[i] = bload_h8(rBl, boff[i], c * CK * 2);
    }
#pragma unroll
    for (int i = 0; i < NPI; ++i) {
      const int off = hoff[i] >= 0 ? (hoff[i] + c * CK) * AES : kOOB;
      if constexpr (SA) {
        hah[i] = bload_h8(rAh, off, 0);
        if constexpr (!X1) hal[i] = bload_h8(rAl, off, 0);
      } else {
        ha4[i] = bload_f4(rAh, off, 0);
      }
    }
  };
  auto store_chunk = [&]() {
#pragma unroll
    for (int i = 0; i < NPB; ++i) {
      if (bsl[i] < 0) continue;
      const int row = bsl[i] >> 2, q = bsl[i] & 3;
      *reinterpret_cast<half8*>(&Bhs[row][q * 8]) = rbh[i];
      if constexpr (!X1) *reinterpret_cast<half8*>(&Bls[row][q * 8]) = rbl[i];
    }
#pragma unroll
    for (int i = 0; i < NPI; ++i) {
      if (tid + NTH * i >= HP * PPR) continue;
      const int h = hpix[i], q = hq[i];
      if constexpr (SA) {
        *reinterpret_cast<half8*>(&Ah[h][q * 8]) = hah[i];
        if constexpr (!X1) *reinterpret_cast<half8*>(&Al[h][q * 8]) = hal[i];
      } else if constexpr (X1) {
        *reinterpret_cast<half4*>(&Ah[h][q * 4]) = __builtin_convertvector(ha4[i], half4);
      } else {
        half4 hh, ll;
        split4(ha4[i], hh, ll);
        *reinterpret_cast<half4*>(&Ah[h][q * 4]) = hh;
        *reinterpret_cast<half4*>(&Al[h][q * 4]) = ll;
      }
    }
  };

  const int fr = lane & 31, fh = lane >> 5;
  int abase;
  {
    const int r = wm * 32 + fr;  // tile pixel of this lane's fragment row
    const int s = r / HW, ly = (r - s * HW) / W, lx = r % W;
    abase = (1 + s * (W + 1) + ly) * HWD + lx + 1;
  }
  const int bcol = wn * 32 + fr;
  floatx16 acc[1][1];
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[0][0][r] = 0.f;
  // 18 k16 steps per chunk (tap kk / 2, half kk % 2), fragments read one step ahead
  half8 fa[2], fal[2], fb[2], fbl[2];
  auto ldf = [&](int kk, int d) {
    const int t = kk >> 1, s = kk & 1;
    const int ty = (t * 11) >> 5;  // t / 3
    const int row = abase + (ty - 1) * HWD + (t - 3 * ty - 1);
    fa[d] = *reinterpret_cast<const half8*>(&Ah[row][16 * s + 8 * fh]);
    if constexpr (!X1) fal[d] = *reinterpret_cast<const half8*>(&Al[row][16 * s + 8 * fh]);
    fb[d] = *reinterpret_cast<const half8*>(&Bhs[t * BN + bcol][16 * s + 8 * fh]);
    if constexpr (!X1) fbl[d] = *reinterpret_cast<const half8*>(&Bls[t * BN + bcol][16 * s + 8 * fh]);
  };
  constexpr int NR = X1 ? 2 : 4, NM = X1 ? 1 : 3;
  auto compute_chunk = [&]() {
    ldf(0, 0);
#pragma unroll
    for (int kk = 0; kk < 18; ++kk) {
      const int d = kk & 1;
      if (kk + 1 < 18) ldf(kk + 1, d ^ 1);
      if constexpr (!X1) {
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fal[d], fb[d], acc[0][0], 0, 0, 0);
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[d], fbl[d], acc[0][0], 0, 0, 0);
      }
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[d], fb[d], acc[0][0], 0, 0, 0);
      if (kk + 1 < 18) {
        __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, NM, 0);
      }
    }
  };

  load_chunk(0);
  store_chunk();
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    if (c + 1 < nch) load_chunk(c + 1);  // in flight under this chunk's MFMAs
    compute_chunk();
    if (c + 1 < nch) {
      __syncthreads();  // every wave done reading chunk c
      store_chunk();
      __syncthreads();
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[0][0][r] *= P.inv_scale;
  igemm_epilogue<64, 64, EPI>(p, acc, 0, m0 + (wm >> 1) * 64, n0, wm & 1, wn, fr, fh);
}

// The split weight planes ([Npad][Kpad] f16) re-laid out in MFMA-fragment order: the B operand of
// v_mfma_f32_32x32x16_f16 for columns 32*nb .. +31 and k = 16*kk .. +15 is 64 lanes x 8 f16, lane
// (fr, fh) holding column 32*nb + fr, k = 16*kk + 8*fh .. +7 — stored as 1 KB contiguous at
// ((nb * Kpad/16 + kk) * 64 + lane) * 8, so a wave loads a fragment with one coalesced 16-byte-per-
// lane load.  Replayed after every plane refresh (engine.hip split_planes).
static __global__ void frag_planes_kernel(const _Float16* bh, const _Float16* bl, _Float16* fh, _Float16* fl,
                                          int npad, int kpad) {
  const size_t chunks = (size_t)npad * kpad / 8;
  const int kc8 = kpad / 8;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < chunks; i += (size_t)gridDim.x * blockDim.x) {
    const int n = (int)(i / kc8), kc = (int)(i - (size_t)n * kc8);
    const int nb = n >> 5, fr = n & 31, kk = kc >> 1, hh = kc & 1;
    const size_t dst = ((size_t)(nb * (kpad / 16) + kk) * 64 + hh * 32 + fr) * 8;
    *reinterpret_cast<half8*>(fh + dst) = *reinterpret_cast<const half8*>(bh + i * 8);
    *reinterpret_cast<half8*>(fl + dst) = *reinterpret_cast<const half8*>(bl + i * 8);
  }
}

// ---------------------------------------------------------------------------
// Halo conv with B read straight into registers ("B-direct").  The A halo is staged as above;
// every wave loads its own B fragments for the NEXT (chunk, tap) step from the fragment-ordered
// planes (P.Fh / P.Fl: one coalesced 1 KB load per fragment, L2-resident weights; the four waves
// of a column group read the same bytes, mostly L1 hits) while the current step's MFMAs run, so
// B never touches LDS and the only barrier is the one per 32-channel chunk (halo buffer swap):
// MFMAs flow across the nine taps of a chunk.  A fragments are read one k16 step ahead, across
// tap boundaries too.  Same K order as igemm_halo_kernel.
// ---------------------------------------------------------------------------
template <int BN, int EPI, int SA, int X1, int W>
__global__ __launch_bounds__(512) void igemm_halo_bd_kernel(const X3Params P) {
  const IgemmParams& p = P.g;
  constexpr int TR = 256 / W;
  constexpr int HWD = W + 2, HP = (TR + 2) * HWD;
  constexpr int CK = 32, RS = CK + 8;
  constexpr int WN = BN / 2, TM = 2, TN = WN / 32;
  constexpr int PW = SA ? 8 : 4;
  constexpr int PPR = CK / PW;
  constexpr int NPI = (HP * PPR + 511) / 512;
  constexpr int NP = X1 ? 1 : 2;  // B planes
  static_assert(TN >= 1, "tile");

  constexpr int LA = X1 ? 1 : HP;
  __shared__ __attribute__((aligned(16))) _Float16 Ah[2][HP][RS];
  __shared__ __attribute__((aligned(16))) _Float16 Al[2][LA][RS];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  int mt, nt, bz;
  xcd_tile(mt, nt, bz);
  const int m0 = mt * 256, n0 = nt * BN;
  const int HW = p.H * W;
  const int C = p.src.C;
  const int nsmp = m0 / HW, y0 = (m0 - nsmp * HW) / W;
  constexpr int AES = SA ? 2 : 4;

  // halo pieces of this thread (index e = tid + 512 i): element offset of channel 0 (chunk 0) or -1
  int hoff[NPI];
#pragma unroll
  for (int i = 0; i < NPI; ++i) {
    const int e = tid + 512 * i;
    const int h = e / PPR, q = e - h * PPR;
    const int hy = h / HWD, hx = h - hy * HWD;
    const int y = y0 + hy - 1, x = hx - 1;
    const bool ok = e < HP * PPR && y >= 0 && y < p.H && x >= 0 && x < W;
    hoff[i] = ok ? (((nsmp * p.H + y) * W + x) * C + q * PW) : -1;
  }
  const __amdgpu_buffer_rsrc_t rAh = rsrc_of(SA ? (const void*)P.Ash : (const void*)p.src.src0, P.a_bytes);
  const __amdgpu_buffer_rsrc_t rAl = rsrc_of(SA ? (const void*)P.Asl : (const void*)p.src.src0, P.a_bytes);
  const __amdgpu_buffer_rsrc_t rFh = rsrc_of(P.Fh, P.b_bytes), rFl = rsrc_of(P.Fl, P.b_bytes);

  // The next chunk's halo is staged in HR rounds of PR pieces per thread (round r: loaded at tap 2r,
  // written at tap 2r + 1) so only PR pieces are held in registers at a time.
  constexpr int HR = 4, PR = (NPI + HR - 1) / HR;
  floatx4 ha4[SA ? 1 : PR];
  half8 hah[SA ? PR : 1], hal[SA ? PR : 1];
  auto load_halo = [&](int c, int r) {
#pragma unroll
    for (int k = 0; k < PR; ++k) {
      const int i = r * PR + k;
      if (i >= NPI) break;
      const int off = hoff[i] >= 0 ? (hoff[i] + c * CK) * AES : kOOB;
      if constexpr (SA) {
        hah[k] = bload_h8(rAh, off, 0);
        if constexpr (!X1) hal[k] = bload_h8(rAl, off, 0);
      } else {
        ha4[k] = bload_f4(rAh, off, 0);
      }
    }
  };
  auto store_halo = [&](int buf, int r) {
#pragma unroll
    for (int k = 0; k < PR; ++k) {
      const int i = r * PR + k;
      if (i >= NPI) break;
      const int e = tid + 512 * i;
      if (e >= HP * PPR) continue;
      const int h = e / PPR, q = e - h * PPR;
      if constexpr (SA) {
        *reinterpret_cast<half8*>(&Ah[buf][h][q * 8]) = hah[k];
        if constexpr (!X1) *reinterpret_cast<half8*>(&Al[buf][h][q * 8]) = hal[k];
      } else if constexpr (X1) {
        *reinterpret_cast<half4*>(&Ah[buf][h][q * 4]) = __builtin_convertvector(ha4[k], half4);
      } else {
        half4 hh, ll;
        split4(ha4[k], hh, ll);
        *reinterpret_cast<half4*>(&Ah[buf][h][q * 4]) = hh;
        *reinterpret_cast<half4*>(&Al[buf][h][q * 4]) = ll;
      }
    }
  };
  // B fragments of one step: [column tile j][k16 step s][plane]
  struct BF {
    half8 v[TN][2][NP];
  };
  const int kk16 = p.Kpad / 16;
  const int voff = lane * 16;
  auto load_bf = [&](int c, int t, BF& b) {
    const int kk = (t * C + c * CK) / 16;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int nb = (n0 + wn * WN + j * 32) >> 5;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int soff = (nb * kk16 + kk + s) * 1024;
        b.v[j][s][0] = bload_h8(rFh, voff, soff);
        if constexpr (!X1) b.v[j][s][1] = bload_h8(rFl, voff, soff);
      }
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
  int abase[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int r = wm * 64 + i * 32 + fr;
    const int ly = r / W, lx = r - ly * W;
    abase[i] = (ly + 1) * HWD + lx + 1;
  }
  auto tap_delta = [&](int tap) {
    const int ty = (tap * 11) >> 5;
    return (ty - 1) * HWD + (tap - 3 * ty - 1);
  };
  // A fragments, two k16 slots
  half8 ah[2][TM], al[2][TM];
  auto lda = [&](int abuf, int tap, int s, int d) {
    const int delta = tap_delta(tap);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = abase[i] + delta;
      ah[d][i] = *reinterpret_cast<const half8*>(&Ah[abuf][row][16 * s + 8 * fh]);
      if constexpr (!X1) al[d][i] = *reinterpret_cast<const half8*>(&Al[abuf][row][16 * s + 8 * fh]);
    }
  };
  auto mfmas = [&](int d, const BF& b, int s) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (!X1) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[d][i], b.v[j][s][0], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[d][i], b.v[j][s][1], acc[i][j], 0, 0, 0);
        }
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[d][i], b.v[j][s][0], acc[i][j], 0, 0, 0);
      }
  };
  constexpr int NRA = (X1 ? 1 : 2) * TM, NM = (X1 ? 1 : 3) * TM * TN;

  const int nch = C / CK;
  const int S = nch * 9;
  BF b0, b1;
  load_bf(0, 0, b0);
#pragma unroll
  for (int r = 0; r < HR; ++r) {
    load_halo(0, r);
    store_halo(0, r);
  }
  __syncthreads();
  lda(0, 0, 0, 0);
  // one (chunk, tap) step: MFMAs from A buffer c & 1 and `cur`; loads the next step's B into `nxt`
  auto step = [&](int s, BF& cur, BF& nxt) {
    const int c = s / 9, t = s - c * 9;
    const int abuf = c & 1;
    if (s + 1 < S) load_bf(t == 8 ? c + 1 : c, t == 8 ? 0 : t + 1, nxt);
    if ((t & 1) == 0 && t < 2 * HR && c + 1 < nch) load_halo(c + 1, t >> 1);
    lda(abuf, t, 1, 1);  // k16 step 1 of this tap, under step 0's MFMAs
    mfmas(0, cur, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
#pragma unroll
    for (int r = 0; r < NRA; ++r) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, NM - NRA - 1, 0);
    if (t < 8) {
      lda(abuf, t + 1, 0, 0);  // next tap's k16 step 0, under step 1's MFMAs
      mfmas(1, cur, 1);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
#pragma unroll
      for (int r = 0; r < NRA; ++r) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, NM - NRA - 1, 0);
    } else {
      mfmas(1, cur, 1);
    }
    if ((t & 1) == 1 && t < 2 * HR && c + 1 < nch) store_halo((c + 1) & 1, t >> 1);
    if (t == 8 && s + 1 < S) {
      __syncthreads();  // chunk c + 1's halo complete in buffer (c + 1) & 1; buffer c & 1 free
      lda((c + 1) & 1, 0, 0, 0);
    }
  };
  for (int s = 0; s < S; s += 2) {
    step(s, b0, b1);
    if (s + 1 < S) step(s + 1, b1, b0);
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] *= P.inv_scale;

  igemm_epilogue<128, BN, EPI>(p, acc, 0, m0 + (wm >> 1) * 128, n0, wm & 1, wn, fr, fh);
}

}  // namespace dmx
