// dmx — split-precision 3x3 convolution as Winograd F(2x2, 3x3) on the f16 matrix cores, gfx950.
//
// Reference op: nn.Conv2d(k=3, padding=1, bias=False) of every ResBlock (models/unet_cond.py:17-23).
//
// A 3x3 / pad-1 convolution of a 2x2 output tile is Y = Aᵀ [ (G g Gᵀ) ⊙ (Bᵀ d B) ] A with d the 4x4
// input patch of the tile (zero outside the image) and the 4x4 "positions" xi = (i, j):
//   Bᵀ = [[1, 0,-1, 0], [0, 1, 1, 0], [0,-1, 1, 0], [0, 1, 0,-1]],  G = [[1,0,0], [½,½,½], [½,-½,½], [0,0,1]],
//   Aᵀ = [[1, 1, 1, 0], [0, 1,-1,-1]].
// Summed over input channels, each position is an independent GEMM
//   M_xi[tile, cout] = sum_cin V_xi[tile, cin] * U_xi[cin, cout],   V = Bᵀ d B,  U = G g Gᵀ,
// i.e. 16 multiply-adds per 4 output pixels instead of 36: 2.25x fewer MFMAs than the direct conv.
// Precision is the direct kernels' (igemm_x3.h): V is formed in fp32 (sums / differences of input
// values, one rounding each), U in double on the device at load time (wino_pack_kernel), both split
// into f16 hi + lo and multiplied as al*bh + ah*bl + ah*bh with fp32 accumulation; the output
// transform runs in fp32.  Every constant of B, G, A is ±1 or ½, so no transform step amplifies
// rounding beyond the sums themselves (F(2x2,3x3) is the well-conditioned member of the family).
//
// Block: 512 threads = 8 waves, 64 tiles (256 output pixels = whole image rows of one sample at
// W = 32 / one whole sample at W = 16) x 64 output channels, all 16 positions.  Wave w owns the two
// positions (i, 2jp) and (i, 2jp + 1), i = w / 2, jp = w % 2: accumulators 2 positions x 2 (32-tile)
// x 2 (32-channel) MFMA tiles = 128 VGPRs.  K walks 16-channel chunks (one k16 MFMA step):
//   * the chunk's input halo ((rows + 2) x (W + 2) pixels x 16 channels, fp32, GroupNorm (+ residual)
//     + GELU applied for GNA = 1 / 2 exactly as igemm_halo_kernel does) is staged once in LDS, with
//     even and odd columns in separate planes so the 2-pixel tile stride becomes a 1-pixel stride
//     (conflict-free ds_read_b128 with the row pitches below);
//   * each wave forms ITS OWN A fragments V_(i,j)[tile, 8 channels] straight from the halo: two input
//     rows (Bᵀ row i) x three input columns (B columns j) — 5 fma per channel for both positions,
//     then the hi / lo split;
//   * B (U) fragments come straight from the fragment-ordered planes into registers (1 KB coalesced
//     per fragment, L2-resident), each reloaded for the next chunk right after its last MFMA;
//   * one barrier per chunk (halo double buffer).
// X1 = 1 (config 4, BASELINE configs[3]): U hi and V rounded to f16 once, one MFMA per product
// (fp32 accumulate), transforms in fp32 as in the x3 instances.
// Epilogue: in four passes of (32 tiles x 32 channels) the 16 position accumulators go through LDS,
// every thread applies Aᵀ M A to two tiles of one channel in a fixed order, stores the 2x2 pixels
// (NHWC fp32) and the GroupNorm (sum, sum of squares) partials of 16-pixel x 32-channel groups
// (one partial row per 4 geometry tiles: the caller's consumers reduce a sample's partials in any layout).
// Maps narrower than the geometry (the reference's 28 x 28 latents: 28 / 14 / 7 / 3 maps in the 32 / 16
// / 8 / 4 geometries) run the same blocks with the missing columns and rows as zero padding.
#pragma once
#include "common.h"
#include "igemm.h"
#include "igemm_x3.h"
#include "source.h"

namespace dmx {

// Diagnostic builds only (-DDMX_DIAG=1, k_wino.hip's dmx_diag_wino_stamps reads them): wave 0 of
// every block records s_memtime at kernel start, after the prologue barrier, after the chunk loop
// and at the end, plus the hardware id (XCC, CU), into g_wstamp[launch slot][block] — timing only,
// no output value depends on them (MI355X_MICROARCH.md DVFS note 6).  (Round 5's timing
// decompositions — builds without MFMAs, transforms, stores, ... — are recorded in DESIGN §6d / §6e.)
#ifndef DMX_DIAG
#define DMX_DIAG 0
#endif
#if DMX_DIAG
constexpr int WSTAMP_SLOTS = 32, WSTAMP_BLOCKS = 2048;
__device__ unsigned long long g_wstamp[WSTAMP_SLOTS * WSTAMP_BLOCKS * 5];
DMX_DEV void wstamp(int slot, int k) {
  if (threadIdx.x == 0 && slot >= 0 && slot < WSTAMP_SLOTS) {
    const int b = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    if (b < WSTAMP_BLOCKS) {
      unsigned long long* q = g_wstamp + ((size_t)slot * WSTAMP_BLOCKS + b) * 5;
      q[k] = __builtin_amdgcn_s_memtime();
      if (k == 0) q[4] = ((unsigned long long)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11)) << 32) |
                         (unsigned)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
    }
  }
}
#define WSTAMP(k) wstamp(P.dslot, k)
#else
#define WSTAMP(k)
#endif

// U = G g Gᵀ of one 3x3 kernel for position (i, j), in double (exact products of ½-multiples).
DMX_DEV double wino_u(const double (&g)[3][3], int i, int j) {
  double r[3];  // (G g)[i][b]
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    const double a0 = g[0][b], a1 = g[1][b], a2 = g[2][b];
    r[b] = i == 0 ? a0 : i == 1 ? 0.5 * (a0 + a1 + a2) : i == 2 ? 0.5 * (a0 - a1 + a2) : a2;
  }
  return j == 0 ? r[0] : j == 1 ? 0.5 * (r[0] + r[1] + r[2]) : j == 2 ? 0.5 * (r[0] - r[1] + r[2]) : r[2];
}

// Weight transform + split into MFMA-fragment order: B operand of v_mfma_f32_32x32x16_f16 for
// position xi, output channels 32 nb .. +31, input channels 16 kk .. +15 is 64 lanes x 8 f16 (lane
// (fr, fh): channel 32 nb + fr, inputs 16 kk + 8 fh .. +7), stored 1 KB contiguous at
// ((xi * NB + nb) * KK + kk) * 512 halves.  B: packed fp32 [npad][kpad] (k = tap * cin + c).
static __global__ void wino_pack_kernel(const float* B, int kpad, int cin, int cout, float scale, _Float16* uh,
                                        _Float16* ul) {
  const int NB = cout / 32, KK = cin / 16;
  const size_t total = (size_t)16 * NB * KK * 64;
  for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += (size_t)gridDim.x * blockDim.x) {
    const int lane = (int)(q & 63);
    const size_t f = q >> 6;
    const int kk = (int)(f % KK), nb = (int)((f / KK) % NB), xi = (int)(f / ((size_t)KK * NB));
    const int co = 32 * nb + (lane & 31), c0 = 16 * kk + 8 * (lane >> 5);
    half8 h, l;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      double g[3][3];
#pragma unroll
      for (int t = 0; t < 9; ++t) g[t / 3][t % 3] = (double)B[(size_t)co * kpad + (size_t)t * cin + c0 + e];
      const float u = (float)(wino_u(g, xi >> 2, xi & 3) * (double)scale);
      const _Float16 hh = (_Float16)u;
      h[e] = hh;
      l[e] = (_Float16)(u - (float)hh);
    }
    *reinterpret_cast<half8*>(uh + q * 8) = h;
    *reinterpret_cast<half8*>(ul + q * 8) = l;
  }
}

// Geometry.  W = 32: a block is 8 output rows of one sample (4 tile rows x 16); W = 16: one whole
// sample (8 x 8 tiles); W = 8: four whole samples (4 x 4 tiles each), their halos stacked at a pitch
// of PS = 11 halo rows (the 11th row is padding); W = 4: sixteen whole samples.  Halo pixel (row, col)
// of stacked sample s lives at float offset s * SQ + (row * 2 + col % 2) * RP * 4 + (col / 2) * 20 + channel: even / odd columns in separate planes,
// 20 floats (16 channels + 4 pad) per pixel, RP 16-byte units per plane row.  A fragment row (tile)
// of lane fr then reads at (s * PS + 2 ty) * 8 RP + 5 tx units + const, and RP is chosen so that each
// 16-lane group of ds_read_b128 ({0-3,12-15,20-27}, {4-11,16-19,28-31}, +32) hits 16 distinct
// 16-byte bank slots: W = 32 (2 tile rows per 32 tiles) needs 4 RP = 0 mod 16 (RP = 88), W = 16
// (4 tile rows) 4 RP = 8 mod 16 (RP = 46), W = 8 (2 samples x 4 tile rows, PS = 11) 2 RP = 4 mod 16
// (RP = 26).  W = 4: sixteen whole samples (2 x 2 tiles each), 6 halo rows each; no whole-row pitch
// spreads the 16 lanes of a group over 16 slots there, so a stacked sample starts every SQ = 218
// units (> 12 RP = 216, RP = 18: 4 RP = 8 mod 16), which does.
// EPI = EPI_STATS: the conv output and its GroupNorm partials; EPI_PARTIAL (grid.z = K splits over
// 16-channel chunks, P.g.ksplit chunks each): the split's transformed partial output to slab z,
// reduced in split order by reduce_norm_kernel / splitk_reduce_kernel (the output transform is
// linear, so transforming each split's partial sums and adding the pixels equals transforming the
// total).
template <int W, int GNA, int EPI = EPI_STATS, int X1 = 0>
__global__ __launch_bounds__(512) void wino_kernel(const X3Params P) {
  static_assert(EPI == EPI_STATS || EPI == EPI_PARTIAL, "Winograd epilogues");
  static_assert(W == 32 || W == 16 || W == 8 || W == 4, "Winograd conv: image width 4, 8, 16 or 32");
  static_assert(W != 4 || GNA == 0, "W = 4: no GroupNorm-on-load instances");
  const IgemmParams& p = P.g;
  constexpr int TW = W / 2;                       // tiles per tile row
  constexpr int SPB = W == 8 ? 4 : W == 4 ? 16 : 1;  // samples per block
  constexpr int TPS = 64 / SPB;                   // tiles per sample in the block
  constexpr int HRS = (W == 32 ? 8 : W) + 2;      // halo rows per sample
  constexpr int PS = W == 8 ? 11 : HRS;           // halo row pitch between stacked samples
  constexpr int HR = SPB * PS, HC = W + 2;        // halo rows / columns
  constexpr int RP = W == 32 ? 88 : W == 16 ? 46 : W == 8 ? 26 : 18;  // parity-plane row pitch, 16-byte units
  constexpr int SQ = W == 4 ? 218 * 4 : PS * 8 * RP;  // floats per stacked sample (W = 4: not whole rows)
  constexpr int HBUF = SPB * SQ;                  // floats per halo buffer
  // W = 4: the halo ring of every (whole) sample is zero padding — written once, both buffers, before
  // the loop; the chunks stage the 4 x 4 interiors only (1024 pieces: 2 per thread instead of 5)
  constexpr bool RING0 = W == 4;
  constexpr int CK = 16;                    // channels per chunk
  constexpr int NPC = RING0 ? SPB * W * W * (CK / 4) : HR * HC * (CK / 4);  // float4 pieces per chunk
  constexpr int NPI = (NPC + 511) / 512;    // pieces per thread
  // W = 4: the zero rings written once before the loop are never a store_halo target — every piece
  // is an interior pixel (NPC a whole number of 512-thread rounds, so no piece takes a scratch slot)
  static_assert(!RING0 || NPC % 512 == 0, "W = 4: interior pieces must fill whole thread rounds");
  // epilogue LDS row pitch: 32 tiles + 2 — with 8-byte stores / reads, 34 cc mod 64 dwords puts
  // the 32 lanes of each ds_read_b64 group on 32 distinct bank pairs (a pitch of 36, needed by
  // 16-byte stores, made every read 2-way conflicted): Winograd launches -2 % in the eager
  // breakdown
  constexpr int EPP = 34;
  constexpr int EPF = 16 * 32 * EPP;        // epilogue floats (one 32 x 32 pass, 16 positions)
  constexpr int LDSF = 2 * HBUF + 1024 > EPF ? 2 * HBUF + 1024 : EPF;
  __shared__ __attribute__((aligned(16))) float lds[LDSF];

  WSTAMP(0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wi = wid >> 1, jp = wid & 1;
  int mt, nt, bz;
  xcd_tile(mt, nt, bz);
  // The map is p.H x p.W (WA) inside the W-wide geometry: WA <= W columns (W = 32: any height, 8-row
  // bands, BPS per sample; W <= 16: p.H <= W, whole samples).  Halo pixels past the map stage zeros
  // (the conv's zero padding), outputs past it are neither stored nor counted in the partials.
  const int WA = p.W;
  const int BPS = W == 32 ? (p.H + 7) >> 3 : 1;  // blocks per sample
  const int HW = p.H * WA, C = p.src.C;
  const int nsmp = W == 32 ? mt / BPS : mt * SPB;  // first sample of the block
  const int band = W == 32 ? mt - nsmp * BPS : 0;
  const int y0 = 8 * band;  // W = 32: first row of the band
  const int nsamp = p.M / HW;  // W = 8 / 4: samples past the batch (last block) stage zeros, write nothing
  const int nch_all = C / CK;
  const int cbeg = EPI == EPI_PARTIAL ? bz * p.ksplit : 0;  // first chunk of this split
  const int nch = EPI == EPI_PARTIAL ? min(p.ksplit, nch_all - cbeg) : nch_all;

  // ---- halo pieces of this thread: (halo pixel, 4-channel quad), global element offset (chunk 0)
  // or -1 (zero padding), LDS float offset
  int hoff[NPI], hls[NPI];
#pragma unroll
  for (int k = 0; k < NPI; ++k) {
    const int e = tid + 512 * k;
    const int h = e >> 2, q = e & 3;
    // halo row (all stacked samples) and column of pixel slot h.  The 8-lane groups of ds_write_b128
    // (two pixels each) must cover 32 distinct banks: the two pixels' 16-float pieces must sit 16 mod
    // 32 floats apart.  W = 32 (4 RP = 0 mod 32): columns c and c + 8 of one row (10 pixel-pitches
    // of 20 floats apart: 16 mod 32); W = 16 / 8 (8 RP = 16 mod 32): one column in rows 2t, 2t + 1.
    // Plain row-major slots put parity-plane neighbours on the same banks (2-way conflicts on every
    // halo store).
    int hrow, hcol;
    if constexpr (RING0) {
      hrow = h / HC;
      hcol = h - hrow * HC;
    } else if constexpr (W == 32) {
      const int pr = (h >> 1) % 17, m = h & 1;  // 17 pixel pairs per 34-column row
      hrow = (h >> 1) / 17;
      hcol = pr < 8 ? pr + 8 * m : pr < 16 ? 8 + pr + 8 * m : 32 + m;
    } else {
      const int t = (h >> 1) / HC;  // HR is even: row pairs
      hcol = (h >> 1) - t * HC;
      hrow = 2 * t + (h & 1);
    }
    // stacked sample, halo row inside it, halo column (RING0: interior pixel h of the block's samples)
    const int sh = RING0 ? h >> 4 : hrow / PS;
    const int ry = RING0 ? ((h >> 2) & 3) + 1 : hrow - sh * PS;
    const int hx = RING0 ? (h & 3) + 1 : hcol;
    const int y = y0 + ry - 1, x = hx - 1;
    const bool ok = e < NPC && ry < HRS && y >= 0 && y < p.H && x >= 0 && x < WA && nsmp + sh < nsamp;
    hoff[k] = ok ? ((((nsmp + sh) * p.H + y) * WA + x) * C + q * 4) : -1;
    // pieces past the halo store to a scratch slot of their own (no divergent branch around the store)
    hls[k] = e < NPC ? (sh * SQ + (ry * 2 + (hx & 1)) * RP * 4 + (hx >> 1) * 20 + q * 4) : 2 * HBUF + (tid & 255) * 4;
  }
  const __amdgpu_buffer_rsrc_t rA = rsrc_of(p.src.src0, P.a_bytes);
  const __amdgpu_buffer_rsrc_t rRes = rsrc_of(GNA == 2 ? (const void*)P.gn_res : (const void*)p.src.src0, P.a_bytes);

  // ---- GroupNorm(1, C) statistics of the block's samples (as igemm_halo_kernel / norm_kernel reduce
  // them: 256 threads sum strided partials in double, wave shuffle tree, ((w0 + w1) + (w2 + w3)))
  __shared__ float2 gst_s[SPB];
  if constexpr (GNA) {
    __shared__ double gr1[4], gr2[4];
    for (int sp = 0; sp < SPB; ++sp) {
      if (tid < 256 && nsmp + sp < nsamp) {
        const float2* rp = P.gn_rowpart + (size_t)(nsmp + sp) * P.gn_cnt;
        double s1 = 0.0, s2 = 0.0;
        for (int i = tid; i < P.gn_cnt; i += 256) {
          const float2 q = rp[i];
          s1 += (double)q.x;
          s2 += (double)q.y;
        }
        s1 = wave_sum_dpp(s1);
        s2 = wave_sum_dpp(s2);
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
        gst_s[sp] = make_float2((float)mean, (float)(1.0 / sqrt(var + 1e-5)));
      }
      __syncthreads();
    }
  }

  floatx4 ha[NPI];
  floatx4 hr[GNA == 2 ? NPI : 1];
  auto load_halo = [&](int c) {
#pragma unroll
    for (int k = 0; k < NPI; ++k) {
      const int off = hoff[k] >= 0 ? (hoff[k] + (cbeg + c) * CK) * 4 : kOOB;
      ha[k] = bload_f4(rA, off, 0);
      if constexpr (GNA == 2) hr[k] = bload_f4(rRes, off, 0);
    }
  };
  auto store_halo = [&](int buf, int c) {
    float* hb = lds + buf * HBUF;
    floatx4 ggam = {0.f, 0.f, 0.f, 0.f}, gbet = {0.f, 0.f, 0.f, 0.f};
    if constexpr (GNA) {  // every piece of this thread holds the same channel quad (512 % 4 == 0)
      const int ch = (cbeg + c) * CK + (tid & 3) * 4;
      ggam = ld4(P.gn_gamma + ch);  // (L1 / L2 hits: 32 bytes per thread per chunk)
      gbet = ld4(P.gn_beta + ch);
    }
#pragma unroll
    for (int k = 0; k < NPI; ++k) {
      floatx4 v = ha[k];
      if constexpr (GNA) {  // GroupNorm (+ residual) + GELU of the raw source; zero padding stays zero
        const float2 gst = gst_s[SPB == 1 ? 0 : min(hls[k] / SQ, SPB - 1)];  // (the piece's stacked sample)
        v = gn_apply4v(v, gst, ggam, gbet, GNA == 1 ? 1 : 0);
        if constexpr (GNA == 2) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = gelu(hr[k][j] + v[j]);
        }
        if (hoff[k] < 0) v = floatx4{0.f, 0.f, 0.f, 0.f};
      }
      *reinterpret_cast<floatx4*>(hb + hls[k]) = v;
    }
  };

  // ---- U fragments: positions xi0, xi0 + 1 (wave-uniform), column tiles 2 nt, 2 nt + 1
  const int xi0 = 4 * wi + 2 * jp;
  const int NB = p.Cout / 32, KK = C / 16;
  const __amdgpu_buffer_rsrc_t rUh = rsrc_of(P.Uh, P.u_bytes), rUl = rsrc_of(P.Ul, P.u_bytes);
  int ub[2][2];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int n = 0; n < 2; ++n) ub[q][n] = (((xi0 + q) * NB + 2 * nt + n) * KK) * 1024;
  const int voff = lane * 16;
  half8 bh[2][2], bl[2][2];
  int cnext = 0;  // chunk whose fragments load_b(.., -1) fetches
  auto load_b = [&](int q, int n, int c) {
    const int cc = c < 0 ? cnext : c;
    bh[q][n] = bload_h8(rUh, voff, ub[q][n] + (cbeg + cc) * 1024);
    if constexpr (!X1) bl[q][n] = bload_h8(rUl, voff, ub[q][n] + (cbeg + cc) * 1024);
  };

  // ---- A fragments: rows (Bᵀ row wi) and columns (B columns of positions 2jp, 2jp + 1)
  // T(col) = d(ra, col) + sr d(rb, col);  V_a = T(cp) - T(cq);  V_b = T(cq) + sb T(cs)
  const int ra = wi == 0 ? 0 : wi == 2 ? 2 : 1;
  const int rb = wi == 0 ? 2 : wi == 2 ? 1 : wi == 1 ? 2 : 3;
  const float sr = wi == 1 ? 1.f : -1.f;
  const int cp = jp ? 2 : 0, cq = jp ? 1 : 2, cs = jp ? 3 : 1;
  const float sb = jp ? -1.f : 1.f;
  auto coff = [&](int col) { return (col & 1) * RP * 4 + (col >> 1) * 20; };
  const int oa = ra * 8 * RP, ob = rb * 8 * RP;
  const int op = coff(cp), oq = coff(cq), os = coff(cs);
  const int fr = lane & 31, fh = lane >> 5;
  int tb[2];
#pragma unroll
  for (int mb = 0; mb < 2; ++mb) {
    const int t = 32 * mb + fr, st = t / TPS, tt = t - st * TPS, ty = tt / TW, tx = tt - ty * TW;
    tb[mb] = st * SQ + 2 * ty * 8 * RP + tx * 20 + 8 * fh;
  }
  half8 ah[2][2], al[2][2];  // [m tile][position]
  auto build = [&](int buf, int mb) {
    const float* hb = lds + buf * HBUF + tb[mb];
    unsigned vh[2][4], vl[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {  // channels 4h .. 4h + 3 of the lane's eight (fewer live registers)
      floatx4 T[3];
      const int oc[3] = {op, oq, os};
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const floatx4 da = *reinterpret_cast<const floatx4*>(hb + oa + oc[k] + 4 * h);
        const floatx4 db = *reinterpret_cast<const floatx4*>(hb + ob + oc[k] + 4 * h);
#pragma unroll
        for (int e = 0; e < 4; ++e) T[k][e] = fmaf(db[e], sr, da[e]);
      }
#pragma unroll
      for (int e = 0; e < 4; e += 2) {
        const float a0 = T[0][e] - T[1][e], a1 = T[0][e + 1] - T[1][e + 1];
        const float b0 = fmaf(T[2][e], sb, T[1][e]), b1 = fmaf(T[2][e + 1], sb, T[1][e + 1]);
        if constexpr (X1) {  // config 4: V rounded to f16 once, no lo part
          vh[0][2 * h + e / 2] = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){a0, a1}, half2v));
          vh[1][2 * h + e / 2] = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){b0, b1}, half2v));
        } else {
          split2u(a0, a1, vh[0][2 * h + e / 2], vl[0][2 * h + e / 2]);
          split2u(b0, b1, vh[1][2 * h + e / 2], vl[1][2 * h + e / 2]);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      ah[mb][q] = __builtin_bit_cast(half8, (u32x4){vh[q][0], vh[q][1], vh[q][2], vh[q][3]});
      if constexpr (!X1) al[mb][q] = __builtin_bit_cast(half8, (u32x4){vl[q][0], vl[q][1], vl[q][2], vl[q][3]});
    }
  };

  floatx16 acc[2][2][2];  // [position][m tile][n tile]
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[q][i][j][r] = 0.f;

  // ---- prologue: chunk 0's halo in LDS, chunk 1's halo and chunk 0's U fragments in flight — issued
  // in the loop's steady-state order (halo loads older than U loads), so the counted vmcnt waits the
  // compiler derives at the loop head (merged over entry and back edge) let the store of the halo
  // retire only the halo loads instead of draining the U fragments too
  if constexpr (RING0) {  // zero both halo buffers once (the rings are never stored again)
    for (int i = tid; i < 2 * HBUF / 4; i += 512) *reinterpret_cast<floatx4*>(lds + 4 * i) = floatx4{0.f, 0.f, 0.f, 0.f};
  }
  load_halo(0);
  if constexpr (RING0) __syncthreads();
  store_halo(0, 0);
  load_halo(min(1, nch - 1));
  // Pin the issue order (chunk 1's halo loads older than chunk 0's U loads, as in the loop body): the
  // scheduler otherwise hoisted four U loads above them, and the vmcnt wait the compiler derives at
  // the loop head (merged over this entry and the back edge) then also drained two U loads of the
  // previous chunk before every halo store — the U latency landed in front of the store and the A
  // build instead of under them.
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int n = 0; n < 2; ++n) load_b(q, n, 0);
  __syncthreads();
  WSTAMP(1);

  // Per chunk c (halo buffers alternate; U fragments rolling in registers):
  //   store chunk c + 1's halo (registers loaded one chunk earlier) -> buffer (c + 1) & 1, issue chunk
  //   c + 2's halo loads; A fragments of m tile 0 + its 12 MFMAs; A fragments of m tile 1 + its 12
  //   MFMAs, each U fragment reloaded for chunk c + 1 right after its last use; BARRIER.
  // (Measured: the barrier placed before the last MFMA group — to overlap those MFMAs with the next
  // chunk's halo store — raced: with the sched barriers below, stored halo values of the next chunk
  // reached LDS before slower waves' reads of the buffer, i.e. the hardware barrier no longer split
  // the two; some GroupNorm-on-load outputs came out wrong.  Kept at the chunk end.)  Global loads are
  // pinned by sched barriers (only VALU / SALU / LDS ops may move across), so the compiler cannot
  // sink them to the loop end, and they are issued unconditionally (chunk indices clamped; the loads
  // of the last iterations are never used) so the vector-memory counter waits stay exact.
  auto mfmas = [&](int i, bool reload) {
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        if constexpr (!X1) {
          acc[q][i][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i][q], bh[q][n], acc[q][i][n], 0, 0, 0);
          acc[q][i][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i][q], bl[q][n], acc[q][i][n], 0, 0, 0);
        }
        acc[q][i][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i][q], bh[q][n], acc[q][i][n], 0, 0, 0);
        if (reload) {
          load_b(q, n, -1);
          __builtin_amdgcn_sched_barrier(0x0086);
        }
      }
  };
  // (GroupNorm-on-load instances keep the plain loop: their halo store's VALU and registers make the
  // pipelined one spill)
  if constexpr (GNA == 0) {
  // Software-pipelined A build (one barrier per chunk, in the middle).  Iteration c runs m tile 0's
  // MFMAs beside the build of m tile 1's A fragments (halo buffer c & 1); then, after the barrier
  // that publishes chunk c + 1's halo, m tile 1's MFMAs beside the build of chunk c + 1's m tile 0
  // fragments (buffer (c + 1) & 1) and the U reloads — so the matrix pipe never waits for a whole A
  // build.  Buffer (c + 1) & 1 is stored at the top of iteration c; its previous readers (chunk
  // c - 1's builds) all precede barrier c - 1, and its readers in iteration c follow barrier c.
  // The build is cut into pieces (LDS reads of a 4-channel half, its T columns, its V / split), one
  // piece per MFMA slot; sched_barrier(0) between slots keeps the order as written, so the reads run
  // ahead of their VALU by three slots and every MFMA has the transform work of its slot beside it.
  constexpr int NM = X1 ? 4 : 12;  // MFMAs per m tile and chunk
  floatx4 pda[2][3], pdb[2][3], pT[3];
  u32x4 pah[2][2], pal[2][2];  // [m tile][position] A fragments (f16 pairs)
  auto p_read = [&](int buf, int mb, int h) {
    const float* hb = lds + buf * HBUF + tb[mb];
    const int oc[3] = {op, oq, os};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      pda[h][k] = *reinterpret_cast<const floatx4*>(hb + oa + oc[k] + 4 * h);
      pdb[h][k] = *reinterpret_cast<const floatx4*>(hb + ob + oc[k] + 4 * h);
    }
  };
  auto p_T = [&](int h) {
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) pT[k][e] = fmaf(pdb[h][k][e], sr, pda[h][k][e]);
  };
  auto p_V = [&](int mb, int h, int e) {  // channels 4h + e, 4h + e + 1
    const float a0 = pT[0][e] - pT[1][e], a1 = pT[0][e + 1] - pT[1][e + 1];
    const float b0 = fmaf(pT[2][e], sb, pT[1][e]), b1 = fmaf(pT[2][e + 1], sb, pT[1][e + 1]);
    const int j = 2 * h + e / 2;
    if constexpr (X1) {
      pah[mb][0][j] = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){a0, a1}, half2v));
      pah[mb][1][j] = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){b0, b1}, half2v));
    } else {
      unsigned h0, l0, h1, l1;
      split2u(a0, a1, h0, l0);
      split2u(b0, b1, h1, l1);
      pah[mb][0][j] = h0;
      pal[mb][0][j] = l0;
      pah[mb][1][j] = h1;
      pal[mb][1][j] = l1;
    }
  };
  // build piece of slot s (build target m tile mb from buffer buf); -1: none
  auto p_piece = [&](int s, int buf, int mb) {
    if constexpr (X1) {
      if (s == 0) { p_read(buf, mb, 0); p_read(buf, mb, 1); }
      if (s == 1) { p_T(0); p_V(mb, 0, 0); p_V(mb, 0, 2); }
      if (s == 2) { p_T(1); p_V(mb, 1, 0); p_V(mb, 1, 2); }
    } else {
      if (s == 0) p_read(buf, mb, 0);
      if (s == 3) { p_T(0); p_read(buf, mb, 1); }
      if (s == 4) p_V(mb, 0, 0);
      if (s == 5) p_V(mb, 0, 2);
      if (s == 6) p_T(1);
      if (s == 7) p_V(mb, 1, 0);
      if (s == 8) p_V(mb, 1, 2);
    }
  };
  // MFMA slot s of m tile i: position q, column tile n, product (x3: al*bh, ah*bl, ah*bh)
  auto p_mfma = [&](int i, int s) {
    const int pr = X1 ? 2 : s % 3, qn = X1 ? s : s / 3, q = qn >> 1, n = qn & 1;
    const half8 A = __builtin_bit_cast(half8, pr == 0 ? pal[i][q] : pah[i][q]);
    const half8 Bf = pr == 1 ? bl[q][n] : bh[q][n];
    acc[q][i][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A, Bf, acc[q][i][n], 0, 0, 0);
  };
  // prologue build: chunk 0's m tile 0 (buffer 0, published by the prologue barrier)
  p_read(0, 0, 0);
  p_T(0);
  p_read(0, 0, 1);
  p_V(0, 0, 0);
  p_V(0, 0, 2);
  p_T(1);
  p_V(0, 1, 0);
  p_V(0, 1, 2);
  constexpr bool LATE = GNA == 2 || (W != 32 && GNA == 1);  // (register pressure: after the barrier)
  auto iter = [&](int c, auto last) {
    store_halo((c + 1) & 1, min(c + 1, nch - 1));  // c + 1 = nch: an unused store of the last chunk
    if constexpr (!LATE) load_halo(min(c + 2, nch - 1));
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int sl = 0; sl < NM; ++sl) {  // phase X: m tile 0 (A built last phase) | build m tile 1
      p_mfma(0, sl);
      p_piece(sl, c & 1, 1);
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
    if constexpr (LATE) load_halo(min(c + 2, nch - 1));
    cnext = min(c + 1, nch - 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int sl = 0; sl < NM; ++sl) {  // phase Y: m tile 1 | build chunk c + 1's m tile 0, U reloads
      p_mfma(1, sl);
      if constexpr (!decltype(last)::value) p_piece(sl, (c + 1) & 1, 0);
      if (X1 || sl % 3 == 2) {
        const int qn = X1 ? sl : sl / 3;
        load_b(qn >> 1, qn & 1, -1);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  for (int c = 0; c < nch - 1; ++c) iter(c, std::false_type{});
  iter(nch - 1, std::true_type{});
  } else {
  for (int c = 0; c < nch; ++c) {
    store_halo((c + 1) & 1, min(c + 1, nch - 1));  // c + 1 = nch: an unused store of the last chunk
    // (No barrier here: buffer (c + 1) & 1 was last read by chunk c - 1's builds, which the previous
    // iteration's closing barrier orders before this store, and this chunk's builds read the other
    // buffer.  An earlier build with the GroupNorm affine in an LDS table was nondeterministic
    // without a barrier here (tools/det_check.py); with the affine read from global memory the
    // barrier is not needed — 0 of 9 repeats and 0 of 36 concurrent-process steps differ — and
    // dropping it is +1.7-2.2 % per CFG step, 3 / 3 same-box rounds.)
    constexpr bool LATE = GNA == 2 || (W != 32 && GNA == 1);  // (register pressure: after m tile 0)
    if constexpr (!LATE) {
      load_halo(min(c + 2, nch - 1));
      __builtin_amdgcn_sched_barrier(0x0086);
    }
    build(c & 1, 0);
    mfmas(0, false);
    if constexpr (LATE) {
      load_halo(min(c + 2, nch - 1));
      __builtin_amdgcn_sched_barrier(0x0086);
    }
    build(c & 1, 1);
    cnext = min(c + 1, nch - 1);
    mfmas(1, true);
    __syncthreads();
  }
  }

  // ---- epilogue: Aᵀ M A per tile, four passes of 32 tiles x 32 channels through LDS
  __syncthreads();  // (the halo buffers become the epilogue's staging area)
  WSTAMP(2);
  // GroupNorm partial rows per sample: one per 4 geometry tiles (rows wholly past the map hold zeros)
  const int HW16 = BPS * 64 / SPB / 4, nseg = p.Cout / 32;
  const int tile0 = band * 64;  // first tile of the block inside its sample
  const int cc = tid & 31, tp = tid >> 5;  // output task: channel cc, tiles 2 tp, 2 tp + 1
#pragma unroll
  for (int mb = 0; mb < 2; ++mb)
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      // positions -> LDS [xi][channel][tile] (rows of a lane's accumulator are 4 consecutive tiles)
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          floatx4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = acc[q][mb][n][4 * k + e] * P.inv_scale;
          float* e = &lds[((xi0 + q) * 32 + fr) * EPP + 8 * k + 4 * fh];
          *reinterpret_cast<f32x2*>(e) = f32x2{v[0], v[1]};
          *reinterpret_cast<f32x2*>(e + 2) = f32x2{v[2], v[3]};
        }
      __syncthreads();
      float m[16][2];
#pragma unroll
      for (int xi = 0; xi < 16; ++xi) {
        const f32x2 v = *reinterpret_cast<const f32x2*>(&lds[(xi * 32 + cc) * EPP + 2 * tp]);
        m[xi][0] = v.x;
        m[xi][1] = v.y;
      }
      const int col = 64 * nt + 32 * n + cc;
      // (split partials carry no bias: the slab reduction adds it once)
      const float bias = (EPI == EPI_STATS && p.bias != nullptr) ? p.bias[col] : 0.f;
      float* dst = EPI == EPI_PARTIAL ? p.partial + (size_t)bz * p.M * p.Cout : p.out;
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        float z[4][2];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          z[i][0] = (m[4 * i][e] + m[4 * i + 1][e]) + m[4 * i + 2][e];
          z[i][1] = (m[4 * i + 1][e] - m[4 * i + 2][e]) - m[4 * i + 3][e];
        }
        const int t = 32 * mb + 2 * tp + e, st = t / TPS, tt = t - st * TPS, ty = tt / TW, tx = tt - ty * TW;
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const float y = (r == 0 ? (z[0][s] + z[1][s]) + z[2][s] : (z[1][s] - z[2][s]) - z[3][s]) + bias;
            const int oy = y0 + 2 * ty + r, ox = 2 * tx + s;
            const bool in = oy < p.H && ox < WA;
            // non-temporal: the output streams to memory instead of sitting dirty in the XCDs' L2s
            // until the end-of-kernel writeback (+1.5-1.7 % per CFG step, split slabs +0.8 %)
            if (nsmp + st < nsamp && in)
              __builtin_nontemporal_store(y, &dst[(((size_t)(nsmp + st) * p.H + oy) * WA + ox) * p.Cout + col]);
            const float yv = in ? y : 0.f;
            s1 += yv;
            s2 += yv * yv;
          }
      }
      // partial of 4 tiles (16 pixels) x 32 channels = this wave's 64 lanes
      if constexpr (EPI == EPI_STATS) {  // (DPP / permlane: no LDS round trips in the epilogue)
        s1 = wave_sum_dpp(s1);
        s2 = wave_sum_dpp(s2);
      }
      if (EPI == EPI_STATS && lane == 0) {  // the wave's 4 tiles: one tile row of one sample
        const int t = 32 * mb + 4 * wid, st = t / TPS, g = (tile0 + t - st * TPS) / 4;
        if (nsmp + st < nsamp) p.rowpart[((size_t)(nsmp + st) * HW16 + g) * nseg + 2 * nt + n] = make_float2(s1, s2);
      }
      __syncthreads();
    }
  WSTAMP(3);
}

}  // namespace dmx
