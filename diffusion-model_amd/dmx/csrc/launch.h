// dmx — host launchers of the templated kernel families.  Each family is instantiated in its
// own translation unit (k_*.hip) so the library builds in parallel; engine.hip only calls
// these functions.
#pragma once
#include <cstdlib>

#include "common.h"
#include "igemm.h"
#include "igemm_x3.h"
#include "tokmlp.h"

namespace dmx {

// split-precision implicit GEMM (igemm_x3.h): bm, bn in {64, 128}; sa = A from f16 hi/lo planes;
// x1 = config-4 fp16 arithmetic.  k_x3_stats.hip (EPI_STATS), k_x3_part.hip (EPI_PARTIAL),
// k_x3_epi.hip (EPI_BIAS / EPI_BIAS_GELU / EPI_BIAS_RES).
void launch_x3_stats(int bm, int bn, int sa, int x1, const X3Params& p, dim3 grid, hipStream_t st);
// (EPI_STATS / EPI_PARTIAL instances: 8-wave blocks for 128 x 128 tiles — up1.0 -3 %, same-box A/B —
// and 4 waves otherwise; the 64 x 128 split-K tiles at 4x4 / 8x8 are at parity or slower with 8.)
void launch_x3_partial(int bm, int bn, int sa, int x1, const X3Params& p, dim3 grid, hipStream_t st);
void launch_x3_epi(int epi, int bm, int bn, int sa, int x1, const X3Params& p, dim3 grid, hipStream_t st);
// 512-thread ping-pong split-precision GEMM (igemm_pp.h), EPI_STATS, 256 x bn tiles.
void launch_pp(int bn, int sa, int x1, const X3Params& p, dim3 grid, hipStream_t st);
// halo-staged split-precision 3x3 conv (igemm_halo.h), EPI_STATS, 256-pixel x bn tiles, image
// width w in {16, 32}; k_halo.hip.
// mode 1: B fragments read straight from the fragment-ordered planes into registers (one barrier
// per channel chunk); mode 2: B staged in LDS per step (one barrier per step).
// gna = 1 (mode 2, sa = 0): GroupNorm + GELU of the raw source applied while staging.
void launch_halo(int mode, int bn, int w, int sa, int x1, int gna, const X3Params& p, dim3 grid, hipStream_t st);
// the same kernel on low-resolution maps (w in {8, 4}, H == w): 256-pixel tiles of whole samples;
// epi EPI_PARTIAL (grid.z = K splits over 32-channel chunks, P.g.ksplit chunks each) or EPI_STATS
// (w = 8); bn 128 or 64 (w = 4: 64 only); k_halo_ms.hip.
void launch_halo_ms(int epi, int bn, int w, int sa, int x1, const X3Params& p, dim3 grid, hipStream_t st);
// chunk-staged variant (igemm_halo_cs_kernel): BN = 64, all nine taps of a chunk's B slice in LDS.
void launch_halo_cs(int epi, int w, int sa, int x1, const X3Params& p, dim3 grid, hipStream_t st);
// Winograd F(2x2, 3x3) split-precision 3x3 conv (igemm_wino.h), 64 tiles (256 pixels) x 64 channels
// per block, w in {4, 8, 16, 32} (4: EPI_PARTIAL, gna 0 only), gna as launch_halo, x1 = 1 the fp16
// (config 4) instances; k_wino.hip.  epi EPI_STATS (GroupNorm partials: HW / 16 rows per sample) or
// EPI_PARTIAL (grid.z = K splits over 16-channel chunks).
void launch_wino(int epi, int w, int gna, int x1, const X3Params& p, dim3 grid, hipStream_t st);
// U = G g Gᵀ of a packed fp32 3x3 weight ([npad][kpad], k = tap * cin + c), scaled, split, fragment order
void launch_wino_pack(const float* B, int kpad, int cin, int cout, float scale, _Float16* uh, _Float16* ul,
                      hipStream_t st);
// exact-fp32 MFMA implicit GEMM (igemm.h), k_f32.hip.
void launch_f32(int src_mode, int epi, int bm, int bn, const IgemmParams& p, dim3 grid, hipStream_t st);
// attention cores (k_attn.hip): split-precision (D, waves-per-EU hint, x1) and exact fp32 (D, QT).
void launch_attention_x3(int D, int wpe, int x1, const float* qkv, float* out, int L, int C, dim3 grid,
                         hipStream_t st, float* stats = nullptr);
// D = 16 core with the head resident in LDS; grid (1, 4, N), nw waves per block.
hipError_t launch_attention16(int nw, int x1, const float* qkv, float* out, int L, int C, int N, hipStream_t st,
                              float* stats = nullptr);
void launch_attention_f32(int D, int qt, const float* qkv, float* out, int L, int C, dim3 grid, hipStream_t st,
                          float* stats = nullptr);
// fused attention-block token kernels (tokmlp.h), k_tok.hip.
void launch_tok_qkv_lds(int C, int tpb, int x1, const TokParams& tp, dim3 grid, hipStream_t st);
// C = 256 QKV with 8-wave blocks of 64 tokens x 384 columns (tok_ln_qkv_w_kernel); grid (M / 64, 2).
void launch_tok_qkv_w(int C, int x1, const TokParams& tp, dim3 grid, hipStream_t st);
void launch_tok_qkv(int C, int nb, int x1, const TokParams& tp, dim3 grid, hipStream_t st);
void launch_tok_out(int C, int tm, int x1, int nw, int lds, int tpb, const TokParams& tp, int blocks,
                    hipStream_t st);

}  // namespace dmx
