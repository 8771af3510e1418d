// dmx — exact-fp32 MFMA kernels (precision mode 0): igemm_f32_kernel and attention_kernel
// instantiations (see launch.h).
#include "kernels.h"
#include "launch.h"

namespace dmx {

template <int BM, int BN, int SRC, int EPI>
static void go(const IgemmParams& p, dim3 grid, hipStream_t st) {
  igemm_f32_kernel<BM, BN, SRC, EPI><<<grid, 256, 0, st>>>(p);
}

template <int SRC, int EPI>
static void tiles(int bm, int bn, const IgemmParams& p, dim3 grid, hipStream_t st) {
  if (bm == 128 && bn == 128) go<128, 128, SRC, EPI>(p, grid, st);
  else if (bm == 128) go<128, 64, SRC, EPI>(p, grid, st);
  else if (bn == 128) go<64, 128, SRC, EPI>(p, grid, st);
  else go<64, 64, SRC, EPI>(p, grid, st);
}

void launch_f32(int src_mode, int epi, int bm, int bn, const IgemmParams& p, dim3 grid, hipStream_t st) {
  if (src_mode == SRC_NCHW) {
    if (epi == EPI_PARTIAL) tiles<SRC_NCHW, EPI_PARTIAL>(bm, bn, p, grid, st);
    else tiles<SRC_NCHW, EPI_STATS>(bm, bn, p, grid, st);
    return;
  }
  switch (epi) {
    case EPI_STATS: tiles<SRC_PLAIN, EPI_STATS>(bm, bn, p, grid, st); break;
    case EPI_BIAS: tiles<SRC_PLAIN, EPI_BIAS>(bm, bn, p, grid, st); break;
    case EPI_BIAS_GELU: tiles<SRC_PLAIN, EPI_BIAS_GELU>(bm, bn, p, grid, st); break;
    case EPI_BIAS_RES: tiles<SRC_PLAIN, EPI_BIAS_RES>(bm, bn, p, grid, st); break;
    case EPI_PARTIAL: tiles<SRC_PLAIN, EPI_PARTIAL>(bm, bn, p, grid, st); break;
    default: break;
  }
}

void launch_attention_f32(int D, int qt, const float* qkv, float* out, int L, int C, dim3 grid, hipStream_t st,
                          float* stats) {
#define ATT(DD, QQ) attention_kernel<DD, QQ><<<grid, 256, 0, st>>>(qkv, out, L, C, stats)
  if (D == 16) { if (qt == 2) ATT(16, 2); else ATT(16, 1); }
  else if (D == 32) { if (qt == 2) ATT(32, 2); else ATT(32, 1); }
  else { if (qt == 2) ATT(64, 2); else ATT(64, 1); }
#undef ATT
}

}  // namespace dmx
