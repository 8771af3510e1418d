// dmx — igemm_x3_kernel instantiations with the bias / GELU / residual epilogues (see launch.h).
#include "launch.h"

namespace dmx {

template <int BM, int BN, int EPI, int SA, int X1>
static void go(const X3Params& p, dim3 grid, hipStream_t st) {
  igemm_x3_kernel<BM, BN, EPI, 64, 1, SA, X1><<<grid, 256, 0, st>>>(p);
}

template <int EPI, int SA, int X1>
static void tiles(int bm, int bn, const X3Params& p, dim3 grid, hipStream_t st) {
  if (bm == 128 && bn == 128) go<128, 128, EPI, SA, X1>(p, grid, st);
  else if (bm == 128) go<128, 64, EPI, SA, X1>(p, grid, st);
  else if (bn == 128) go<64, 128, EPI, SA, X1>(p, grid, st);
  else go<64, 64, EPI, SA, X1>(p, grid, st);
}

template <int EPI>
static void by_mode(int bm, int bn, int sa, int x1, const X3Params& p, dim3 grid, hipStream_t st) {
  if (sa) { if (x1) tiles<EPI, 1, 1>(bm, bn, p, grid, st); else tiles<EPI, 1, 0>(bm, bn, p, grid, st); }
  else { if (x1) tiles<EPI, 0, 1>(bm, bn, p, grid, st); else tiles<EPI, 0, 0>(bm, bn, p, grid, st); }
}

void launch_x3_epi(int epi, int bm, int bn, int sa, int x1, const X3Params& p, dim3 grid, hipStream_t st) {
  switch (epi) {
    case EPI_BIAS: by_mode<EPI_BIAS>(bm, bn, sa, x1, p, grid, st); break;
    case EPI_BIAS_GELU: by_mode<EPI_BIAS_GELU>(bm, bn, sa, x1, p, grid, st); break;
    case EPI_BIAS_RES: by_mode<EPI_BIAS_RES>(bm, bn, sa, x1, p, grid, st); break;
    default: break;
  }
}

}  // namespace dmx
