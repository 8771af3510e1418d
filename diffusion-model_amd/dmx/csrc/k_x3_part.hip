// dmx — igemm_x3_kernel instantiations with the split-K partial-slab epilogue (see launch.h).
#include "launch.h"

namespace dmx {

template <int BM, int BN, int SA, int X1>
static void go(const X3Params& p, dim3 grid, hipStream_t st) {
  if constexpr (BN == 128) {  // 8 waves: 2 x 4 waves of (BM/2) x 32
    if (BM == 128) {
      igemm_x3_kernel<BM, BN, EPI_PARTIAL, 64, 1, SA, X1, 8><<<grid, 512, 0, st>>>(p);
      return;
    }
  }
  igemm_x3_kernel<BM, BN, EPI_PARTIAL, 64, 1, SA, X1><<<grid, 256, 0, st>>>(p);
}

template <int SA, int X1>
static void tiles(int bm, int bn, const X3Params& p, dim3 grid, hipStream_t st) {
  if (bm == 128 && bn == 128) go<128, 128, SA, X1>(p, grid, st);
  else if (bm == 128) go<128, 64, SA, X1>(p, grid, st);
  else if (bn == 128) go<64, 128, SA, X1>(p, grid, st);
  else go<64, 64, SA, X1>(p, grid, st);
}

void launch_x3_partial(int bm, int bn, int sa, int x1, const X3Params& p, dim3 grid, hipStream_t st) {
  if (sa) { if (x1) tiles<1, 1>(bm, bn, p, grid, st); else tiles<1, 0>(bm, bn, p, grid, st); }
  else { if (x1) tiles<0, 1>(bm, bn, p, grid, st); else tiles<0, 0>(bm, bn, p, grid, st); }
}

}  // namespace dmx
