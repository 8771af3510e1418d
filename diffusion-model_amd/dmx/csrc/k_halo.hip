// dmx — igemm_halo_kernel / igemm_halo_bd_kernel (halo-staged split-precision 3x3 conv)
// instantiations (see launch.h).
#include "igemm_halo.h"
#include "launch.h"

namespace dmx {

template <int BN, int SA, int X1, int W, int NWN, int NWM>
static void go16(int gna, const X3Params& p, dim3 grid, hipStream_t st) {
  if constexpr (SA == 0) {
    if (gna == 1) {
      igemm_halo_kernel<BN, EPI_STATS, 0, X1, W, 1, NWN, NWM><<<grid, 64 * NWN * NWM, 0, st>>>(p);
      return;
    }
    if (gna == 2) {
      igemm_halo_kernel<BN, EPI_STATS, 0, X1, W, 2, NWN, NWM><<<grid, 64 * NWN * NWM, 0, st>>>(p);
      return;
    }
  }
  igemm_halo_kernel<BN, EPI_STATS, SA, X1, W, 0, NWN, NWM><<<grid, 64 * NWN * NWM, 0, st>>>(p);
}

template <int BN, int SA, int X1, int W>
static void go(int mode, int gna, const X3Params& p, dim3 grid, hipStream_t st) {
  // mode 4: 16-wave blocks — 4 x 4 waves of 64 x 32 (BN = 128) / 8 x 2 waves of 32 x 32 (BN = 64)
  if (mode == 4 || mode == 5) {  // mode 5: BN = 128 as 8 x 2 waves of 32 x 64
    if constexpr (BN == 128) {
      if (mode == 5) go16<BN, SA, X1, W, 2, 8>(gna, p, grid, st);
      else go16<BN, SA, X1, W, 4, 4>(gna, p, grid, st);
    } else {
      go16<BN, SA, X1, W, 2, 8>(gna, p, grid, st);
    }
    return;
  }
  if (mode == 1 && !gna) igemm_halo_bd_kernel<BN, EPI_STATS, SA, X1, W><<<grid, 512, 0, st>>>(p);
  else go16<BN, SA, X1, W, 2, 4>(gna, p, grid, st);
}

template <int SA, int X1>
static void by_shape(int mode, int bn, int w, int gna, const X3Params& p, dim3 grid, hipStream_t st) {
  if (w == 32) {
    if (bn == 128) go<128, SA, X1, 32>(mode, gna, p, grid, st); else go<64, SA, X1, 32>(mode, gna, p, grid, st);
  } else {
    if (bn == 128) go<128, SA, X1, 16>(mode, gna, p, grid, st); else go<64, SA, X1, 16>(mode, gna, p, grid, st);
  }
}

void launch_halo(int mode, int bn, int w, int sa, int x1, int gna, const X3Params& p, dim3 grid, hipStream_t st) {
  if (sa) { if (x1) by_shape<1, 1>(mode, bn, w, 0, p, grid, st); else by_shape<1, 0>(mode, bn, w, 0, p, grid, st); }
  else { if (x1) by_shape<0, 1>(mode, bn, w, gna, p, grid, st); else by_shape<0, 0>(mode, bn, w, gna, p, grid, st); }
}

}  // namespace dmx
