// dmx — igemm_pp_kernel (512-thread ping-pong split-precision GEMM) instantiations (see launch.h).
#include "igemm_pp.h"
#include "launch.h"

namespace dmx {

template <int BN, int SA, int X1>
static void go(const X3Params& p, dim3 grid, hipStream_t st) {
  igemm_pp_kernel<BN, EPI_STATS, SA, X1><<<grid, 512, 0, st>>>(p);
}

void launch_pp(int bn, int sa, int x1, const X3Params& p, dim3 grid, hipStream_t st) {
  if (bn == 128) {
    if (sa) { if (x1) go<128, 1, 1>(p, grid, st); else go<128, 1, 0>(p, grid, st); }
    else { if (x1) go<128, 0, 1>(p, grid, st); else go<128, 0, 0>(p, grid, st); }
  } else {
    if (sa) { if (x1) go<64, 1, 1>(p, grid, st); else go<64, 1, 0>(p, grid, st); }
    else { if (x1) go<64, 0, 1>(p, grid, st); else go<64, 0, 0>(p, grid, st); }
  }
}

}  // namespace dmx
