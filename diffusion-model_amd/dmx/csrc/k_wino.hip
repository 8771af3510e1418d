// dmx — wino_kernel (Winograd F(2x2, 3x3) split-precision 3x3 conv) instantiations (see launch.h).
#include "igemm_wino.h"
#include "launch.h"

#include <algorithm>

namespace dmx {

template <int W, int EPI>
static void go(int gna, const X3Params& p, dim3 grid, hipStream_t st) {
  if (gna == 1) wino_kernel<W, 1, EPI><<<grid, 512, 0, st>>>(p);
  else if (gna == 2) wino_kernel<W, 2, EPI><<<grid, 512, 0, st>>>(p);
  else wino_kernel<W, 0, EPI><<<grid, 512, 0, st>>>(p);
}

template <int EPI>
static void by_w(int w, int gna, const X3Params& p, dim3 grid, hipStream_t st) {
  if (w == 32) go<32, EPI>(gna, p, grid, st);
  else if (w == 16) go<16, EPI>(gna, p, grid, st);
  else go<8, EPI>(gna, p, grid, st);
}

void launch_wino(int epi, int w, int gna, const X3Params& p, dim3 grid, hipStream_t st) {
  if (epi == EPI_PARTIAL) by_w<EPI_PARTIAL>(w, gna, p, grid, st);
  else by_w<EPI_STATS>(w, gna, p, grid, st);
}

void launch_wino_pack(const float* B, int kpad, int cin, int cout, float scale, _Float16* uh, _Float16* ul,
                      hipStream_t st) {
  const size_t total = (size_t)16 * (cout / 32) * (cin / 16) * 64;
  wino_pack_kernel<<<(int)std::min<size_t>((total + 255) / 256, 4096), 256, 0, st>>>(B, kpad, cin, cout, scale, uh, ul);
}

}  // namespace dmx
