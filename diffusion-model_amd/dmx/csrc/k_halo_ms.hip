// dmx — igemm_halo_kernel instantiations for the low-resolution convs (W = 8, 4: 256-pixel tiles of
// whole samples, stacked halos; igemm_halo.h), EPI_PARTIAL (split-K over channel chunks) and
// EPI_STATS (W = 8 only: 32-row GroupNorm partials need H W % 32 == 0).  16-wave blocks as the
// default mode of the whole-row kernel: 4 x 4 waves of 64 x 32 at BN = 128, 8 x 2 of 32 x 32 at
// BN = 64.  W = 4 runs BN = 64 only (its 406-pixel double-buffered halo leaves no LDS for BN = 128).
#include "igemm_halo.h"
#include "launch.h"

namespace dmx {

template <int EPI, int BN, int SA, int X1, int W>
static void go_ms(const X3Params& p, dim3 grid, hipStream_t st) {
  if constexpr (BN == 128) igemm_halo_kernel<128, EPI, SA, X1, W, 0, 4, 4><<<grid, 1024, 0, st>>>(p);
  else igemm_halo_kernel<64, EPI, SA, X1, W, 0, 2, 8><<<grid, 1024, 0, st>>>(p);
}

template <int SA, int X1>
static void ms_shape(int epi, int bn, int w, const X3Params& p, dim3 grid, hipStream_t st) {
  if (w == 8) {
    if (epi == EPI_STATS) {
      if (bn == 128) go_ms<EPI_STATS, 128, SA, X1, 8>(p, grid, st);
      else go_ms<EPI_STATS, 64, SA, X1, 8>(p, grid, st);
    } else {
      if (bn == 128) go_ms<EPI_PARTIAL, 128, SA, X1, 8>(p, grid, st);
      else go_ms<EPI_PARTIAL, 64, SA, X1, 8>(p, grid, st);
    }
  } else {
    go_ms<EPI_PARTIAL, 64, SA, X1, 4>(p, grid, st);
  }
}

template <int SA, int X1>
static void cs_shape(int epi, int w, const X3Params& p, dim3 grid, hipStream_t st) {
  if (w == 8) {
    if (epi == EPI_STATS) igemm_halo_cs_kernel<EPI_STATS, SA, X1, 8><<<grid, 1024, 0, st>>>(p);
    else igemm_halo_cs_kernel<EPI_PARTIAL, SA, X1, 8><<<grid, 1024, 0, st>>>(p);
  } else {
    igemm_halo_cs_kernel<EPI_PARTIAL, SA, X1, 4><<<grid, 1024, 0, st>>>(p);
  }
}

void launch_halo_cs(int epi, int w, int sa, int x1, const X3Params& p, dim3 grid, hipStream_t st) {
  if (sa) { if (x1) cs_shape<1, 1>(epi, w, p, grid, st); else cs_shape<1, 0>(epi, w, p, grid, st); }
  else { if (x1) cs_shape<0, 1>(epi, w, p, grid, st); else cs_shape<0, 0>(epi, w, p, grid, st); }
}

void launch_halo_ms(int epi, int bn, int w, int sa, int x1, const X3Params& p, dim3 grid, hipStream_t st) {
  if (sa) { if (x1) ms_shape<1, 1>(epi, bn, w, p, grid, st); else ms_shape<1, 0>(epi, bn, w, p, grid, st); }
  else { if (x1) ms_shape<0, 1>(epi, bn, w, p, grid, st); else ms_shape<0, 0>(epi, bn, w, p, grid, st); }
}

}  // namespace dmx
