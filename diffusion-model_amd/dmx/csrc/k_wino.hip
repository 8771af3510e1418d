// dmx — wino_kernel (Winograd F(2x2, 3x3) split-precision 3x3 conv) instantiations (see launch.h).
#include "igemm_wino.h"
#include "launch.h"

#include <algorithm>
#include <stdexcept>
#include <vector>

namespace dmx {

#if DMX_DIAG
static int g_wstamp_next = 0;  // stamp slot of the next Winograd launch (reset by dmx_diag_wino_stamps)
#endif

template <int W, int EPI, int X1>
static void go(int gna, const X3Params& p, dim3 grid, hipStream_t st) {
  // (GNA = 2, the residual GELU(x + GN) on load, is never dispatched: engine.hip wino_gna_pays — it
  // lost 10-42 us per conv against a norm pass — so its instances are not built)
  if (gna == 1) wino_kernel<W, 1, EPI, X1><<<grid, 512, 0, st>>>(p);
  else if (gna == 0) wino_kernel<W, 0, EPI, X1><<<grid, 512, 0, st>>>(p);
  else throw std::runtime_error("launch_wino: no GroupNorm-residual-GELU instances");
}

template <int EPI, int X1>
static void by_w(int w, int gna, const X3Params& p, dim3 grid, hipStream_t st) {
  if (w == 32) go<32, EPI, X1>(gna, p, grid, st);
  else if (w == 16) go<16, EPI, X1>(gna, p, grid, st);
  else if (w == 8) go<8, EPI, X1>(gna, p, grid, st);
  else if (EPI == EPI_PARTIAL && gna == 0) wino_kernel<4, 0, EPI_PARTIAL, X1><<<grid, 512, 0, st>>>(p);
  else throw std::runtime_error("launch_wino: W = 4 runs split-K without GroupNorm-on-load only");
}

void launch_wino(int epi, int w, int gna, int x1, const X3Params& p0, dim3 grid, hipStream_t st) {
  X3Params p = p0;
#if DMX_DIAG
  p.dslot = g_wstamp_next++;
#else
  p.dslot = -1;
#endif
  if (x1) {
    if (epi == EPI_PARTIAL) by_w<EPI_PARTIAL, 1>(w, gna, p, grid, st);
    else by_w<EPI_STATS, 1>(w, gna, p, grid, st);
  } else {
    if (epi == EPI_PARTIAL) by_w<EPI_PARTIAL, 0>(w, gna, p, grid, st);
    else by_w<EPI_STATS, 0>(w, gna, p, grid, st);
  }
}

void launch_wino_pack(const float* B, int kpad, int cin, int cout, float scale, _Float16* uh, _Float16* ul,
                      hipStream_t st) {
  const size_t total = (size_t)16 * (cout / 32) * (cin / 16) * 64;
  wino_pack_kernel<<<(int)std::min<size_t>((total + 255) / 256, 4096), 256, 0, st>>>(B, kpad, cin, cout, scale, uh, ul);
}

}  // namespace dmx

// Diagnostic (DMX_DIAG builds): copy the Winograd stamp table (slots x 2048 blocks x {t0, t1, t2,
// t3, hw id}) to the host; returns the number of uint64 copied, 0 in regular builds.
extern "C" int dmx_diag_wino_stamps(unsigned long long* host, int cap) {
#if DMX_DIAG
  if (host == nullptr) {  // reset: the next launch stamps into slot 0, the table is cleared
    dmx::g_wstamp_next = 0;
    static const std::vector<unsigned long long> zeros(sizeof(dmx::g_wstamp) / 8, 0ull);
    return hipMemcpyToSymbol(HIP_SYMBOL(dmx::g_wstamp), zeros.data(), sizeof(dmx::g_wstamp)) == hipSuccess ? 0 : -1;
  }
  const size_t n = std::min<size_t>((size_t)cap, sizeof(dmx::g_wstamp) / 8);
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(dmx::g_wstamp), n * 8, 0, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return (int)n;
#else
  (void)host;
  (void)cap;
  return 0;
#endif
}
