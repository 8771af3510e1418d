// dmx — split-precision attention core instantiations (attention_x3_kernel, see launch.h).
#include "launch.h"

#include <cstdlib>

namespace dmx {

void launch_attention_x3(int D, int wpe, int x1, const float* qkv, float* out, int L, int C, dim3 grid,
                         hipStream_t st) {
#define ATX(DD, W, X) attention_x3_kernel<DD, W, X><<<grid, 256, 0, st>>>(qkv, out, L, C)
  if (D == 16) { if (wpe == 4) { if (x1) ATX(16, 4, 1); else ATX(16, 4, 0); } else { if (x1) ATX(16, 1, 1); else ATX(16, 1, 0); } }
  else if (D == 32) { if (x1) ATX(32, 1, 1); else ATX(32, 1, 0); }
  else { if (x1) ATX(64, 1, 1); else ATX(64, 1, 0); }
#undef ATX
}

// D = 16 with the head resident in LDS (attention16_kernel): one block per (sample, head);
// nw = 16 waves for L > 256, 8 for L <= 256.  More than 64 KB of dynamic LDS needs the
// attribute, set once per instantiation (not a stream operation: capture-safe).
template <int NW, int X1>
static hipError_t go16(const float* qkv, float* out, int L, int C, int N, hipStream_t st) {
  static size_t granted = 0;
  const size_t bytes = att16_lds_bytes(L, X1);
  if (bytes > granted) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&attention16_kernel<NW, X1>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return e;
    granted = bytes;
  }
  static const int stag = [] {  // DMX_ATT_STAGGER (same-box A/B): start offset of half the waves
    const char* e = std::getenv("DMX_ATT_STAGGER");
    return e == nullptr ? 0 : std::atoi(e);
  }();
  attention16_kernel<NW, X1><<<dim3(1, 4, N), NW * 64, bytes, st>>>(qkv, out, L, C, stag);
  return hipSuccess;
}

// The 16 x 16 x 32 PV variant (attention16pv_kernel): measured in the eager breakdown (same box,
// B = 64 CFG) 24.6 vs 26.7 us at L = 256 (sa5) but 175.1 vs 170.5 us at L = 1024 (sa6) — the core is
// bound by its per-score VALU (exp, hi / lo split, max), which the variant's permlane swaps and fp32
// denominator sums add to, not by the MFMAs it halves; at L <= 256 only it is neutral in the whole
// step (-0.1 %, 2 / 2 same-box rounds).  DMX_ATT_PV16: 0 (default) never, 2 L <= 256 only, 1 always
// (same-box A/B; the stress-magnitude and golden tests pass with 1).
template <int NW, int X1>
static hipError_t go16pv(const float* qkv, float* out, int L, int C, int N, hipStream_t st) {
  static size_t granted = 0;
  const size_t bytes = att16pv_lds_bytes(L, X1);
  if (bytes > granted) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&attention16pv_kernel<NW, X1>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return e;
    granted = bytes;
  }
  attention16pv_kernel<NW, X1><<<dim3(1, 4, N), NW * 64, bytes, st>>>(qkv, out, L, C);
  return hipSuccess;
}

static int attention16_pv16() {
  static const int v = [] {
    const char* e = std::getenv("DMX_ATT_PV16");
    return e == nullptr ? 0 : std::atoi(e);
  }();
  return v;
}

hipError_t launch_attention16(int nw, int x1, const float* qkv, float* out, int L, int C, int N, hipStream_t st) {
  const int pv = attention16_pv16();
  if (pv == 1 || (pv == 2 && L <= 256)) {
    if (nw == 16) return x1 ? go16pv<16, 1>(qkv, out, L, C, N, st) : go16pv<16, 0>(qkv, out, L, C, N, st);
    return x1 ? go16pv<8, 1>(qkv, out, L, C, N, st) : go16pv<8, 0>(qkv, out, L, C, N, st);
  }
  if (nw == 16) return x1 ? go16<16, 1>(qkv, out, L, C, N, st) : go16<16, 0>(qkv, out, L, C, N, st);
  return x1 ? go16<8, 1>(qkv, out, L, C, N, st) : go16<8, 0>(qkv, out, L, C, N, st);
}

}  // namespace dmx
