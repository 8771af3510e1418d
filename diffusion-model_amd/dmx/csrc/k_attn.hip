// dmx — split-precision attention core instantiations (attention_x3_kernel, see launch.h).
#include "launch.h"

namespace dmx {

void launch_attention_x3(int D, int wpe, int x1, const float* qkv, float* out, int L, int C, dim3 grid,
                         hipStream_t st, float* stats) {
#define ATX(DD, W, X) attention_x3_kernel<DD, W, X><<<grid, 256, 0, st>>>(qkv, out, L, C, stats)
  if (D == 16) { if (wpe == 4) { if (x1) ATX(16, 4, 1); else ATX(16, 4, 0); } else { if (x1) ATX(16, 1, 1); else ATX(16, 1, 0); } }
  else if (D == 32) { if (x1) ATX(32, 1, 1); else ATX(32, 1, 0); }
  else { if (x1) ATX(64, 1, 1); else ATX(64, 1, 0); }
#undef ATX
}

// D = 16 with the head resident in LDS (attention16_kernel): one block per (sample, head);
// nw = 16 waves for L > 256, 8 for L <= 256.  More than 64 KB of dynamic LDS needs the
// attribute, set once per instantiation (not a stream operation: capture-safe).
template <int NW, int X1>
static hipError_t go16(const float* qkv, float* out, int L, int C, int N, hipStream_t st, float* stats) {
  static size_t granted = 0;
  const size_t bytes = att16_lds_bytes(L, X1);
  if (bytes > granted) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&attention16_kernel<NW, X1>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return e;
    granted = bytes;
  }
  attention16_kernel<NW, X1><<<dim3(1, 4, N), NW * 64, bytes, st>>>(qkv, out, L, C, stats);
  return hipSuccess;
}

hipError_t launch_attention16(int nw, int x1, const float* qkv, float* out, int L, int C, int N, hipStream_t st,
                              float* stats) {
  if (nw == 16) return x1 ? go16<16, 1>(qkv, out, L, C, N, st, stats) : go16<16, 0>(qkv, out, L, C, N, st, stats);
  return x1 ? go16<8, 1>(qkv, out, L, C, N, st, stats) : go16<8, 0>(qkv, out, L, C, N, st, stats);
}

}  // namespace dmx
