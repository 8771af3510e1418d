// dmx — split-precision attention core instantiations (attention_x3_kernel, see launch.h).
#include "launch.h"

namespace dmx {

void launch_attention_x3(int D, int wpe, int x1, const float* qkv, float* out, int L, int C, dim3 grid,
                         hipStream_t st) {
#define ATX(DD, W, X) attention_x3_kernel<DD, W, X><<<grid, 256, 0, st>>>(qkv, out, L, C)
  if (D == 16) { if (wpe == 4) { if (x1) ATX(16, 4, 1); else ATX(16, 4, 0); } else { if (x1) ATX(16, 1, 1); else ATX(16, 1, 0); } }
  else if (D == 32) { if (x1) ATX(32, 1, 1); else ATX(32, 1, 0); }
  else { if (x1) ATX(64, 1, 1); else ATX(64, 1, 0); }
#undef ATX
}

}  // namespace dmx
