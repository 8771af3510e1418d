// dmx — split-precision attention core instantiations (attention_x3_kernel, see launch.h).
#include <cstdlib>

#include "launch.h"

namespace dmx {

static bool att_pipe() {  // A/B knob DMX_ATT_PIPE=0: the non-pipelined core for D = 16 / 32
  static const bool v = [] {
    const char* e = std::getenv("DMX_ATT_PIPE");
    return e ? std::atoi(e) != 0 : true;
  }();
  return v;
}

void launch_attention_x3(int D, int wpe, int x1, const float* qkv, float* out, int L, int C, dim3 grid,
                         hipStream_t st) {
  if (att_pipe() && (D == 16 || D == 32)) {
    if (D == 16) { if (x1) attention_x3p_kernel<16, 1><<<grid, 256, 0, st>>>(qkv, out, L, C); else attention_x3p_kernel<16, 0><<<grid, 256, 0, st>>>(qkv, out, L, C); }
    else { if (x1) attention_x3p_kernel<32, 1><<<grid, 256, 0, st>>>(qkv, out, L, C); else attention_x3p_kernel<32, 0><<<grid, 256, 0, st>>>(qkv, out, L, C); }
    return;
  }
#define ATX(DD, W, X) attention_x3_kernel<DD, W, X><<<grid, 256, 0, st>>>(qkv, out, L, C)
  if (D == 16) { if (wpe == 4) { if (x1) ATX(16, 4, 1); else ATX(16, 4, 0); } else { if (x1) ATX(16, 1, 1); else ATX(16, 1, 0); } }
  else if (D == 32) { if (x1) ATX(32, 1, 1); else ATX(32, 1, 0); }
  else { if (x1) ATX(64, 1, 1); else ATX(64, 1, 0); }
#undef ATX
}

}  // namespace dmx
