// dmx — fused attention-block token kernel instantiations (tokmlp.h, see launch.h).
#include "launch.h"

#include <stdexcept>

namespace dmx {

void launch_tok_qkv_lds(int C, int tpb, int x1, const TokParams& tp, dim3 gl, hipStream_t st) {
#define TQL(CC, NN, TT) (x1 ? tok_ln_qkv_lds_kernel<CC, NN, TT, 1><<<gl, 256, 0, st>>>(tp) \
                            : tok_ln_qkv_lds_kernel<CC, NN, TT, 0><<<gl, 256, 0, st>>>(tp))
  if (C == 64) {
    if (tpb == 4) TQL(64, 192, 4);
    else if (tpb == 2) TQL(64, 192, 2);
    else TQL(64, 192, 1);
  } else {
    if (tpb == 4) TQL(128, 64, 4);
    else if (tpb == 2) TQL(128, 64, 2);
    else TQL(128, 64, 1);
  }
#undef TQL
}

void launch_tok_qkv(int C, int nb, int x1, const TokParams& tp, dim3 grid, hipStream_t st) {
#define TQ(CC, NN) (x1 ? tok_ln_qkv_kernel<CC, NN, 1><<<grid, 256, 0, st>>>(tp) \
                       : tok_ln_qkv_kernel<CC, NN, 0><<<grid, 256, 0, st>>>(tp))
  switch (C) {
    case 64:
      if (nb == 192) TQ(64, 192);
      else TQ(64, 64);
      break;
    case 128: TQ(128, 128); break;
    default:
      if (nb == 64) TQ(256, 64);
      else TQ(256, 128);
      break;
  }
#undef TQ
}

void launch_tok_qkv_w(int C, int x1, const TokParams& tp, dim3 grid, hipStream_t st) {
  if (C != 256) throw std::runtime_error("launch_tok_qkv_w: C = 256 only");
  if (x1) tok_ln_qkv_w_kernel<256, 384, 8, 4, 1><<<grid, 512, 0, st>>>(tp);
  else tok_ln_qkv_w_kernel<256, 384, 8, 4, 0><<<grid, 512, 0, st>>>(tp);
}

void launch_tok_out(int C, int tm, int x1, int nw, int lds, int tpb, const TokParams& tp, int blocks,
                    hipStream_t st) {
#define TB(CC, TT) (x1 ? tok_attn_out_kernel<CC, TT, 1><<<blocks, 256, 0, st>>>(tp) \
                       : tok_attn_out_kernel<CC, TT, 0><<<blocks, 256, 0, st>>>(tp))
  if (lds) {
#define TBL(TP) (x1 ? tok_attn_out_kernel<64, 128, 1, 8, 1, TP><<<blocks, 512, 0, st>>>(tp) \
                    : tok_attn_out_kernel<64, 128, 0, 8, 1, TP><<<blocks, 512, 0, st>>>(tp))
    if (tpb == 4) TBL(4);
    else if (tpb == 2) TBL(2);
    else TBL(1);
#undef TBL
  } else if (C == 64) TB(64, 64);
  else if (C == 128 && tm == 64) TB(128, 64);
  else if (C == 128) TB(128, 32);
  else if (nw == 8) {
    if (x1) tok_attn_out_kernel<256, 32, 1, 8><<<blocks, 512, 0, st>>>(tp);
    else tok_attn_out_kernel<256, 32, 0, 8><<<blocks, 512, 0, st>>>(tp);
  } else TB(256, 32);
#undef TB
}

}  // namespace dmx
