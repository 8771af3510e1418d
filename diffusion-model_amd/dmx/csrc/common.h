// dmx — MI355X (gfx950) native CFG latent-diffusion sampler: shared device/host helpers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DMX_DEV __device__ __forceinline__

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace dmx {

// ---------------------------------------------------------------------------
// Exact (erf) GELU and SiLU in fp32, matching the reference's nn.GELU() /
// F.gelu default (approximate='none') and nn.SiLU (models/unet_cond.py:21,28,63).
// ---------------------------------------------------------------------------
DMX_DEV float gelu(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f)); }
DMX_DEV float silu(float x) { return x / (1.0f + expf(-x)); }

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));

// fp32 -> f16 hi + f16 lo (split-precision operand; lo = f16(v - hi) is exact to ~2^-22 |v|)
DMX_DEV void split4(floatx4 v, half4& h, half4& l) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const _Float16 hi = (_Float16)v[j];
    h[j] = hi;
    l[j] = (_Float16)(v[j] - (float)hi);
  }
}

// Input-source modes of a convolution / token GEMM (how the A operand's
// element (n, iy, ix, c) is produced from HBM).
enum SrcMode : int {
  SRC_PLAIN = 0,    // NHWC tensor src0[n][iy][ix][c]
  SRC_GNACT = 1,    // GELU(GroupNorm(src0)) using per-(n,g) (mean, rstd) stats
  SRC_MAXPOOL = 2,  // max_pool2d(src0, 2): src0 is [n][2H'][2W'][c] (floor mode)
  SRC_UPCAT = 3,    // cat[src0 (skip, C0 ch), pad(bilinear_x2_align(src1))]
  SRC_NCHW = 4,     // NCHW tensor src0[n][c][iy][ix], optionally divided by `scale`
};

// Epilogues of the implicit GEMM.
enum EpiMode : int {
  EPI_STATS = 0,     // store (acc + bias?) and per-row GroupNorm partial sums
  EPI_BIAS = 1,      // acc + bias
  EPI_BIAS_GELU = 2, // GELU(acc + bias)
  EPI_BIAS_RES = 3,  // acc + bias + res
  EPI_PARTIAL = 4,   // split-K: raw accumulator into slab[split] (epilogue in splitk_reduce)
};

struct SrcDesc {
  const float* src0;       // primary tensor
  const float* src1;       // UPCAT: the low-resolution tensor to upsample
  const float2* stats;     // GNACT: (mean, rstd) per (n, g)
  const float* gamma;      // GNACT affine
  const float* beta;
  int C;                   // total channels delivered
  int C0;                  // UPCAT: channels of src0 (skip); src1 has C - C0
  int G;                   // GNACT: groups
  int Hs, Ws;              // MAXPOOL: src0 spatial dims; UPCAT: src1 spatial dims
  int padT, padL;          // UPCAT: F.pad offsets of the upsampled map
  int act;                 // GNACT: 1 => apply GELU after the affine
  float scale;             // NCHW: divide by scale (VAE z / 0.18215), 1 => identity
  int n_mod;               // NCHW / UPCAT skip: sample index taken modulo n_mod (CFG: halves share it)
};

}  // namespace dmx
