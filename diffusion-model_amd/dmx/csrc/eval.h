// dmx — generated-image quality metrics of eval_iou_noise.py:
// binarisation, exact Euclidean distance transform to the ground-truth strokes, IoU /
// GT-IoU, far-noise ratio and Gaussian-weighted recall, one workgroup per image pair.
//
// Reference: eval_iou_noise.py:77-94 (load_binary_mask threshold / invert), 162-182
// (_distance_map_to_gt = scipy.ndimage.distance_transform_edt(~gt)), 185-232 (gauss recall,
// far noise) and 239-272 (compute_metrics).
//
// EDT: exact.  Pass 1 (per column) gives the squared vertical distance to the nearest GT pixel
// of that column; pass 2 (per row) takes min_x' (x - x')^2 + g2(x') over the row (brute force,
// every pixel's minimum over its row kept in integers; the row is staged in LDS up to W = 1024
// and read from the workspace beyond), so d2 is the exact integer squared distance and
// dist = sqrt((double)d2) is scipy's float64 value bit for bit.  h, w <= 16384 keeps every
// finite d2 below EV_INF.
// An image with no GT pixel: scipy's transform then measures from the virtual feature (-1, 0),
// d2 = (y + 1)^2 + x^2 (scipy 1.15.3, checked in the oracle tests); reproduced.
// Sums: counts in 64-bit integers, the weighted hits in double, reduced in a fixed order.
#pragma once
#include "common.h"

namespace dmx {

constexpr int EV_INF = 1 << 30;
constexpr int EV_NOUT = 9;  // iou, gt_iou, far_noise_ratio, gauss_recall, inter, union, gt_area, pred_area, fp

struct EvalParams {
  const uint8_t* gt;    // [n][h][w]: masks (0/1) or grayscale (gray = 1)
  const uint8_t* pred;
  int h, w, gray, threshold, invert;
  double sigma;
  int* g2;              // workspace [n][h][w]
  double* out;          // [n][EV_NOUT]
};

DMX_DEV bool ev_fg(const EvalParams& p, uint8_t v) {
  if (!p.gray) return v != 0;
  return p.invert ? (int)v < p.threshold : (int)v >= p.threshold;  // eval_iou_noise.py:89-92
}

static __global__ __launch_bounds__(256) void eval_metrics_kernel(const EvalParams p) {
  const int n = blockIdx.x, tid = threadIdx.x, H = p.h, W = p.w;
  const size_t base = (size_t)n * H * W;
  const uint8_t* gt = p.gt + base;
  const uint8_t* pr = p.pred + base;
  int* g2 = p.g2 + base;
  __shared__ int row[1024];
  __shared__ long long cnt_s[4][5];
  __shared__ double wsum_s[4];
  __shared__ int any_gt;
  if (tid == 0) any_gt = 0;
  __syncthreads();
  // pass 1: per column, squared distance to the nearest GT pixel of the column (down + up sweeps)
  int mine = 0;
  for (int x = tid; x < W; x += 256) {
    int d = EV_INF;
    for (int y = 0; y < H; ++y) {
      const bool f = ev_fg(p, gt[(size_t)y * W + x]);
      d = f ? 0 : (d == EV_INF ? EV_INF : d + 1);
      mine |= f ? 1 : 0;
      g2[(size_t)y * W + x] = d;
    }
    d = EV_INF;
    for (int y = H - 1; y >= 0; --y) {
      const int cur = g2[(size_t)y * W + x];
      d = cur == 0 ? 0 : (d == EV_INF ? EV_INF : d + 1);
      const int m = min(cur, d);
      g2[(size_t)y * W + x] = m == EV_INF ? EV_INF : m * m;
    }
  }
  if (mine) any_gt = 1;  // benign race: every writer stores 1
  __syncthreads();
  const bool empty_gt = any_gt == 0;
  const double two_s2 = 2.0 * (p.sigma * p.sigma);
  long long inter = 0, uni = 0, ga = 0, pa = 0, far = 0;
  double wsum = 0.0;
  const bool staged = W <= 1024;
  for (int y = 0; y < H; ++y) {
    if (staged)
      for (int x = tid; x < W; x += 256) row[x] = g2[(size_t)y * W + x];
    __syncthreads();
    const int* rw = staged ? row : g2 + (size_t)y * W;
    for (int x = tid; x < W; x += 256) {
      int d2;
      if (empty_gt) {
        d2 = (y + 1) * (y + 1) + x * x;
      } else {
        d2 = EV_INF;
        for (int xx = 0; xx < W; ++xx) {
          const int dx = x - xx, v = rw[xx];
          if (v != EV_INF) d2 = min(d2, dx * dx + v);
        }
      }
      const bool g = ev_fg(p, gt[(size_t)y * W + x]), q = ev_fg(p, pr[(size_t)y * W + x]);
      inter += (g && q) ? 1 : 0;
      uni += (g || q) ? 1 : 0;
      ga += g ? 1 : 0;
      pa += q ? 1 : 0;
      if (q) {
        const double dist = sqrt((double)d2);  // scipy's float64 distance
        far += dist > p.sigma ? 1 : 0;
        wsum += exp(-(dist * dist) / two_s2);  // eval_iou_noise.py:205
      }
    }
    __syncthreads();
  }
  // fixed-order block reduction: lanes (shuffle tree) then waves 0..3
  long long v5[5] = {inter, uni, ga, pa, far};
#pragma unroll
  for (int k = 0; k < 5; ++k)
    for (int o = 32; o > 0; o >>= 1) v5[k] += __shfl_xor(v5[k], o, 64);
  for (int o = 32; o > 0; o >>= 1) wsum += __shfl_xor(wsum, o, 64);
  if ((tid & 63) == 0) {
#pragma unroll
    for (int k = 0; k < 5; ++k) cnt_s[tid >> 6][k] = v5[k];
    wsum_s[tid >> 6] = wsum;
  }
  __syncthreads();
  if (tid == 0) {
    long long c[5];
    for (int k = 0; k < 5; ++k) c[k] = (cnt_s[0][k] + cnt_s[1][k]) + (cnt_s[2][k] + cnt_s[3][k]);
    const double ws = (wsum_s[0] + wsum_s[1]) + (wsum_s[2] + wsum_s[3]);
    const long long I = c[0], U = c[1], G = c[2], P = c[3], F = c[4];
    double* o = p.out + (size_t)n * EV_NOUT;
    o[0] = U > 0 ? (double)I / (double)U : 1.0;          // iou (both empty => 1)
    o[1] = G > 0 ? (double)I / (double)G : 1.0;          // gt_iou
    o[2] = P > 0 ? (double)F / (double)P : 0.0;          // far_noise_ratio
    o[3] = G > 0 ? ws / (double)G : 1.0;                 // gauss_recall
    o[4] = (double)I;
    o[5] = (double)U;
    o[6] = (double)G;
    o[7] = (double)P;
    o[8] = (double)(P - I);                              // fp = pred & !gt
  }
}

}  // namespace dmx
