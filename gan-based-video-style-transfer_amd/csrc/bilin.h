// Bilinear sample geometry of the reference warp (utils/flowtools.py:18-32, F.grid_sample bilinear,
// zeros padding), shared by the warp kernels (flow.hip) and the deterministic warp backward
// (flow_det.hip).  Included after `#pragma clang fp contract(off)`: every rounding step is spelled out.
#pragma once
#include "common.h"

namespace vst {

struct Bilin {
  int x0, y0;
  float nw, ne, sw, se;
};

__device__ __forceinline__ float src_index(float g, int size, int align) {
  // ATen's grid-sampler unnormalize: (g + 1) * ((size - 1) / 2), resp. fma(g + 1, size / 2, -0.5)
  return align ? (g + 1.f) * ((float)(size - 1) * 0.5f) : fmaf(g + 1.f, (float)size * 0.5f, -0.5f);
}

// bilinear combination of the four corner values in ATen's order (an fma chain)
__device__ __forceinline__ float bilerp(float v_nw, float v_ne, float v_sw, float v_se, float nw, float ne,
                                        float sw, float se) {
  return fmaf(v_se, se, fmaf(v_sw, sw, fmaf(v_ne, ne, v_nw * nw)));
}

// sample position for output pixel (h, w) displaced by (fx, fy), reference normalisation
__device__ __forceinline__ Bilin bilin(int h, int w, float fx, float fy, int H, int W, int align) {
  const float vx = (float)w + fx, vy = (float)h + fy;
  const float gx = 2.0f * vx / (float)max(W - 1, 1) - 1.0f;
  const float gy = 2.0f * vy / (float)max(H - 1, 1) - 1.0f;
  const float ix = src_index(gx, W, align), iy = src_index(gy, H, align);
  const float fx0 = floorf(ix), fy0 = floorf(iy);
  const float we = ix - fx0, wn = iy - fy0;  // distance to west / north side
  const float e = 1.f - we, s = 1.f - wn;
  Bilin b;
  b.x0 = (int)fx0;
  b.y0 = (int)fy0;
  b.nw = s * e;
  b.ne = s * we;
  b.sw = wn * e;
  b.se = wn * we;
  return b;
}

__device__ __forceinline__ bool inb(int y, int x, int H, int W) {
  return (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
}

template <typename F>
__device__ __forceinline__ void for_corners(const Bilin& b, int H, int W, F f) {
  if (inb(b.y0, b.x0, H, W)) f(b.y0, b.x0, b.nw);
  if (inb(b.y0, b.x0 + 1, H, W)) f(b.y0, b.x0 + 1, b.ne);
  if (inb(b.y0 + 1, b.x0, H, W)) f(b.y0 + 1, b.x0, b.sw);
  if (inb(b.y0 + 1, b.x0 + 1, H, W)) f(b.y0 + 1, b.x0 + 1, b.se);
}

// fs_lib.warp validity (methods/learning-based/fs_lib.py:33-39): grid_sample of a ones image with
// the same grid, i.e. the in-bounds corner weights summed in nw, ne, sw, se order; the sample is
// kept iff that sum >= 0.9999 (mask < 0.9999 -> 0, mask > 0 -> 1).
__device__ __forceinline__ bool warp_valid(const Bilin& b, int H, int W) {
  float m = 0.f;
  m += inb(b.y0, b.x0, H, W) ? b.nw : 0.f;
  m += inb(b.y0, b.x0 + 1, H, W) ? b.ne : 0.f;
  m += inb(b.y0 + 1, b.x0, H, W) ? b.sw : 0.f;
  m += inb(b.y0 + 1, b.x0 + 1, H, W) ? b.se : 0.f;
  return !(m < 0.9999f) && m > 0.f;
}

}  // namespace vst
