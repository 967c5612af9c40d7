// Optical-flow warp, forward/backward consistency mask and the fused temporal loss.
//
// warp: utils/flowtools.py:18-32 and its inline copy in
// methods/GAN-based/CycleGANCon/models/cycle_gan_model.py:191-203 — F.grid_sample(x, grid),
// bilinear, zeros padding, with the pixel grid normalised by max(W-1,1) / max(H-1,1) and sampled
// with align_corners=False.  Arithmetic follows PyTorch's CPU grid sampler
// (floor, distances to the far side, nw/ne/sw/se weights, sum in that order).
// fbcheck: utils/flowtools.py:34-58 fbcCheckTorch (+ gradient 12-16).
// The data-plane is HBM-bound: one pass reads each pixel's flow once, gathers 4 corner vectors of
// the image (NHWC, one 16-byte load per corner for 3-channel images stored as NHWC4) and writes
// the result; the backward scatters with fp32 atomics into the zero-initialised input gradient.
#include "common.h"

// No implicit a*b+c -> fma contraction in this file: every rounding step is spelled out to match
// the reference's PyTorch CPU kernels bit for bit (tests/golden/warp.npz, fbc.npz were written by
// the reference itself).  Those kernels are built with FMA contraction, so where they fuse we fuse
// explicitly: the source index is fma(g + 1, size / 2, -0.5), the bilinear sample is the fma chain
// nw -> ne -> sw -> se, a 2-vector squared norm is fma(q, q, p*p); everything else (grid
// normalisation, weights, thresholds, which PyTorch evaluates as separate tensor ops) rounds each
// operation on its own.
#pragma clang fp contract(off)
#include "bilin.h"

namespace vst {

// out (NHWC, Cs channels, processed 4 at a time) = warp(x, flow) (MASKED: * fs_lib validity mask).
// Grid (ceil(W*C4 / 256), H, N): image and row come from the block index and the thread's pixel and
// channel chunk from a 32-bit split of its row offset (CT = C4 at compile time for the common widths,
// 0 = runtime), so no thread pays 64-bit divisions; a row's threads read its flow values once per
// pixel (broadcast within the pixel's C4 lanes) and gather each corner as C4 contiguous float4s.
template <int MASKED, int CT>
__global__ __launch_bounds__(256) void warp_fwd_k(const float* __restrict__ x, const float* __restrict__ flow,
                                                  float* __restrict__ out, int N, int H, int W, int C4_, int align) {
  const int C4 = CT ? CT : C4_;
  const int local = blockIdx.x * 256 + threadIdx.x;
  if (local >= W * C4) return;
  const int h = blockIdx.y, n = blockIdx.z;
  const int w = CT == 1 ? local : local / C4, c4 = CT == 1 ? 0 : local - w * C4;
  const long plane = (long)H * W;
  const long fo = (long)n * 2 * plane + (long)h * W + w;
  const Bilin b = bilin(h, w, flow[fo], flow[fo + plane], H, W, align);
  float4* op = reinterpret_cast<float4*>(out) + ((long)n * plane + (long)h * W) * C4 + local;
  if (MASKED && !warp_valid(b, H, W)) {
    *op = make_float4(0.f, 0.f, 0.f, 0.f);
    return;
  }
  const float4* xs = reinterpret_cast<const float4*>(x) + (long)n * plane * C4 + c4;
  float4 v_nw = make_float4(0, 0, 0, 0), v_ne = v_nw, v_sw = v_nw, v_se = v_nw;
  const int r0 = b.y0 * W, r1 = r0 + W;
  if (inb(b.y0, b.x0, H, W)) v_nw = xs[(long)(r0 + b.x0) * C4];
  if (inb(b.y0, b.x0 + 1, H, W)) v_ne = xs[(long)(r0 + b.x0 + 1) * C4];
  if (inb(b.y0 + 1, b.x0, H, W)) v_sw = xs[(long)(r1 + b.x0) * C4];
  if (inb(b.y0 + 1, b.x0 + 1, H, W)) v_se = xs[(long)(r1 + b.x0 + 1) * C4];
  float4 o;
  o.x = bilerp(v_nw.x, v_ne.x, v_sw.x, v_se.x, b.nw, b.ne, b.sw, b.se);
  o.y = bilerp(v_nw.y, v_ne.y, v_sw.y, v_se.y, b.nw, b.ne, b.sw, b.se);
  o.z = bilerp(v_nw.z, v_ne.z, v_sw.z, v_se.z, b.nw, b.ne, b.sw, b.se);
  o.w = bilerp(v_nw.w, v_ne.w, v_sw.w, v_se.w, b.nw, b.ne, b.sw, b.se);
  *op = o;
}

template <int MASKED>
static int warp_fwd_launch(const float* x, const float* flow, float* out, int N, int H, int W, int Cs, int align,
                           hipStream_t s) {
  VST_REQUIRE(H <= 65535 && N <= 65535 && (long)W * (Cs / 4) < (1L << 31), "warp_fwd: grid too large");
  const int C4 = Cs / 4;
  const dim3 grid(ceil_div((long)W * C4, 256), H, N);
#define VST_WARP(CT) hipLaunchKernelGGL((warp_fwd_k<MASKED, CT>), grid, dim3(256), 0, s, x, flow, out, N, H, W, C4, align)
  if (C4 == 1) VST_WARP(1);
  else if (C4 == 16) VST_WARP(16);
  else if (C4 == 32) VST_WARP(32);
  else VST_WARP(0);
#undef VST_WARP
  return VST_OK;
}

template <int MASKED>
__global__ void warp_bwd_k(const float* __restrict__ gout, const float* __restrict__ flow,
                           float* __restrict__ gx, int N, int H, int W, int Cs, int align) {
  const long total = (long)N * H * W;
  const long pix = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= total) return;
  const int w = pix % W, h = (pix / W) % H, n = pix / ((long)W * H);
  const long fo = (long)n * 2 * H * W + (long)h * W + w;
  const Bilin b = bilin(h, w, flow[fo], flow[fo + (long)H * W], H, W, align);
  if (MASKED && !warp_valid(b, H, W)) return;
  const float* g = gout + pix * Cs;
  float* base = gx + (long)n * H * W * Cs;
  for_corners(b, H, W, [&](int y, int xx, float wt) {
    float* d = base + ((long)y * W + xx) * Cs;
    for (int c = 0; c < Cs; ++c) atomicAdd(d + c, wt * g[c]);
  });
}

// Fused temporal loss: per pixel e_c = mask * (b_c - warp(a)_c); partial sums of e^2 per block.
// With grads: gb = k * mask * e, ga += scatter(-k * mask * e), k = 2 * lambda * gout / count.
__global__ void temporal_k(const float* __restrict__ a, const float* __restrict__ bimg,
                           const float* __restrict__ flow, const float* __restrict__ mask,
                           float* __restrict__ part, float* __restrict__ ga, float* __restrict__ gb,
                           const float* __restrict__ gout, float kscale, int N, int H, int W, int Cs,
                           int Cl) {
  __shared__ float red[4];
  const long total = (long)N * H * W;
  const long pix = (long)blockIdx.x * blockDim.x + threadIdx.x;
  float acc = 0.f;
  if (pix < total) {
    const int w = pix % W, h = (pix / W) % H, n = pix / ((long)W * H);
    const long fo = (long)n * 2 * H * W + (long)h * W + w;
    const Bilin b = bilin(h, w, flow[fo], flow[fo + (long)H * W], H, W, 0);
    const float m = mask[pix];
    const float* an = a + (long)n * H * W * Cs;
    const float k = gout ? kscale * gout[0] : 0.f;
    for (int c = 0; c < Cl; ++c) {
      float v_nw = 0.f, v_ne = 0.f, v_sw = 0.f, v_se = 0.f;
      if (inb(b.y0, b.x0, H, W)) v_nw = an[((long)b.y0 * W + b.x0) * Cs + c];
      if (inb(b.y0, b.x0 + 1, H, W)) v_ne = an[((long)b.y0 * W + b.x0 + 1) * Cs + c];
      if (inb(b.y0 + 1, b.x0, H, W)) v_sw = an[((long)(b.y0 + 1) * W + b.x0) * Cs + c];
      if (inb(b.y0 + 1, b.x0 + 1, H, W)) v_se = an[((long)(b.y0 + 1) * W + b.x0 + 1) * Cs + c];
      const float wv = bilerp(v_nw, v_ne, v_sw, v_se, b.nw, b.ne, b.sw, b.se);
      const float e = m * (bimg[pix * Cs + c] - wv);
      acc += e * e;
      if (gout) {
        const float gbv = k * m * e;
        if (gb) gb[pix * Cs + c] = gbv;
        if (ga) {
          float* d = ga + (long)n * H * W * Cs + c;
          for_corners(b, H, W, [&](int y, int xx, float wt) { atomicAdd(d + ((long)y * W + xx) * Cs, -wt * gbv); });
        }
      }
    }
    if (gout && gb)
      for (int c = Cl; c < Cs; ++c) gb[pix * Cs + c] = 0.f;
  }
  if (part) {
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
  }
}

// fixed-order final reduction: out[0] = scale * sum(part[0..n)) / count
__global__ void finish_sum_k(const float* __restrict__ part, int n, float* __restrict__ out,
                             double scale) {
  __shared__ double red[4];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) s += part[i];
  s = wave_sum_d(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = (float)((red[0] + red[1] + red[2] + red[3]) * scale);
}

__global__ void fbcheck_k(const float* __restrict__ ff, const float* __restrict__ bf,
                          float* __restrict__ mask, int N, int H, int W) {
  const long total = (long)N * H * W;
  const long pix = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= total) return;
  const int w = pix % W, h = (pix / W) % H, n = pix / ((long)W * H);
  const long plane = (long)H * W;
  const float* u = bf + n * 2 * plane;   // bf x-component
  const float* v = u + plane;            // bf y-component
  const float* f0 = ff + n * 2 * plane;
  const float* f1 = f0 + plane;
  const long o = (long)h * W + w;
  const float bu = u[o], bv = v[o];
  const Bilin b = bilin(h, w, bu, bv, H, W, 0);
  float w0 = 0.f, w1 = 0.f;
  {
    float a_nw = 0, a_ne = 0, a_sw = 0, a_se = 0, c_nw = 0, c_ne = 0, c_sw = 0, c_se = 0;
    if (inb(b.y0, b.x0, H, W)) { a_nw = f0[(long)b.y0 * W + b.x0]; c_nw = f1[(long)b.y0 * W + b.x0]; }
    if (inb(b.y0, b.x0 + 1, H, W)) { a_ne = f0[(long)b.y0 * W + b.x0 + 1]; c_ne = f1[(long)b.y0 * W + b.x0 + 1]; }
    if (inb(b.y0 + 1, b.x0, H, W)) { a_sw = f0[(long)(b.y0 + 1) * W + b.x0]; c_sw = f1[(long)(b.y0 + 1) * W + b.x0]; }
    if (inb(b.y0 + 1, b.x0 + 1, H, W)) { a_se = f0[(long)(b.y0 + 1) * W + b.x0 + 1]; c_se = f1[(long)(b.y0 + 1) * W + b.x0 + 1]; }
    w0 = bilerp(a_nw, a_ne, a_sw, a_se, b.nw, b.ne, b.sw, b.se);
    w1 = bilerp(c_nw, c_ne, c_sw, c_se, b.nw, b.ne, b.sw, b.se);
  }
  // torch.norm(., dim=1)**2 : sqrt of the sum of squares (ATen's fused reduction), then squared
  auto n2 = [](float p, float q) { const float r = sqrtf(fmaf(q, q, p * p)); return r * r; };
  const float nwb = n2(w0 + bu, w1 + bv);
  const float nw_ = n2(w0, w1);
  const float nb = n2(bu, bv);
  const bool occ = nwb > 0.01f * (nw_ + nb) + 0.5f;
  // zero-padded central differences / 2 (flowtools.gradient)
  auto at = [&](const float* f, int y, int x) { return inb(y, x, H, W) ? f[(long)y * W + x] : 0.f; };
  const float ux = (at(u, h, w + 1) - at(u, h, w - 1)) / 2, uy = (at(u, h + 1, w) - at(u, h - 1, w)) / 2;
  const float vx = (at(v, h, w + 1) - at(v, h, w - 1)) / 2, vy = (at(v, h + 1, w) - at(v, h - 1, w)) / 2;
  const bool mob = n2(ux, uy) + n2(vx, vy) > 0.01f * nb + 0.002f;
  mask[pix] = (occ || mob) ? 0.f : 1.f;
}

}  // namespace vst

using namespace vst;

extern "C" int vst_warp_fwd(const float* x, const float* flow, float* out, int N, int H, int W,
                            int Cs, int align_corners, void* stream) {
  VST_REQUIRE(x && flow && out && Cs % 4 == 0 && N > 0 && H > 0 && W > 0, "warp_fwd: bad args");
  if (int e = warp_fwd_launch<0>(x, flow, out, N, H, W, Cs, align_corners, (hipStream_t)stream)) return e;
  return check_launch("warp_fwd");
}

extern "C" int vst_warp_masked_fwd(const float* x, const float* flow, float* out, int N, int H, int W,
                                   int Cs, int align_corners, void* stream) {
  VST_REQUIRE(x && flow && out && Cs % 4 == 0 && N > 0 && H > 0 && W > 0, "warp_masked_fwd: bad args");
  if (int e = warp_fwd_launch<1>(x, flow, out, N, H, W, Cs, align_corners, (hipStream_t)stream)) return e;
  return check_launch("warp_masked_fwd");
}

extern "C" int vst_warp_bwd_input(const float* gout, const float* flow, float* gx, int N, int H,
                                  int W, int Cs, int align_corners, void* stream) {
  VST_REQUIRE(gout && flow && gx && Cs > 0, "warp_bwd_input: bad args");
  const long total = (long)N * H * W;
  hipLaunchKernelGGL(warp_bwd_k<0>, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, gout,
                     flow, gx, N, H, W, Cs, align_corners);
  return check_launch("warp_bwd_input");
}

extern "C" int vst_warp_masked_bwd_input(const float* gout, const float* flow, float* gx, int N, int H,
                                         int W, int Cs, int align_corners, void* stream) {
  VST_REQUIRE(gout && flow && gx && Cs > 0, "warp_masked_bwd_input: bad args");
  const long total = (long)N * H * W;
  hipLaunchKernelGGL(warp_bwd_k<1>, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, gout,
                     flow, gx, N, H, W, Cs, align_corners);
  return check_launch("warp_masked_bwd_input");
}

extern "C" int vst_fbcheck(const float* ff, const float* bf, float* mask, int N, int H, int W,
                           void* stream) {
  VST_REQUIRE(ff && bf && mask && N > 0 && H > 0 && W > 0, "fbcheck: bad args");
  const long total = (long)N * H * W;
  hipLaunchKernelGGL(fbcheck_k, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, ff, bf,
                     mask, N, H, W);
  return check_launch("fbcheck");
}

extern "C" int vst_loss_part_floats(long n) { return ceil_div(n, 256) + 1; }

extern "C" int vst_loss_temporal(const float* a, const float* b, const float* flow,
                                 const float* mask, float* loss, float* part, int N, int H, int W,
                                 int Cs, int Cl, float lambda, void* stream) {
  VST_REQUIRE(a && b && flow && mask && loss && part && Cl <= Cs, "loss_temporal: bad args");
  hipStream_t s = (hipStream_t)stream;
  const long total = (long)N * H * W;
  const int nb = ceil_div(total, 256);
  hipLaunchKernelGGL(temporal_k, dim3(nb), dim3(256), 0, s, a, b, flow, mask, part, (float*)nullptr,
                     (float*)nullptr, (const float*)nullptr, 0.f, N, H, W, Cs, Cl);
  hipLaunchKernelGGL(finish_sum_k, dim3(1), dim3(256), 0, s, part, nb, loss,
                     (double)lambda / ((double)total * Cl));
  return check_launch("loss_temporal");
}

extern "C" int vst_loss_temporal_bwd(const float* a, const float* b, const float* flow,
                                     const float* mask, const float* gout, float* ga, float* gb,
                                     int N, int H, int W, int Cs, int Cl, float lambda,
                                     void* stream) {
  VST_REQUIRE(a && b && flow && mask && gout && (ga || gb) && Cl <= Cs, "loss_temporal_bwd: bad args");
  const long total = (long)N * H * W;
  const float k = (float)(2.0 * lambda / ((double)total * Cl));
  hipLaunchKernelGGL(temporal_k, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, a, b,
                     flow, mask, (float*)nullptr, ga, gb, gout, k, N, H, W, Cs, Cl);
  return check_launch("loss_temporal_bwd");
}

extern "C" int vst_finish_sum(const float* part, int n, float* out, double scale, void* stream) {
  hipLaunchKernelGGL(finish_sum_k, dim3(1), dim3(256), 0, (hipStream_t)stream, part, n, out, scale);
  return check_launch("finish_sum");
}
