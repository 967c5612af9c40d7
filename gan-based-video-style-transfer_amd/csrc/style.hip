// Kernels of the perceptual / learning-based style path and the RAFT correlation pyramid
// (SURVEY §8 rows A17-A19, A21):
//   channel normalise      fast_style_transfer.py:819-822 normalize ((img - mean) / std), with the
//                          fs_johnson.py:31 `/ 255` folded in as a pre-divisor
//   nearest 2x upsample    network.py:206-207 F.interpolate(scale_factor=2) (UpsampleConvLayer)
//   scaled tanh            network.py:111-118 ConvTanh: tanh(x / 255) * 150 + 255 / 2
//   2x2 max pool           torchvision VGG MaxPool2d(2, 2) inside network.py:45-78 (Vgg16/Vgg19)
//   TV loss                fast_style_transfer.py:795-803 calc_tv_loss
//   MSE(a, b)              nn.MSELoss (content loss fs_johnson.py:37, Gram style loss :41)
//   Gram symmetrise        backward of fast_style_transfer.py:813-817 gram_matrix (bmm(F,F^T)/hw)
//   avg-pool pyramid       utils/raft/raft/corr.py:24-26 F.avg_pool2d(corr, 2, stride=2)
//   window lookup          utils/raft/raft/corr.py:29-51 + utils/utils.py:57-71 bilinear_sampler
//                          (align_corners=True, zeros padding, meshgrid(dy, dx) window order)
// All are HBM-bound streams over NHWC fp32 tensors (float4 rows where the layout allows).
#include "common.h"

namespace vst {

// y = ((x / d0) - mean[c]) / std[c] on the Cl logical channels; padding channels are written 0.
// backward (BWD=1): gx = (gy / std[c]) / d0.
template <int BWD>
__global__ void chnorm_k(const float* __restrict__ x, float* __restrict__ y,
                         const float* __restrict__ mean, const float* __restrict__ stdv, float d0,
                         long total, int Cs, int Cl) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = i % Cs;
  float v = 0.f;
  if (c < Cl) v = BWD ? (x[i] / stdv[c]) / d0 : ((x[i] / d0) - (mean ? mean[c] : 0.f)) / stdv[c];
  y[i] = v;
}

// nearest 2x upsample, NHWC float4 rows: y[n][oh][ow] = x[n][oh/2][ow/2]
__global__ void up2_fwd_k(const float4* __restrict__ x, float4* __restrict__ y, int N, int H, int W,
                          int C4) {
  const long total = (long)N * 4 * H * W * C4;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c4 = i % C4;
  const long pix = i / C4;
  const int ow = pix % (2 * W), oh = (pix / (2 * W)) % (2 * H), n = pix / (4L * H * W);
  y[i] = x[(((long)n * H + (oh >> 1)) * W + (ow >> 1)) * C4 + c4];
}

// backward: gx[h][w] = g[2h][2w] + g[2h][2w+1] + g[2h+1][2w] + g[2h+1][2w+1] (output scan order)
__global__ void up2_bwd_k(const float4* __restrict__ g, float4* __restrict__ gx, int N, int H, int W,
                          int C4) {
  const long total = (long)N * H * W * C4;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c4 = i % C4;
  const long pix = i / C4;
  const int w = pix % W, h = (pix / W) % H, n = pix / ((long)H * W);
  const long r0 = (((long)n * 2 * H + 2 * h) * 2 * W + 2 * w) * C4 + c4;
  const long r1 = r0 + 2L * W * C4;
  float4 a = g[r0];
  add_f4(a, g[r0 + C4]);
  add_f4(a, g[r1]);
  add_f4(a, g[r1 + C4]);
  gx[i] = a;
}

// ConvTanh epilogue: y = tanh(x / 255) * 150 + 127.5 (logical channels; padding channels 0).
// BWD: gx = ((gy * 150) * (1 - t^2)) / 255, t = tanh(x / 255) recomputed from the saved x.
template <int BWD>
__global__ void stanh_k(const float* __restrict__ x, const float* __restrict__ gy,
                        float* __restrict__ y, long total, int Cs, int Cl) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = i % Cs;
  float v = 0.f;
  if (c < Cl) {
    const float t = tanhf(x[i] / 255.f);
    v = BWD ? ((gy[i] * 150.f) * (1.f - t * t)) / 255.f : t * 150.f + 127.5f;
  }
  y[i] = v;
}

// MaxPool2d(2, 2), floor mode, NHWC float4.  The window is scanned (0,0),(0,1),(1,0),(1,1) and a
// later element wins only if strictly greater (or NaN), as ATen's CPU max_pool2d.
__device__ __forceinline__ void mp_pick(float v, int k, float& m, int& am) {
  if (v > m || isnan(v)) { m = v; am = k; }
}

__global__ void maxpool2_fwd_k(const float* __restrict__ x, float* __restrict__ y, int N, int H,
                               int W, int Cs) {
  const int Ho = H / 2, Wo = W / 2;
  const long total = (long)N * Ho * Wo * Cs;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = i % Cs;
  const long pix = i / Cs;
  const int wo = pix % Wo, ho = (pix / Wo) % Ho, n = pix / ((long)Ho * Wo);
  const float* b = x + (((long)n * H + 2 * ho) * W + 2 * wo) * Cs + c;
  float m = b[0];
  int am = 0;
  mp_pick(b[Cs], 1, m, am);
  mp_pick(b[(long)W * Cs], 2, m, am);
  mp_pick(b[(long)W * Cs + Cs], 3, m, am);
  y[i] = m;
}

// one thread per INPUT element: its gradient is gy of its window if it is the window's argmax
__global__ void maxpool2_bwd_k(const float* __restrict__ gy, const float* __restrict__ x,
                               float* __restrict__ gx, int N, int H, int W, int Cs) {
  const int Ho = H / 2, Wo = W / 2;
  const long total = (long)N * H * W * Cs;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = i % Cs;
  const long pix = i / Cs;
  const int w = pix % W, h = (pix / W) % H, n = pix / ((long)H * W);
  const int ho = h >> 1, wo = w >> 1;
  float g = 0.f;
  if (ho < Ho && wo < Wo) {
    const float* b = x + (((long)n * H + 2 * ho) * W + 2 * wo) * Cs + c;
    float m = b[0];
    int am = 0;
    mp_pick(b[Cs], 1, m, am);
    mp_pick(b[(long)W * Cs], 2, m, am);
    mp_pick(b[(long)W * Cs + Cs], 3, m, am);
    if (am == (h & 1) * 2 + (w & 1)) g = gy[(((long)n * Ho + ho) * Wo + wo) * Cs + c];
  }
  gx[i] = g;
}

// ---- MSE between two tensors (logical channels), partial sums + fixed-order finish ----------
__global__ void mse2_part_k(const float* __restrict__ a, const float* __restrict__ b,
                            float* __restrict__ part, long npix, int Cs, int Cl) {
  __shared__ float red[4];
  const long pix = (long)blockIdx.x * blockDim.x + threadIdx.x;
  float acc = 0.f;
  if (pix < npix)
    for (int c = 0; c < Cl; ++c) {
      const float d = a[pix * Cs + c] - b[pix * Cs + c];
      acc += d * d;
    }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// grad = k * gout * 2 (a - b) (padding channels 0); written or accumulated
__global__ void mse2_grad_k(const float* __restrict__ a, const float* __restrict__ b,
                            const float* __restrict__ gout, float k, float* __restrict__ grad,
                            long total, int Cs, int Cl, int accumulate) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = i % Cs;
  float g = 0.f;
  if (c < Cl) g = k * gout[0] * 2.f * (a[i] - b[i]);
  grad[i] = accumulate ? grad[i] + g : g;
}

// ---- total variation (calc_tv_loss) on NHWC images -----------------------------------------
__device__ __forceinline__ float tv_at(const float* __restrict__ I, int n, int y, int x, int H, int W,
                                       int Cs, int Cl, float* d1, float* d2) {
  const float* p = I + (((long)n * H + y) * W + x) * Cs;
  float s1 = 0.f, s2 = 0.f;
  for (int c = 0; c < Cl; ++c) {
    const float a = p[(long)W * Cs + c] - p[c];  // I[y+1][x] - I[y][x]
    const float b = p[Cs + c] - p[c];            // I[y][x+1] - I[y][x]
    if (d1) { d1[c] = a; d2[c] = b; }
    s1 += a * a;
    s2 += b * b;
  }
  // torch.norm(., dim=1) ** 2 then (tv1 + tv2) ** 0.5
  const float n1 = sqrtf(s1), n2 = sqrtf(s2);
  return sqrtf(n1 * n1 + n2 * n2);
}

__global__ void tv_part_k(const float* __restrict__ I, float* __restrict__ part, int N, int H, int W,
                          int Cs, int Cl) {
  __shared__ float red[4];
  const long total = (long)N * (H - 1) * (W - 1);
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  float acc = 0.f;
  if (i < total) {
    const int x = i % (W - 1), y = (i / (W - 1)) % (H - 1), n = i / ((long)(H - 1) * (W - 1));
    acc = tv_at(I, n, y, x, H, W, Cs, Cl, nullptr, nullptr);
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// gather-form backward: pixel (y,x) collects -(d1+d2)/r of its own term, +d1/r of the term above
// and +d2/r of the term to its left.  r == 0 terms contribute 0.
__global__ void tv_grad_k(const float* __restrict__ I, const float* __restrict__ gout, float scale,
                          float* __restrict__ grad, int N, int H, int W, int Cs, int Cl) {
  const long total = (long)N * H * W;
  const long pix = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= total) return;
  const int x = pix % W, y = (pix / W) % H, n = pix / ((long)H * W);
  const float k = scale * gout[0];
  float g[4] = {0.f, 0.f, 0.f, 0.f};
  float d1[4], d2[4];
  if (y < H - 1 && x < W - 1) {
    const float r = tv_at(I, n, y, x, H, W, Cs, Cl, d1, d2);
    if (r > 0.f)
      for (int c = 0; c < Cl; ++c) g[c] -= k * (d1[c] + d2[c]) / r;
  }
  if (y > 0 && x < W - 1) {
    const float r = tv_at(I, n, y - 1, x, H, W, Cs, Cl, d1, d2);
    if (r > 0.f)
      for (int c = 0; c < Cl; ++c) g[c] += k * d1[c] / r;
  }
  if (x > 0 && y < H - 1) {
    const float r = tv_at(I, n, y, x - 1, H, W, Cs, Cl, d1, d2);
    if (r > 0.f)
      for (int c = 0; c < Cl; ++c) g[c] += k * d2[c] / r;
  }
  float* o = grad + pix * Cs;
  for (int c = 0; c < Cs; ++c) o[c] = c < Cl ? g[c] : 0.f;
}

// S[i][j] = (dG[i][j] + dG[j][i]) * scale — the 1x1-conv weight of the Gram backward
__global__ void gram_sym_k(const float* __restrict__ dG, float* __restrict__ S, int C, float scale) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)C * C) return;
  const int r = i / C, c = i % C;
  S[i] = (dG[i] + dG[(long)c * C + r]) * scale;
}

// ---- RAFT correlation pyramid ----------------------------------------------------------------
// level l+1 = avg_pool2d(level l, 2, 2) over each of P planes (floor mode); sum order as ATen CPU
// ((x00 + x01) + x10) + x11, then / 4.
__global__ void avgpool2_planes_k(const float* __restrict__ x, float* __restrict__ y, long P, int H,
                                  int W, long ldx, long ldy) {
  const int Ho = H / 2, Wo = W / 2;
  const long total = P * Ho * Wo;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int wo = i % Wo, ho = (i / Wo) % Ho;
  const long p = i / ((long)Ho * Wo);
  const float* b = x + p * ldx + (long)(2 * ho) * W + 2 * wo;
  float s = b[0];
  s += b[1];
  s += b[W];
  s += b[W + 1];
  y[p * ldy + (long)ho * Wo + wo] = s / 4.f;
}

// out[b][h][w][lvl*(2r+1)^2 + a*(2r+1) + c] = bilinear(level lvl of plane (b,h,w),
//    x = cx/2^lvl + (a - r), y = cy/2^lvl + (c - r)), align_corners=True, zeros outside.
// One thread per output element; the plane's window is L2-resident across the 81 threads of a pixel.
struct PyrGeom {
  long off[9];
  int hw[24];  // (h, w) per level, then the plane stride per level
};

__global__ void corr_lookup_k(const float* __restrict__ pyr, const PyrGeom geo,
                              const float* __restrict__ coords,
                              float* __restrict__ out, int B, int H1, int W1, int levels, int r,
                              int Cs) {
  const int K = 2 * r + 1, KK = K * K;
  const long total = (long)B * H1 * W1 * Cs;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int ch = i % Cs;
  const long pix = i / Cs;
  if (ch >= levels * KK) { out[i] = 0.f; return; }
  const int lvl = ch / KK, q = ch % KK, a = q / K, c = q % K;
  const int w = pix % W1, h = (pix / W1) % H1, b = pix / ((long)H1 * W1);
  const float cx = coords[(((long)b * 2) * H1 + h) * W1 + w];
  const float cy = coords[(((long)b * 2 + 1) * H1 + h) * W1 + w];
  const float div = (float)(1 << lvl);
  const int Hl = geo.hw[2 * lvl], Wl = geo.hw[2 * lvl + 1];
  const float px = cx / div + (float)(a - r), py = cy / div + (float)(c - r);
  // bilinear_sampler: normalise by (size-1), then grid_sample(align_corners=True) unnormalises
  const float gx = 2.f * px / (float)(Wl - 1) - 1.f, gy = 2.f * py / (float)(Hl - 1) - 1.f;
  const float ix = ((gx + 1.f) / 2.f) * (float)(Wl - 1), iy = ((gy + 1.f) / 2.f) * (float)(Hl - 1);
  const float fx0 = floorf(ix), fy0 = floorf(iy);
  const int x0 = (int)fx0, y0 = (int)fy0;
  const float we = ix - fx0, wn = iy - fy0, e = 1.f - we, s = 1.f - wn;
  const long ld = geo.hw[2 * levels + lvl];
  const float* pl = pyr + geo.off[lvl] + pix * ld;
  auto at = [&](int yy, int xx) {
    return ((unsigned)yy < (unsigned)Hl && (unsigned)xx < (unsigned)Wl) ? pl[(long)yy * Wl + xx] : 0.f;
  };
  out[i] = at(y0, x0) * (s * e) + at(y0, x0 + 1) * (s * we) + at(y0 + 1, x0) * (wn * e) +
           at(y0 + 1, x0 + 1) * (wn * we);
}

__global__ void finish_sum3_k(const float* __restrict__ part, int n, float* __restrict__ out,
                              double scale, int accumulate) {
  __shared__ double red[4];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) s += part[i];
  s = wave_sum_d(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float v = (float)((red[0] + red[1] + red[2] + red[3]) * scale);
    out[0] = accumulate ? out[0] + v : v;
  }
}


// StarGAN Generator.forward (model.py:59-64): cat([x, c replicated over H, W], dim=1) written as
// NHWC with channel stride Cs: y[n][h][w] = {x[n][0..Cx)[h][w], c[n][0..Cl), 0...}
__global__ void concat_label_k(const float* __restrict__ x, const float* __restrict__ lab,
                               float* __restrict__ y, int N, int Cx, int Cl, int H, int W, int Cs) {
  const long total = (long)N * H * W * Cs;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = i % Cs;
  const long pix = i / Cs;
  const int w = pix % W, h = (pix / W) % H, n = pix / ((long)H * W);
  float v = 0.f;
  if (c < Cx) v = x[(((long)n * Cx + c) * H + h) * W + w];
  else if (c < Cx + Cl) v = lab[(long)n * Cl + (c - Cx)];
  y[i] = v;
}

}  // namespace vst

using namespace vst;

static inline dim3 grid1(long n) { return dim3(ceil_div(n, 256)); }

extern "C" int vst_channel_normalize(const float* x, float* y, const float* mean, const float* stdv,
                                     float d0, long npix, int Cs, int Cl, int backward,
                                     void* stream) {
  VST_REQUIRE(x && y && stdv && Cl <= Cs && npix >= 0 && d0 != 0.f, "channel_normalize: bad args");
  const long total = npix * Cs;
  if (total == 0) return VST_OK;
  if (backward)
    hipLaunchKernelGGL(chnorm_k<1>, grid1(total), dim3(256), 0, (hipStream_t)stream, x, y, mean, stdv,
                       d0, total, Cs, Cl);
  else
    hipLaunchKernelGGL(chnorm_k<0>, grid1(total), dim3(256), 0, (hipStream_t)stream, x, y, mean, stdv,
                       d0, total, Cs, Cl);
  return check_launch("channel_normalize");
}

extern "C" int vst_upsample2x_fwd(const float* x, float* y, int N, int H, int W, int Cs, void* stream) {
  VST_REQUIRE(x && y && Cs % 4 == 0 && N > 0 && H > 0 && W > 0, "upsample2x_fwd: bad args");
  const long total = (long)N * 4 * H * W * (Cs / 4);
  hipLaunchKernelGGL(up2_fwd_k, grid1(total), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const float4*>(x), reinterpret_cast<float4*>(y), N, H, W, Cs / 4);
  return check_launch("upsample2x_fwd");
}

extern "C" int vst_upsample2x_bwd(const float* gy, float* gx, int N, int H, int W, int Cs, void* stream) {
  VST_REQUIRE(gy && gx && Cs % 4 == 0 && N > 0 && H > 0 && W > 0, "upsample2x_bwd: bad args");
  const long total = (long)N * H * W * (Cs / 4);
  hipLaunchKernelGGL(up2_bwd_k, grid1(total), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const float4*>(gy), reinterpret_cast<float4*>(gx), N, H, W, Cs / 4);
  return check_launch("upsample2x_bwd");
}

extern "C" int vst_scaled_tanh_fwd(const float* x, float* y, long npix, int Cs, int Cl, void* stream) {
  VST_REQUIRE(x && y && Cl <= Cs, "scaled_tanh_fwd: bad args");
  const long total = npix * Cs;
  if (total == 0) return VST_OK;
  hipLaunchKernelGGL(stanh_k<0>, grid1(total), dim3(256), 0, (hipStream_t)stream, x,
                     (const float*)nullptr, y, total, Cs, Cl);
  return check_launch("scaled_tanh_fwd");
}

extern "C" int vst_scaled_tanh_bwd(const float* x, const float* gy, float* gx, long npix, int Cs,
                                   int Cl, void* stream) {
  VST_REQUIRE(x && gy && gx && Cl <= Cs, "scaled_tanh_bwd: bad args");
  const long total = npix * Cs;
  if (total == 0) return VST_OK;
  hipLaunchKernelGGL(stanh_k<1>, grid1(total), dim3(256), 0, (hipStream_t)stream, x, gy, gx, total, Cs,
                     Cl);
  return check_launch("scaled_tanh_bwd");
}

extern "C" int vst_maxpool2_fwd(const float* x, float* y, int N, int H, int W, int Cs, void* stream) {
  VST_REQUIRE(x && y && N > 0 && H >= 2 && W >= 2 && Cs > 0, "maxpool2_fwd: bad args");
  const long total = (long)N * (H / 2) * (W / 2) * Cs;
  hipLaunchKernelGGL(maxpool2_fwd_k, grid1(total), dim3(256), 0, (hipStream_t)stream, x, y, N, H, W, Cs);
  return check_launch("maxpool2_fwd");
}

extern "C" int vst_maxpool2_bwd(const float* gy, const float* x, float* gx, int N, int H, int W, int Cs,
                                void* stream) {
  VST_REQUIRE(gy && x && gx && N > 0 && H >= 2 && W >= 2 && Cs > 0, "maxpool2_bwd: bad args");
  const long total = (long)N * H * W * Cs;
  hipLaunchKernelGGL(maxpool2_bwd_k, grid1(total), dim3(256), 0, (hipStream_t)stream, gy, x, gx, N, H, W,
                     Cs);
  return check_launch("maxpool2_bwd");
}

extern "C" int vst_loss_mse(const float* a, const float* b, float* loss, float* part, long npix, int Cs,
                            int Cl, float scale, int accumulate, void* stream) {
  VST_REQUIRE(a && b && loss && part && Cl <= Cs && npix > 0, "loss_mse: bad args");
  hipStream_t s = (hipStream_t)stream;
  const int nb = ceil_div(npix, 256);
  hipLaunchKernelGGL(mse2_part_k, dim3(nb), dim3(256), 0, s, a, b, part, npix, Cs, Cl);
  hipLaunchKernelGGL(finish_sum3_k, dim3(1), dim3(256), 0, s, part, nb, loss,
                     (double)scale / ((double)npix * Cl), accumulate);
  return check_launch("loss_mse");
}

extern "C" int vst_loss_mse_bwd(const float* a, const float* b, const float* gout, float* grad,
                                long npix, int Cs, int Cl, float scale, int accumulate, void* stream) {
  VST_REQUIRE(a && b && gout && grad && Cl <= Cs, "loss_mse_bwd: bad args");
  const float k = (float)((double)scale / ((double)npix * Cl));
  const long total = npix * Cs;
  hipLaunchKernelGGL(mse2_grad_k, grid1(total), dim3(256), 0, (hipStream_t)stream, a, b, gout, k, grad,
                     total, Cs, Cl, accumulate);
  return check_launch("loss_mse_bwd");
}

extern "C" int vst_loss_tv(const float* img, float* loss, float* part, int N, int H, int W, int Cs,
                           int Cl, float scale, int accumulate, void* stream) {
  VST_REQUIRE(img && loss && part && Cl <= Cs && Cl <= 4 && N > 0 && H > 1 && W > 1, "loss_tv: bad args");
  hipStream_t s = (hipStream_t)stream;
  const long total = (long)N * (H - 1) * (W - 1);
  const int nb = ceil_div(total, 256);
  hipLaunchKernelGGL(tv_part_k, dim3(nb), dim3(256), 0, s, img, part, N, H, W, Cs, Cl);
  hipLaunchKernelGGL(finish_sum3_k, dim3(1), dim3(256), 0, s, part, nb, loss, (double)scale, accumulate);
  return check_launch("loss_tv");
}

extern "C" int vst_loss_tv_bwd(const float* img, const float* gout, float* grad, int N, int H, int W,
                               int Cs, int Cl, float scale, void* stream) {
  VST_REQUIRE(img && gout && grad && Cl <= Cs && Cl <= 4 && N > 0 && H > 1 && W > 1, "loss_tv_bwd: bad args");
  const long total = (long)N * H * W;
  hipLaunchKernelGGL(tv_grad_k, grid1(total), dim3(256), 0, (hipStream_t)stream, img, gout, scale, grad,
                     N, H, W, Cs, Cl);
  return check_launch("loss_tv_bwd");
}

extern "C" int vst_gram_sym(const float* dG, float* S, int C, float scale, void* stream) {
  VST_REQUIRE(dG && S && C > 0 && dG != S, "gram_sym: bad args");
  hipLaunchKernelGGL(gram_sym_k, grid1((long)C * C), dim3(256), 0, (hipStream_t)stream, dG, S, C, scale);
  return check_launch("gram_sym");
}

// Pyramid layout (one buffer): level 0 = P planes of H2*W2 values with plane stride ld0 (>= H2*W2,
// the corr GEMM's padded channel stride); level l >= 1 = P planes of (H2>>l)*(W2>>l) (floor at every
// level), packed, following level l-1.
static void pyr_geom(long P, int H2, int W2, long ld0, int levels, long* off, int* hw) {
  long o = 0;
  int h = H2, w = W2;
  for (int l = 0; l < levels; ++l) {
    if (l > 0) { h /= 2; w /= 2; }
    const long ld = l == 0 ? ld0 : (long)h * w;
    off[l] = o;
    hw[2 * l] = h;
    hw[2 * l + 1] = w;
    hw[2 * levels + l] = (int)ld;
    o += P * ld;
  }
  off[levels] = o;
}

extern "C" long vst_corr_pyramid_floats(long P, int H2, int W2, long ld0, int levels) {
  if (levels < 1 || levels > 8) return -1;
  long off[9];
  int hw[24];
  pyr_geom(P, H2, W2, ld0, levels, off, hw);
  return off[levels];
}

extern "C" int vst_corr_pyramid(float* pyr, long P, int H2, int W2, long ld0, int levels, void* stream) {
  VST_REQUIRE(pyr && P > 0 && levels >= 1 && levels <= 8 && ld0 >= (long)H2 * W2 &&
                  (H2 >> (levels - 1)) >= 1 && (W2 >> (levels - 1)) >= 1,
              "corr_pyramid: bad args");
  long off[9];
  int hw[24];
  pyr_geom(P, H2, W2, ld0, levels, off, hw);
  for (int l = 1; l < levels; ++l) {
    const long total = P * hw[2 * l] * hw[2 * l + 1];
    hipLaunchKernelGGL(avgpool2_planes_k, grid1(total), dim3(256), 0, (hipStream_t)stream,
                       pyr + off[l - 1], pyr + off[l], P, hw[2 * (l - 1)], hw[2 * (l - 1) + 1],
                       (long)hw[2 * levels + l - 1], (long)hw[2 * levels + l]);
  }
  return check_launch("corr_pyramid");
}

extern "C" int vst_corr_lookup(const float* pyr, const float* coords, float* out, int B,
                               int H1, int W1, int H2, int W2, long ld0, int levels, int radius, int Cs,
                               void* stream) {
  VST_REQUIRE(pyr && coords && out && B > 0 && levels >= 1 && levels <= 8 && radius >= 0 &&
                  Cs >= levels * (2 * radius + 1) * (2 * radius + 1),
              "corr_lookup: bad args");
  PyrGeom geo;
  pyr_geom((long)B * H1 * W1, H2, W2, ld0, levels, geo.off, geo.hw);
  for (int l = 0; l < levels; ++l)
    VST_REQUIRE(geo.hw[2 * l] >= 2 && geo.hw[2 * l + 1] >= 2, "corr_lookup: level %d smaller than 2x2", l);
  const long total = (long)B * H1 * W1 * Cs;
  // the level geometry travels as a by-value kernel argument (graph-capturable, no host sync)
  hipLaunchKernelGGL(corr_lookup_k, grid1(total), dim3(256), 0, (hipStream_t)stream, pyr, geo, coords,
                     out, B, H1, W1, levels, radius, Cs);
  return check_launch("corr_lookup");
}

extern "C" int vst_concat_label_nhwc(const float* x, const float* label, float* y, int N, int Cx, int Cl,
                                     int H, int W, int Cs, void* stream) {
  VST_REQUIRE(x && label && y && Cx + Cl <= Cs && N > 0 && H > 0 && W > 0, "concat_label_nhwc: bad args");
  const long total = (long)N * H * W * Cs;
  hipLaunchKernelGGL(concat_label_k, grid1(total), dim3(256), 0, (hipStream_t)stream, x, label, y, N, Cx, Cl,
                     H, W, Cs);
  return check_launch("concat_label_nhwc");
}
