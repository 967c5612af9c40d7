// Reductions for the GAN / cycle / identity losses on NHWC images with channel stride Cs and Cl
// logical channels.  Replaces GANLoss('lsgan') = nn.MSELoss against a constant target
// (methods/GAN-based/CycleGAN/models/networks.py:209-275) and nn.L1Loss
// (methods/GAN-based/CycleGANCon/models/cycle_gan_model.py:94-95, 180-189, 211-213).
// Forward: per-block partial sums + one fixed-order final reduction (deterministic).
// Backward: elementwise, reading the upstream scalar gradient from device memory (no host sync).
#include "common.h"

namespace vst {

template <int KIND>  // 0: |a-b|, 1: (a - t)^2
__global__ void loss_part_k(const float* __restrict__ a, const float* __restrict__ b, float t,
                            float* __restrict__ part, long npix, int Cs, int Cl) {
  __shared__ float red[4];
  const long pix = (long)blockIdx.x * blockDim.x + threadIdx.x;
  float acc = 0.f;
  if (pix < npix) {
    for (int c = 0; c < Cl; ++c) {
      const float d = a[pix * Cs + c] - (KIND == 0 ? b[pix * Cs + c] : t);
      acc += KIND == 0 ? fabsf(d) : d * d;
    }
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

template <int KIND>
__global__ void loss_grad_k(const float* __restrict__ a, const float* __restrict__ b, float t,
                            const float* __restrict__ gout, float k, float* __restrict__ grad,
                            long npix, int Cs, int Cl) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npix * Cs) return;
  const int c = i % Cs;
  float g = 0.f;
  if (c < Cl) {
    const float d = a[i] - (KIND == 0 ? b[i] : t);
    const float kk = k * gout[0];
    g = KIND == 0 ? kk * (float)((d > 0.f) - (d < 0.f)) : kk * 2.f * d;
  }
  grad[i] = g;
}

__global__ void finish_sum2_k(const float* __restrict__ part, int n, float* __restrict__ out,
                              double scale) {
  __shared__ double red[4];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) s += part[i];
  s = wave_sum_d(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = (float)((red[0] + red[1] + red[2] + red[3]) * scale);
}

// masked L1 (MoGAN's motion losses): sum_pix m[pix] * sum_{c<Cl} |a - b|; m == nullptr -> 1
__global__ void masked_l1_part_k(const float* __restrict__ a, const float* __restrict__ b,
                                 const float* __restrict__ m, float* __restrict__ part, long npix, int Cs, int Cl) {
  __shared__ float red[4];
  const long pix = (long)blockIdx.x * blockDim.x + threadIdx.x;
  float acc = 0.f;
  if (pix < npix) {
    const float mk = m ? m[pix] : 1.f;
    for (int c = 0; c < Cl; ++c) acc += mk * fabsf(a[pix * Cs + c] - b[pix * Cs + c]);
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ void masked_l1_grad_k(const float* __restrict__ a, const float* __restrict__ b,
                                 const float* __restrict__ m, const float* __restrict__ gout, float k,
                                 float* __restrict__ grad, long npix, int Cs, int Cl) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npix * Cs) return;
  const int c = i % Cs;
  float g = 0.f;
  if (c < Cl) {
    const float d = a[i] - b[i];
    g = k * gout[0] * (m ? m[i / Cs] : 1.f) * (float)((d > 0.f) - (d < 0.f));
  }
  grad[i] = g;
}

}  // namespace vst

using namespace vst;

extern "C" int vst_loss_masked_l1(const float* a, const float* b, const float* mask, float* loss, float* part,
                                  long npix, int Cs, int Cl, float scale, void* stream) {
  VST_REQUIRE(a && b && loss && part && Cl <= Cs && npix > 0, "loss_masked_l1: bad args");
  hipStream_t s = (hipStream_t)stream;
  const int nb = ceil_div(npix, 256);
  hipLaunchKernelGGL(masked_l1_part_k, dim3(nb), dim3(256), 0, s, a, b, mask, part, npix, Cs, Cl);
  hipLaunchKernelGGL(finish_sum2_k, dim3(1), dim3(256), 0, s, part, nb, loss, (double)scale / ((double)npix * Cl));
  return check_launch("loss_masked_l1");
}

extern "C" int vst_loss_masked_l1_bwd(const float* a, const float* b, const float* mask, const float* gout,
                                      float* grad, long npix, int Cs, int Cl, float scale, void* stream) {
  VST_REQUIRE(a && b && gout && grad && Cl <= Cs && npix > 0, "loss_masked_l1_bwd: bad args");
  const float k = (float)((double)scale / ((double)npix * Cl));
  hipLaunchKernelGGL(masked_l1_grad_k, dim3(ceil_div(npix * Cs, 256)), dim3(256), 0, (hipStream_t)stream, a, b,
                     mask, gout, k, grad, npix, Cs, Cl);
  return check_launch("loss_masked_l1_bwd");
}

extern "C" int vst_loss_l1(const float* a, const float* b, float* loss, float* part, long npix,
                           int Cs, int Cl, float scale, void* stream) {
  VST_REQUIRE(a && b && loss && part && Cl <= Cs && npix > 0, "loss_l1: bad args");
  hipStream_t s = (hipStream_t)stream;
  const int nb = ceil_div(npix, 256);
  hipLaunchKernelGGL(loss_part_k<0>, dim3(nb), dim3(256), 0, s, a, b, 0.f, part, npix, Cs, Cl);
  hipLaunchKernelGGL(finish_sum2_k, dim3(1), dim3(256), 0, s, part, nb, loss,
                     (double)scale / ((double)npix * Cl));
  return check_launch("loss_l1");
}

extern "C" int vst_loss_l1_bwd(const float* a, const float* b, const float* gout, float* grad,
                               long npix, int Cs, int Cl, float scale, void* stream) {
  VST_REQUIRE(a && b && gout && grad, "loss_l1_bwd: bad args");
  const float k = (float)((double)scale / ((double)npix * Cl));
  hipLaunchKernelGGL(loss_grad_k<0>, dim3(ceil_div(npix * Cs, 256)), dim3(256), 0, (hipStream_t)stream,
                     a, b, 0.f, gout, k, grad, npix, Cs, Cl);
  return check_launch("loss_l1_bwd");
}

extern "C" int vst_loss_mse_const(const float* a, float target, float* loss, float* part, long npix,
                                  int Cs, int Cl, float scale, void* stream) {
  VST_REQUIRE(a && loss && part && Cl <= Cs && npix > 0, "loss_mse_const: bad args");
  hipStream_t s = (hipStream_t)stream;
  const int nb = ceil_div(npix, 256);
  hipLaunchKernelGGL(loss_part_k<1>, dim3(nb), dim3(256), 0, s, a, (const float*)nullptr, target,
                     part, npix, Cs, Cl);
  hipLaunchKernelGGL(finish_sum2_k, dim3(1), dim3(256), 0, s, part, nb, loss,
                     (double)scale / ((double)npix * Cl));
  return check_launch("loss_mse_const");
}

extern "C" int vst_loss_mse_const_bwd(const float* a, float target, const float* gout, float* grad,
                                      long npix, int Cs, int Cl, float scale, void* stream) {
  VST_REQUIRE(a && gout && grad, "loss_mse_const_bwd: bad args");
  const float k = (float)((double)scale / ((double)npix * Cl));
  hipLaunchKernelGGL(loss_grad_k<1>, dim3(ceil_div(npix * Cs, 256)), dim3(256), 0,
                     (hipStream_t)stream, a, (const float*)nullptr, target, gout, k, grad, npix, Cs, Cl);
  return check_launch("loss_mse_const_bwd");
}
