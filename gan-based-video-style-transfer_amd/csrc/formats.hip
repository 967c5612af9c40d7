// Input formats either side of the train step (SURVEY §8f "formats"): the FC2 sample block and 8-bit
// images, unpacked on the device straight into the layouts the kernels consume.
//
// FC2 .npy sample (CycleGANCon/fc2_dataset.py:35-41): float32 [H][W][9] = img1 0:3, img2 3:6 (in
// [0,1]), mask 6:7, flow 7:9.  The reference turns each image into uint8 (np.uint8(v * 255.0), a
// float32 product truncated toward zero), back to float with ToTensor (u / 255) and Normalize(0.5,
// 0.5) ((t - 0.5) / 0.5).  One pass per pixel reads the 36-byte record once and writes img1/img2 as
// NHWC4 (channel 3 zero), the mask as [B][H][W] and the flow as planar [B][2][H][W].  Pure HBM work:
// 36 B read + 44 B written per pixel.
#include "common.h"

namespace vst {

// np.uint8(float32) for the values an FC2 image holds; out-of-range values wrap like the C cast of
// the truncated integer that numpy performs.
__device__ __forceinline__ float to_u8_norm(float v) {
  const float s = __fmul_rn(v, 255.f);
  const int u = ((int)truncf(s)) & 255;
  return __fdiv_rn(__fsub_rn(__fdiv_rn((float)u, 255.f), 0.5f), 0.5f);
}

__global__ void fc2_unpack_k(const float* __restrict__ raw, float4* __restrict__ img1,
                             float4* __restrict__ img2, float* __restrict__ mask, float* __restrict__ flow,
                             long npix, int HW) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npix) return;
  const float* r = raw + p * 9;
  float v[9];
#pragma unroll
  for (int j = 0; j < 9; ++j) v[j] = r[j];
  img1[p] = make_float4(to_u8_norm(v[0]), to_u8_norm(v[1]), to_u8_norm(v[2]), 0.f);
  img2[p] = make_float4(to_u8_norm(v[3]), to_u8_norm(v[4]), to_u8_norm(v[5]), 0.f);
  mask[p] = v[6];
  const long n = p / HW, q = p % HW;
  flow[(n * 2) * HW + q] = v[7];
  flow[(n * 2 + 1) * HW + q] = v[8];
}

// uint8 HWC RGB (PIL decode of a style frame) -> ToTensor + Normalize(0.5, 0.5) as NHWC4
__global__ void u8_image_k(const unsigned char* __restrict__ x, float4* __restrict__ y, long npix) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npix) return;
  const unsigned char* s = x + p * 3;
  float c[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) c[j] = __fdiv_rn(__fsub_rn(__fdiv_rn((float)s[j], 255.f), 0.5f), 0.5f);
  y[p] = make_float4(c[0], c[1], c[2], 0.f);
}

}  // namespace vst

using namespace vst;

extern "C" int vst_fc2_unpack(const float* raw, float* img1, float* img2, float* mask, float* flow, int B, int H,
                              int W, void* stream) {
  VST_REQUIRE(raw && img1 && img2 && mask && flow && B > 0 && H > 0 && W > 0, "fc2_unpack: bad args");
  const long npix = (long)B * H * W;
  hipLaunchKernelGGL(fc2_unpack_k, dim3(ceil_div(npix, 256)), dim3(256), 0, (hipStream_t)stream, raw,
                     reinterpret_cast<float4*>(img1), reinterpret_cast<float4*>(img2), mask, flow, npix, H * W);
  return check_launch("fc2_unpack");
}

extern "C" int vst_u8_image_to_nhwc4(const unsigned char* x, float* y, long npix, void* stream) {
  VST_REQUIRE(x && y && npix > 0, "u8_image_to_nhwc4: bad args");
  hipLaunchKernelGGL(u8_image_k, dim3(ceil_div(npix, 256)), dim3(256), 0, (hipStream_t)stream, x,
                     reinterpret_cast<float4*>(y), npix);
  return check_launch("u8_image_to_nhwc4");
}
