// InstanceNorm2d(affine=False) + ReLU / LeakyReLU forward and backward, NHWC fp32.
// Replaces nn.InstanceNorm2d (reference networks.py:30, affine=False, track_running_stats=False,
// eps=1e-5, biased variance) followed by nn.ReLU(True) (G) / nn.LeakyReLU(0.2, True) (D).
//
// Statistics are reduced per (n, c) over H*W in fp64 (sum, sum of squares) so the result does not
// depend on the fp32 summation order: each block owns 64 channels of one image and a slice of the
// pixels (split over blockIdx.z for parallelism), writes its partials to the workspace, and a
// finalize kernel folds the slices in a fixed order (deterministic).
#include "common.h"

namespace vst {

constexpr int IN_SPLIT_PIX = 512;  // pixels per block slice

static inline int in_splits(int HW) { return ceil_div(HW, IN_SPLIT_PIX); }

// partial[(n*nsplit + z)*C + c] = {sum, sumsq}  (as double2)
__global__ void in_partial_k(const float* __restrict__ x, double2* __restrict__ part, int HW, int C,
                             int nsplit) {
  __shared__ double2 red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int w = threadIdx.x >> 6;
  const int n = blockIdx.y, z = blockIdx.z;
  const int p0 = z * IN_SPLIT_PIX, p1 = min(HW, p0 + IN_SPLIT_PIX);
  double s = 0.0, q = 0.0;
  if (c < C) {
    const float* base = x + (long)n * HW * C + c;
    for (int p = p0 + w; p < p1; p += 4) {
      const double v = base[(long)p * C];
      s += v;
      q += v * v;
    }
  }
  red[w][threadIdx.x & 63] = make_double2(s, q);
  __syncthreads();
  if (w == 0 && c < C) {
    double2 a = red[0][threadIdx.x];
    for (int i = 1; i < 4; ++i) {
      a.x += red[i][threadIdx.x].x;
      a.y += red[i][threadIdx.x].y;
    }
    part[((long)n * nsplit + z) * C + c] = a;
  }
}

__global__ void in_finalize_k(const double2* __restrict__ part, float* __restrict__ stats, int N,
                              int HW, int C, int nsplit, float eps) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= N * C) return;
  const int n = idx / C, c = idx - n * C;
  double s = 0.0, q = 0.0;
  for (int z = 0; z < nsplit; ++z) {
    const double2 a = part[((long)n * nsplit + z) * C + c];
    s += a.x;
    q += a.y;
  }
  const double mean = s / HW;
  double var = q / HW - mean * mean;
  if (var < 0) var = 0;
  stats[2 * idx] = (float)mean;
  stats[2 * idx + 1] = (float)(1.0 / sqrt(var + (double)eps));
}

__global__ void in_apply_k(const float4* __restrict__ x, const float* __restrict__ stats,
                           const float4* __restrict__ res, float4* __restrict__ y, long total4,
                           int HW, int C4, int act, float slope) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total4) return;
  const int c4 = i % C4;
  const long pix = i / C4;
  const int n = pix / HW;
  const float4* st = reinterpret_cast<const float4*>(stats) + ((long)n * C4 + c4) * 2;
  const float4 s0 = st[0], s1 = st[1];  // {m0,r0,m1,r1}, {m2,r2,m3,r3}
  float4 v = x[i];
  v.x = apply_act((v.x - s0.x) * s0.y, act, slope);
  v.y = apply_act((v.y - s0.z) * s0.w, act, slope);
  v.z = apply_act((v.z - s1.x) * s1.y, act, slope);
  v.w = apply_act((v.w - s1.z) * s1.w, act, slope);
  if (res) {
    const float4 r = res[i];
    v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
  }
  y[i] = v;
}

__device__ __forceinline__ float act_grad_pre(float xh, int act, float slope) {
  if (act == VST_ACT_RELU) return xh > 0.f ? 1.f : 0.f;
  if (act == VST_ACT_LRELU) return xh > 0.f ? 1.f : slope;
  return 1.f;
}

// partials of sum(g) and sum(g * xhat), g = gy * act'(xhat)
__global__ void in_bwd_partial_k(const float* __restrict__ gy, const float* __restrict__ x,
                                 const float* __restrict__ stats, double2* __restrict__ part,
                                 int HW, int C, int nsplit, int act, float slope) {
  __shared__ double2 red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int w = threadIdx.x >> 6;
  const int n = blockIdx.y, z = blockIdx.z;
  const int p0 = z * IN_SPLIT_PIX, p1 = min(HW, p0 + IN_SPLIT_PIX);
  double s = 0.0, q = 0.0;
  if (c < C) {
    const float mean = stats[2 * (n * C + c)], rstd = stats[2 * (n * C + c) + 1];
    const long off = (long)n * HW * C + c;
    for (int p = p0 + w; p < p1; p += 4) {
      const float xh = (x[off + (long)p * C] - mean) * rstd;
      const float g = gy[off + (long)p * C] * act_grad_pre(xh, act, slope);
      s += g;
      q += (double)g * xh;
    }
  }
  red[w][threadIdx.x & 63] = make_double2(s, q);
  __syncthreads();
  if (w == 0 && c < C) {
    double2 a = red[0][threadIdx.x];
    for (int i = 1; i < 4; ++i) {
      a.x += red[i][threadIdx.x].x;
      a.y += red[i][threadIdx.x].y;
    }
    part[((long)n * nsplit + z) * C + c] = a;
  }
}

// coef[(n*C+c)] = {mean(g), mean(g*xhat)} folded into the partial buffer slot 0 (as float2)
__global__ void in_bwd_finalize_k(const double2* __restrict__ part, float2* __restrict__ coef,
                                  int N, int HW, int C, int nsplit) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= N * C) return;
  const int n = idx / C, c = idx - n * C;
  double s = 0.0, q = 0.0;
  for (int z = 0; z < nsplit; ++z) {
    const double2 a = part[((long)n * nsplit + z) * C + c];
    s += a.x;
    q += a.y;
  }
  coef[idx] = make_float2((float)(s / HW), (float)(q / HW));
}

__global__ void in_bwd_apply_k(const float* __restrict__ gy, const float* __restrict__ x,
                               const float* __restrict__ stats, const float2* __restrict__ coef,
                               float* __restrict__ dx, long total, int HW, int C, int act,
                               float slope) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = i % C;
  const int n = (i / C) / HW;
  const int nc = n * C + c;
  const float mean = stats[2 * nc], rstd = stats[2 * nc + 1];
  const float xh = (x[i] - mean) * rstd;
  const float g = gy[i] * act_grad_pre(xh, act, slope);
  const float2 k = coef[nc];
  dx[i] = rstd * (g - k.x - xh * k.y);
}

__global__ void act_bwd_k(const float* __restrict__ gy, const float* __restrict__ y,
                          float* __restrict__ dx, long n, int act, float slope) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dx[i] = gy[i] * act_grad_from_out(y[i], act, slope);
}

}  // namespace vst

using namespace vst;

extern "C" size_t vst_instnorm_ws_bytes(int N, int HW, int C) {
  const size_t part = (size_t)N * in_splits(HW) * C * sizeof(double2);
  const size_t coef = (size_t)N * C * sizeof(float2);
  return part + coef + 256;
}

extern "C" int vst_instnorm_stats(const float* x, float* stats, float* ws, int N, int HW, int C,
                                  float eps, void* stream) {
  VST_REQUIRE(x && stats && ws && N > 0 && HW > 0 && C > 0, "instnorm_stats: bad args");
  hipStream_t s = (hipStream_t)stream;
  const int ns = in_splits(HW);
  double2* part = reinterpret_cast<double2*>(ws);
  hipLaunchKernelGGL(in_partial_k, dim3(ceil_div(C, 64), N, ns), dim3(256), 0, s, x, part, HW, C, ns);
  hipLaunchKernelGGL(in_finalize_k, dim3(ceil_div((long)N * C, 256)), dim3(256), 0, s, part, stats, N,
                     HW, C, ns, eps);
  return check_launch("instnorm_stats");
}

extern "C" int vst_instnorm_act_fwd(const float* x, const float* stats, const float* residual,
                                    float* y, int N, int HW, int C, int act, float slope,
                                    void* stream) {
  VST_REQUIRE(x && stats && y && C % 4 == 0, "instnorm_act_fwd: bad args");
  const long total4 = (long)N * HW * C / 4;
  hipLaunchKernelGGL(in_apply_k, dim3(ceil_div(total4, 256)), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const float4*>(x), stats, reinterpret_cast<const float4*>(residual),
                     reinterpret_cast<float4*>(y), total4, HW, C / 4, act, slope);
  return check_launch("instnorm_act_fwd");
}

extern "C" int vst_instnorm_act_bwd(const float* gy, const float* x, const float* stats, float* dx,
                                    float* ws, int N, int HW, int C, int act, float slope,
                                    void* stream) {
  VST_REQUIRE(gy && x && stats && dx && ws, "instnorm_act_bwd: bad args");
  hipStream_t s = (hipStream_t)stream;
  const int ns = in_splits(HW);
  double2* part = reinterpret_cast<double2*>(ws);
  float2* coef = reinterpret_cast<float2*>(reinterpret_cast<char*>(ws) +
                                           (size_t)N * ns * C * sizeof(double2));
  hipLaunchKernelGGL(in_bwd_partial_k, dim3(ceil_div(C, 64), N, ns), dim3(256), 0, s, gy, x, stats,
                     part, HW, C, ns, act, slope);
  hipLaunchKernelGGL(in_bwd_finalize_k, dim3(ceil_div((long)N * C, 256)), dim3(256), 0, s, part,
                     coef, N, HW, C, ns);
  const long total = (long)N * HW * C;
  hipLaunchKernelGGL(in_bwd_apply_k, dim3(ceil_div(total, 256)), dim3(256), 0, s, gy, x, stats, coef,
                     dx, total, HW, C, act, slope);
  return check_launch("instnorm_act_bwd");
}

extern "C" int vst_act_bwd(const float* gy, const float* y, float* dx, long n, int act, float slope,
                           void* stream) {
  VST_REQUIRE(gy && y && dx, "act_bwd: null pointer");
  hipLaunchKernelGGL(act_bwd_k, dim3(ceil_div(n, 256)), dim3(256), 0, (hipStream_t)stream, gy, y, dx,
                     n, act, slope);
  return check_launch("act_bwd");
}

// ------------------------------------------------------------------ per-channel sum (bias grad)
namespace vst {
constexpr int CS_SPLIT_PIX = 1024;

__global__ void chsum_partial_k(const float* __restrict__ x, float* __restrict__ part, long NHW,
                                int Cs, int Cl) {
  __shared__ float red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int w = threadIdx.x >> 6;
  const long p0 = (long)blockIdx.y * CS_SPLIT_PIX;
  const long p1 = min(NHW, p0 + CS_SPLIT_PIX);
  float s = 0.f;
  if (c < Cl)
    for (long p = p0 + w; p < p1; p += 4) s += x[p * Cs + c];
  red[w][threadIdx.x & 63] = s;
  __syncthreads();
  if (w == 0 && c < Cl)
    part[(long)blockIdx.y * Cl + c] = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] +
                                      red[3][threadIdx.x];
}

__global__ void chsum_final_k(const float* __restrict__ part, float* __restrict__ db, int nsplit,
                              int Cl, int accumulate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= Cl) return;
  double s = 0.0;
  for (int z = 0; z < nsplit; ++z) s += part[(long)z * Cl + c];
  db[c] = accumulate ? db[c] + (float)s : (float)s;
}
}  // namespace vst

extern "C" size_t vst_channel_sum_ws_bytes(long NHW, int Cl) {
  return (size_t)ceil_div(NHW, CS_SPLIT_PIX) * Cl * sizeof(float);
}

extern "C" int vst_channel_sum(const float* x, float* db, float* ws, long NHW, int Cs, int Cl,
                               int accumulate, void* stream) {
  VST_REQUIRE(x && db && ws && Cl <= Cs && NHW > 0, "channel_sum: bad args");
  hipStream_t s = (hipStream_t)stream;
  const int ns = ceil_div(NHW, CS_SPLIT_PIX);
  hipLaunchKernelGGL(chsum_partial_k, dim3(ceil_div(Cl, 64), ns), dim3(256), 0, s, x, ws, NHW, Cs, Cl);
  hipLaunchKernelGGL(chsum_final_k, dim3(ceil_div(Cl, 256)), dim3(256), 0, s, ws, db, ns, Cl, accumulate);
  return check_launch("channel_sum");
}
