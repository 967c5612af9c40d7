// InstanceNorm2d(affine=False) + ReLU / LeakyReLU forward and backward, NHWC fp32.
// Replaces nn.InstanceNorm2d (reference networks.py:30, affine=False, track_running_stats=False,
// eps=1e-5, biased variance) followed by nn.ReLU(True) (G) / nn.LeakyReLU(0.2, True) (D).
//
// Reductions are per (n, c) over H*W.  A block owns a slice of one image's pixels and ALL its
// channels: lanes run along the channel axis 4 at a time (float4, coalesced rows of the NHWC
// tensor), pixel groups stride the slice, partial sums are kept in fp64 (so the result does not
// depend on the fp32 summation order), folded through LDS, and written per slice; a finalize
// kernel folds the slices in a fixed order (deterministic).  The slice size adapts so every layer
// launches ~512 blocks (64x64x256 res tensors and 256x256x64 outer tensors alike).
#include "common.h"

namespace vst {

constexpr int NRED = 256;

struct RedGeom {
  int LP, PG, SP, nsplit;  // lanes per pixel (C/4), pixel groups, pixels per slice, slices
};

static bool red_geom(int N, int HW, int C, RedGeom& g) {
  if (C % 4) return false;
  g.LP = C / 4;
  if (g.LP > NRED) return false;
  g.PG = NRED / g.LP;  // threads beyond LP*PG idle when LP does not divide NRED
  long sp = ((long)N * HW + 511) / 512;
  if (sp < 2L * g.PG) sp = 2L * g.PG;
  sp = (sp + g.PG - 1) / g.PG * g.PG;
  if (sp > HW) sp = HW;
  g.SP = (int)sp;
  g.nsplit = ceil_div(HW, g.SP);
  return true;
}

// MODE 0: stats partials {sum x, sum x^2}; MODE 1: backward partials {sum g, sum g*xhat, sum xhat}
template <int MODE>
__global__ __launch_bounds__(NRED) void in_partial_k(const float* __restrict__ x,
                                                     const float* __restrict__ gy,
                                                     const float* __restrict__ stats,
                                                     double* __restrict__ part, int HW, int C,
                                                     int LP, int PG, int SP, int nsplit, int act,
                                                     float slope) {
  constexpr int NV = MODE == 0 ? 2 : 3;
  __shared__ double red[NV * 4][NRED];
  const int t = threadIdx.x, c4 = t % LP, pg = t / LP;
  const int n = blockIdx.y, z = blockIdx.x;
  const int p0 = z * SP, p1 = min(HW, p0 + SP);
  double acc[NV][4];
#pragma unroll
  for (int v = 0; v < NV; ++v)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[v][j] = 0.0;
  float mean[4] = {0, 0, 0, 0}, rstd[4] = {0, 0, 0, 0};
  if (MODE == 1) {
    const float4 s0 = reinterpret_cast<const float4*>(stats)[((long)n * C + 4 * c4) / 2];
    const float4 s1 = reinterpret_cast<const float4*>(stats)[((long)n * C + 4 * c4) / 2 + 1];
    mean[0] = s0.x; rstd[0] = s0.y; mean[1] = s0.z; rstd[1] = s0.w;
    mean[2] = s1.x; rstd[2] = s1.y; mean[3] = s1.z; rstd[3] = s1.w;
  }
  const float4* xb = reinterpret_cast<const float4*>(x) + (long)n * HW * LP + c4;
  const float4* gb = reinterpret_cast<const float4*>(gy) + (long)n * HW * LP + c4;
  for (int p = p0 + pg; pg < PG && p < p1; p += PG) {
    const float4 v = xb[(long)p * LP];
    const float xv[4] = {v.x, v.y, v.z, v.w};
    if (MODE == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[0][j] += xv[j];
        acc[1][j] += (double)xv[j] * xv[j];
      }
    } else {
      const float4 gv = gb[(long)p * LP];
      const float gg[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float xh = (xv[j] - mean[j]) * rstd[j];
        float d = 1.f;
        if (act == VST_ACT_RELU) d = xh > 0.f ? 1.f : 0.f;
        else if (act == VST_ACT_LRELU) d = xh > 0.f ? 1.f : slope;
        const float g = gg[j] * d;
        acc[0][j] += g;
        acc[1][j] += (double)g * xh;
        acc[2][j] += xh;
      }
    }
  }
#pragma unroll
  for (int v = 0; v < NV; ++v)
#pragma unroll
    for (int j = 0; j < 4; ++j) red[v * 4 + j][t] = acc[v][j];
  __syncthreads();
  if (pg == 0) {
    double out[NV][4];
#pragma unroll
    for (int v = 0; v < NV; ++v)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        double s = 0.0;
        for (int q = 0; q < PG; ++q) s += red[v * 4 + j][q * LP + c4];
        out[v][j] = s;
      }
    double* dst = part + (((long)n * nsplit + z) * C + 4 * c4) * NV;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int v = 0; v < NV; ++v) dst[j * NV + v] = out[v][j];
  }
}

// Fold the per-slice partials of one (n, 64-channel group): 4 waves stride the slices (coalesced
// over c), then combine through LDS in a fixed order.  out[v] = sum_z part[n][z][c][v].
template <int NV>
__device__ __forceinline__ bool fold_slices(const double* __restrict__ part, int n, int C, int nsplit,
                                            double (&out)[NV]) {
  __shared__ double red[NV][4][64];
  const int cl = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  double acc[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) acc[v] = 0.0;
  if (c < C)
    for (int z = q; z < nsplit; z += 4) {
      const double* a = part + (((long)n * nsplit + z) * C + c) * NV;
#pragma unroll
      for (int v = 0; v < NV; ++v) acc[v] += a[v];
    }
#pragma unroll
  for (int v = 0; v < NV; ++v) red[v][q][cl] = acc[v];
  __syncthreads();
  if (q != 0 || c >= C) return false;
#pragma unroll
  for (int v = 0; v < NV; ++v) out[v] = red[v][0][cl] + red[v][1][cl] + red[v][2][cl] + red[v][3][cl];
  return true;
}

// grid (C/64, N), 256 threads
__global__ void in_finalize_k(const double* __restrict__ part, float* __restrict__ stats, int N,
                              int HW, int C, int nsplit, float eps) {
  double sq[2];
  const int n = blockIdx.y;
  if (!fold_slices<2>(part, n, C, nsplit, sq)) return;
  const int idx = n * C + blockIdx.x * 64 + (threadIdx.x & 63);
  const double mean = sq[0] / HW;
  double var = sq[1] / HW - mean * mean;
  if (var < 0) var = 0;
  stats[2 * idx] = (float)mean;
  stats[2 * idx + 1] = (float)(1.0 / sqrt(var + (double)eps));
}

// coef[(n*C+c)] = {mean(g), mean(g*xhat)}; dbn[n*C+c] = sum_p dx = rstd*((sum g - HW*mean g)
// - mean(g xhat)*sum xhat)  (the exact per-channel sum of the IN input gradient).
__global__ void in_bwd_finalize_k(const double* __restrict__ part, const float* __restrict__ stats,
                                  float2* __restrict__ coef, double* __restrict__ dbn, int N, int HW,
                                  int C, int nsplit) {
  double a[3];
  const int n = blockIdx.y;
  if (!fold_slices<3>(part, n, C, nsplit, a)) return;
  const int idx = n * C + blockIdx.x * 64 + (threadIdx.x & 63);
  const double mg = a[0] / HW, mgx = a[1] / HW;
  coef[idx] = make_float2((float)mg, (float)mgx);
  const double rstd = stats[2 * idx + 1];
  dbn[idx] = rstd * ((a[0] - HW * mg) - mgx * a[2]);
}

// db[c] (+)= sum_n dbn[n][c] in a fixed order (conv-bias gradient)
__global__ void in_bias_grad_k(const double* __restrict__ dbn, float* __restrict__ db, int N, int C,
                               int accumulate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0.0;
  for (int n = 0; n < N; ++n) s += dbn[(long)n * C + c];
  db[c] = accumulate ? db[c] + (float)s : (float)s;
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
  if (res) add_f4(v, res[i]);
  y[i] = v;
}

__device__ __forceinline__ float in_bwd1(float gy, float x, float mean, float rstd, float2 k, int act,
                                         float slope) {
  const float xh = (x - mean) * rstd;
  float d = 1.f;
  if (act == VST_ACT_RELU) d = xh > 0.f ? 1.f : 0.f;
  else if (act == VST_ACT_LRELU) d = xh > 0.f ? 1.f : slope;
  return rstd * (gy * d - k.x - xh * k.y);
}

__global__ void in_bwd_apply_k(const float4* __restrict__ gy, const float4* __restrict__ x,
                               const float* __restrict__ stats, const float2* __restrict__ coef,
                               float4* __restrict__ dx, long total4, int HW, int C4, int act,
                               float slope) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total4) return;
  const int c4 = i % C4;
  const int n = (i / C4) / HW;
  const long nc4 = (long)n * C4 + c4;
  const float4* st = reinterpret_cast<const float4*>(stats) + nc4 * 2;
  const float4 s0 = st[0], s1 = st[1];
  const float4 k01 = reinterpret_cast<const float4*>(coef)[nc4 * 2];
  const float4 k23 = reinterpret_cast<const float4*>(coef)[nc4 * 2 + 1];
  const float4 g = gy[i], v = x[i];
  float4 o;
  o.x = in_bwd1(g.x, v.x, s0.x, s0.y, make_float2(k01.x, k01.y), act, slope);
  o.y = in_bwd1(g.y, v.y, s0.z, s0.w, make_float2(k01.z, k01.w), act, slope);
  o.z = in_bwd1(g.z, v.z, s1.x, s1.y, make_float2(k23.x, k23.y), act, slope);
  o.w = in_bwd1(g.w, v.w, s1.z, s1.w, make_float2(k23.z, k23.w), act, slope);
  dx[i] = o;
}

__global__ void act_bwd_k(const float* __restrict__ gy, const float* __restrict__ y,
                          float* __restrict__ dx, long n, int act, float slope) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dx[i] = gy[i] * act_grad_from_out(y[i], act, slope);
}

// per-channel sum (bias gradient of a layer without a following IN), same geometry as in_partial
__global__ __launch_bounds__(NRED) void chsum_partial_k(const float* __restrict__ x,
                                                        double* __restrict__ part, long NHW, int LP,
                                                        int PG, int SP) {
  __shared__ double red[4][NRED];
  const int t = threadIdx.x, c4 = t % LP, pg = t / LP;
  const long p0 = (long)blockIdx.x * SP, p1 = min(NHW, p0 + SP);
  double acc[4] = {0, 0, 0, 0};
  const float4* xb = reinterpret_cast<const float4*>(x) + c4;
  for (long p = p0 + pg; pg < PG && p < p1; p += PG) {
    const float4 v = xb[p * LP];
    acc[0] += v.x; acc[1] += v.y; acc[2] += v.z; acc[3] += v.w;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) red[j][t] = acc[j];
  __syncthreads();
  if (pg == 0)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      double s = 0.0;
      for (int q = 0; q < PG; ++q) s += red[j][q * LP + c4];
      part[(long)blockIdx.x * LP * 4 + 4 * c4 + j] = s;
    }
}

// grid (Cs/64), 256 threads: db[c] (+)= sum_z part[z][c]
__global__ void chsum_final_k(const double* __restrict__ part, float* __restrict__ db, int nsplit,
                              int Cs, int Cl, int accumulate) {
  double s[1];
  if (!fold_slices<1>(part, 0, Cs, nsplit, s)) return;
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  if (c >= Cl) return;
  db[c] = accumulate ? db[c] + (float)s[0] : (float)s[0];
}

}  // namespace vst

using namespace vst;

extern "C" size_t vst_instnorm_ws_bytes(int N, int HW, int C) {
  RedGeom g;
  if (!red_geom(N, HW, C, g)) return 0;
  return (size_t)N * g.nsplit * C * 3 * sizeof(double) + (size_t)N * C * (sizeof(float2) + sizeof(double)) +
         256;
}

extern "C" int vst_instnorm_stats(const float* x, float* stats, float* ws, int N, int HW, int C,
                                  float eps, void* stream) {
  RedGeom g;
  VST_REQUIRE(x && stats && ws && N > 0 && HW > 0 && red_geom(N, HW, C, g),
              "instnorm_stats: bad args (C must be 4*2^k <= 1024)");
  hipStream_t s = (hipStream_t)stream;
  double* part = reinterpret_cast<double*>(ws);
  hipLaunchKernelGGL(in_partial_k<0>, dim3(g.nsplit, N), dim3(NRED), 0, s, x, (const float*)nullptr,
                     (const float*)nullptr, part, HW, C, g.LP, g.PG, g.SP, g.nsplit, 0, 0.f);
  hipLaunchKernelGGL(in_finalize_k, dim3(ceil_div(C, 64), N), dim3(256), 0, s, part, stats, N, HW, C,
                     g.nsplit, eps);
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
                                    float* db, float* ws, int N, int HW, int C, int act, float slope,
                                    int accumulate_db, void* stream) {
  RedGeom g;
  VST_REQUIRE(gy && x && stats && dx && ws && red_geom(N, HW, C, g), "instnorm_act_bwd: bad args");
  hipStream_t s = (hipStream_t)stream;
  double* part = reinterpret_cast<double*>(ws);
  float2* coef = reinterpret_cast<float2*>(reinterpret_cast<char*>(ws) +
                                           (size_t)N * g.nsplit * C * 3 * sizeof(double));
  hipLaunchKernelGGL(in_partial_k<1>, dim3(g.nsplit, N), dim3(NRED), 0, s, x, gy, stats, part, HW, C,
                     g.LP, g.PG, g.SP, g.nsplit, act, slope);
  double* dbn = reinterpret_cast<double*>(reinterpret_cast<char*>(coef) + (size_t)N * C * sizeof(float2));
  hipLaunchKernelGGL(in_bwd_finalize_k, dim3(ceil_div(C, 64), N), dim3(256), 0, s, part, stats, coef, dbn,
                     N, HW, C, g.nsplit);
  if (db)
    hipLaunchKernelGGL(in_bias_grad_k, dim3(ceil_div(C, 256)), dim3(256), 0, s, dbn, db, N, C,
                       accumulate_db);
  const long total4 = (long)N * HW * C / 4;
  hipLaunchKernelGGL(in_bwd_apply_k, dim3(ceil_div(total4, 256)), dim3(256), 0, s,
                     reinterpret_cast<const float4*>(gy), reinterpret_cast<const float4*>(x), stats,
                     coef, reinterpret_cast<float4*>(dx), total4, HW, C / 4, act, slope);
  return check_launch("instnorm_act_bwd");
}

extern "C" int vst_act_bwd(const float* gy, const float* y, float* dx, long n, int act, float slope,
                           void* stream) {
  VST_REQUIRE(gy && y && dx, "act_bwd: null pointer");
  hipLaunchKernelGGL(act_bwd_k, dim3(ceil_div(n, 256)), dim3(256), 0, (hipStream_t)stream, gy, y, dx,
                     n, act, slope);
  return check_launch("act_bwd");
}

extern "C" size_t vst_channel_sum_ws_bytes(long NHW, int Cs) {
  RedGeom g;
  if (!red_geom(1, (int)NHW, Cs, g)) return 0;
  return (size_t)g.nsplit * Cs * sizeof(double);
}

extern "C" int vst_channel_sum(const float* x, float* db, float* ws, long NHW, int Cs, int Cl,
                               int accumulate, void* stream) {
  RedGeom g;
  VST_REQUIRE(x && db && ws && Cl <= Cs && NHW > 0 && red_geom(1, (int)NHW, Cs, g),
              "channel_sum: bad args");
  hipStream_t s = (hipStream_t)stream;
  double* part = reinterpret_cast<double*>(ws);
  hipLaunchKernelGGL(chsum_partial_k, dim3(g.nsplit), dim3(NRED), 0, s, x, part, NHW, g.LP, g.PG, g.SP);
  hipLaunchKernelGGL(chsum_final_k, dim3(ceil_div(Cs, 64)), dim3(256), 0, s, part, db, g.nsplit, Cs, Cl,
                     accumulate);
  return check_launch("channel_sum");
}
