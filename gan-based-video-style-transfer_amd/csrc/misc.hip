// Layout conversion, weight packing, fused Adam and small helpers; error reporting for the C ABI.
#include <stdarg.h>

#include "common.h"

namespace vst {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

__global__ void nchw_to_nhwc_k(const float* __restrict__ x, float* __restrict__ y, int C, int HW,
                               int Cs, long total) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = i % Cs;
  const long pix = i / Cs;
  const long n = pix / HW, p = pix - n * HW;
  y[i] = c < C ? x[(n * C + c) * HW + p] : 0.f;
}

__global__ void nhwc_to_nchw_k(const float* __restrict__ x, float* __restrict__ y, int C, int HW,
                               int Cs, long total) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const long p = i % HW;
  const long nc = i / HW;
  const int c = nc % C;
  const long n = nc / C;
  y[i] = x[(n * HW + p) * Cs + c];
}

// Element idx of a pack of the logical weight w[O][I][R][S] -> its (o, i, tap) coordinates.
// KC: out[r][s][i][o] (Ip x Op per tap), CK: out[r][s][o][i] (Op x Ip per tap), OK: out[o][r][s][i],
// IK / IKF: out[i][r][s][o] (IKF: taps rotated 180 deg).
// SOK: out[s][o][r][i] (the OK pack of the R x 1 conv with S*Op outputs (s, o)).
__device__ __forceinline__ void pack_coords(long idx, int R, int S, int Op, int Ip, int mode, int& o, int& i,
                                            int& rs) {
  const int RS = R * S;
  if (mode == VST_PACK_SOK) {  // idx = ((s*Op + o)*R + r)*Ip + i
    i = idx % Ip;
    const long q = idx / Ip;
    const int r = q % R;
    const long q2 = q / R;
    o = q2 % Op;
    rs = r * S + (int)(q2 / Op);
  } else if (mode == VST_PACK_KC) {  // idx = (rs*Ip + i)*Op + o
    o = idx % Op;
    const long q = idx / Op;
    i = q % Ip;
    rs = q / Ip;
  } else if (mode == VST_PACK_CK) {  // idx = (rs*Op + o)*Ip + i
    i = idx % Ip;
    const long q = idx / Ip;
    o = q % Op;
    rs = q / Op;
  } else if (mode == VST_PACK_OK) {  // idx = (o*RS + rs)*Ip + i
    i = idx % Ip;
    const long q = idx / Ip;
    rs = q % RS;
    o = q / RS;
  } else {  // VST_PACK_IK / VST_PACK_IKF: idx = (i*RS + rs)*Op + o
    o = idx % Op;
    const long q = idx / Op;
    rs = q % RS;
    i = q / RS;
    if (mode == VST_PACK_IKF) rs = RS - 1 - rs;
  }
}

// The three bf16 planes hi, mid, lo of v (vst_weight_split's conversions).
__device__ __forceinline__ void store_split(__bf16* __restrict__ split, long total, long idx, float v) {
  const __bf16 h = (__bf16)v;
  const float r = v - (float)h;
  const __bf16 m = (__bf16)r;
  split[idx] = h;
  split[total + idx] = m;
  split[2 * total + idx] = (__bf16)(r - (float)m);
}

// Batched packing: every pack of a network in one launch (vst_weight_pack_batch).  Job j covers
// blocks [block0, next block0); its logical weight element (o, i, r, s) is read at
// w[o*so + i*si + tr[r]*sr + ts[s]*ss] (tap maps: the transposed-conv phase packs pick taps;
// tr[0] < 0 / ts[0] < 0 = identity, any R / S).
struct PackJob {
  const float* w;
  float* out;
  __bf16* split;
  int O, I, R, S, Op, Ip, mode, pad_;
  long total, block0;
  long so, si, sr, ss;
  int tr[8], ts[8];
};
static_assert(sizeof(PackJob) == 168, "PackJob layout is part of the C ABI (include/vst_hip.h)");

// One 64-lane block per 256-element job block (PackJob.block0 units): a lane packs 4 consecutive elements (their
// gathers issued together), stores them as one float4 and each split plane as one 8-byte word — the per-element
// form moved ~1.5 TB/s (narrow stores, one gather in flight per lane).
// The per-element form (one element per lane, 256-lane blocks): kind 0.
__global__ __launch_bounds__(256) void weight_pack_batch1_k(const PackJob* __restrict__ jobs, int nj) {
  const long b = blockIdx.x;
  int lo = 0, hi = nj - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].block0 <= b) lo = mid;
    else hi = mid - 1;
  }
  const PackJob& J = jobs[lo];
  const long idx = (b - J.block0) * 256 + threadIdx.x;
  if (idx >= J.total) return;
  int o, i, rs;
  pack_coords(idx, J.R, J.S, J.Op, J.Ip, J.mode, o, i, rs);
  const int r = rs / J.S, s = rs - r * J.S;
  const int rr = J.tr[0] < 0 ? r : J.tr[r], ss = J.ts[0] < 0 ? s : J.ts[s];
  const float v = (o < J.O && i < J.I) ? J.w[o * J.so + i * J.si + rr * J.sr + ss * J.ss] : 0.f;
  J.out[idx] = v;
  if (J.split) store_split(J.split, J.total, idx, v);
}

template <bool TILED>
__global__ __launch_bounds__(64) void weight_pack_batch_k(const PackJob* __restrict__ jobs, int nj) {
  const long b = blockIdx.x;
  int lo = 0, hi = nj - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].block0 <= b) lo = mid;
    else hi = mid - 1;
  }
  const PackJob& J = jobs[lo];
  const int RS = J.R * J.S;
  // OK / IK / IKF packs with >= 4 taps and a 64-multiple inner extent: tiled.  Block = (outer index A, 64 inner
  // indices B): the source rows (A, B) are read along their taps (contiguous for identity tap maps) into an LDS
  // tile, then written as whole 64-float rows per tap (+ planes).  The job's 256-element blocks cover its
  // A x Bp / 64 tiles when RS >= 4; the rest of them exit.
  const bool ok_mode = J.mode == VST_PACK_OK;
  if (TILED && (ok_mode || J.mode == VST_PACK_IK || J.mode == VST_PACK_IKF) && RS >= 4 && RS <= 16) {
    const int Ap = ok_mode ? J.Op : J.Ip, Bp = ok_mode ? J.Ip : J.Op;
    if (Bp % 64 == 0) {
      __shared__ float tile[64 * 17];
      const long jb = b - J.block0, nb = Bp / 64;
      if (jb >= (long)Ap * nb) return;
      const int A = (int)(jb / nb), B0 = (int)(jb - (long)A * nb) * 64;
      const bool flip = J.mode == VST_PACK_IKF;
      for (int q = threadIdx.x; q < 64 * RS; q += 64) {
        const int bb = q / RS, rs = q - bb * RS;  // rs: the source tap
        const int o = ok_mode ? A : B0 + bb, i = ok_mode ? B0 + bb : A;
        const int r = rs / J.S, sx = rs - r * J.S;
        const int rr = J.tr[0] < 0 ? r : J.tr[r], ss = J.ts[0] < 0 ? sx : J.ts[sx];
        const float v = (o < J.O && i < J.I) ? J.w[o * J.so + i * J.si + rr * J.sr + ss * J.ss] : 0.f;
        tile[bb * 17 + (flip ? RS - 1 - rs : rs)] = v;
      }
      __syncthreads();
      for (int q = threadIdx.x; q < 64 * RS; q += 64) {
        const int rs = q >> 6, bb = q & 63;  // rs: the pack's tap
        const float v = tile[bb * 17 + rs];
        const long idx = ((long)A * RS + rs) * Bp + B0 + bb;
        J.out[idx] = v;
        if (J.split) store_split(J.split, J.total, idx, v);
      }
      return;
    }
  }
  const long idx0 = (b - J.block0) * 256 + 4 * threadIdx.x;
  if (idx0 >= J.total) return;
  float v[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[e] = 0.f;
    const long idx = idx0 + e;
    if (idx >= J.total) continue;
    int o, i, rs;
    pack_coords(idx, J.R, J.S, J.Op, J.Ip, J.mode, o, i, rs);
    const int r = rs / J.S, s = rs - r * J.S;
    const int rr = J.tr[0] < 0 ? r : J.tr[r], ss = J.ts[0] < 0 ? s : J.ts[s];  // tr[0] < 0: identity
    if (o < J.O && i < J.I) v[e] = J.w[o * J.so + i * J.si + rr * J.sr + ss * J.ss];
  }
  if (J.total % 4 == 0) {  // idx0 % 4 == 0: aligned float4 / 8-byte plane words
    *reinterpret_cast<float4*>(J.out + idx0) = make_float4(v[0], v[1], v[2], v[3]);
    if (J.split) {
      uint16_t q[3][4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const __bf16 h = (__bf16)v[e];
        const float r = v[e] - (float)h;
        const __bf16 m = (__bf16)r;
        const __bf16 l = (__bf16)(r - (float)m);
        q[0][e] = __builtin_bit_cast(uint16_t, h);
        q[1][e] = __builtin_bit_cast(uint16_t, m);
        q[2][e] = __builtin_bit_cast(uint16_t, l);
      }
#pragma unroll
      for (int p = 0; p < 3; ++p)
        *reinterpret_cast<uint2*>(J.split + p * J.total + idx0) =
            make_uint2(q[p][0] | ((uint32_t)q[p][1] << 16), q[p][2] | ((uint32_t)q[p][3] << 16));
    }
    return;
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (idx0 + e >= J.total) break;
    J.out[idx0 + e] = v[e];
    if (J.split) store_split(J.split, J.total, idx0 + e, v[e]);
  }
}

// w[O][I][R][S] -> one pack (modes as pack_coords), optionally with its split planes
__global__ void weight_pack_k(const float* __restrict__ w, float* __restrict__ out, int O, int I,
                              int R, int S, int Op, int Ip, int mode, long total,
                              __bf16* __restrict__ split = nullptr) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int RS = R * S;
  int o, i, rs;
  pack_coords(idx, R, S, Op, Ip, mode, o, i, rs);
  const float v = (o < O && i < I) ? w[((long)o * I + i) * RS + rs] : 0.f;
  out[idx] = v;
  if (split) store_split(split, total, idx, v);
}

__global__ void adam_k(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                       float* __restrict__ v, long n, float lr, float b1, float b2, float eps,
                       float bc1, float bc2_sqrt) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float gi = g[i];
  // exp_avg.lerp_(grad, 1 - beta1) with ATen's two-sided lerp formula
  const float w = 1.f - b1, m0 = m[i];
  const float mi = w < 0.5f ? m0 + w * (gi - m0) : gi - (gi - m0) * (1.f - w);
  // exp_avg_sq.mul_(beta2).addcmul_(grad, grad, value=1 - beta2)
  const float vi = v[i] * b2 + (1.f - b2) * (gi * gi);
  m[i] = mi;
  v[i] = vi;
  // torch.optim.Adam (single-tensor, capturable=False):
  //   denom = sqrt(v) / sqrt(1 - b2^t) + eps ; p -= (lr / (1 - b1^t)) * m / denom
  const float denom = sqrtf(vi) / bc2_sqrt + eps;
  p[i] -= (lr / bc1) * (mi / denom);
}

__global__ void axpby_k(const float* __restrict__ x, float* __restrict__ y, long n, float a,
                        float b) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = a * x[i] + b * y[i];
}

}  // namespace vst

using namespace vst;

extern "C" const char* vst_last_error(void) { return g_err; }
extern "C" int vst_version(void) { return 1; }

extern "C" int vst_nchw_to_nhwc(const float* x, float* y, int N, int C, int H, int W, int Cs,
                                void* stream) {
  VST_REQUIRE(x && y && C <= Cs, "nchw_to_nhwc: bad args");
  const long total = (long)N * H * W * Cs;
  hipLaunchKernelGGL(nchw_to_nhwc_k, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, x,
                     y, C, H * W, Cs, total);
  return check_launch("nchw_to_nhwc");
}

extern "C" int vst_nhwc_to_nchw(const float* x, float* y, int N, int C, int H, int W, int Cs,
                                void* stream) {
  VST_REQUIRE(x && y && C <= Cs, "nhwc_to_nchw: bad args");
  const long total = (long)N * C * H * W;
  hipLaunchKernelGGL(nhwc_to_nchw_k, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, x,
                     y, C, H * W, Cs, total);
  return check_launch("nhwc_to_nchw");
}

extern "C" int vst_weight_pack(const float* w, float* out, int O, int I, int R, int S, int Op,
                               int Ip, int mode, void* stream) {
  VST_REQUIRE(w && out && O <= Op && I <= Ip && mode >= VST_PACK_KC && mode <= VST_PACK_SOK,
              "weight_pack: bad args");
  const long total = (long)R * S * Op * Ip;
  hipLaunchKernelGGL(weight_pack_k, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, w,
                     out, O, I, R, S, Op, Ip, mode, total);
  return check_launch("weight_pack");
}

extern "C" int vst_weight_pack_split(const float* w, float* out, void* split, int O, int I, int R, int S, int Op,
                                     int Ip, int mode, void* stream) {
  VST_REQUIRE(w && out && split && O <= Op && I <= Ip && mode >= VST_PACK_KC && mode <= VST_PACK_SOK,
              "weight_pack_split: bad args");
  const long total = (long)R * S * Op * Ip;
  hipLaunchKernelGGL(weight_pack_k, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, w, out, O, I, R,
                     S, Op, Ip, mode, total, reinterpret_cast<__bf16*>(split));
  return check_launch("weight_pack_split");
}

extern "C" int vst_weight_pack_batch(const void* jobs, int njobs, long nblocks, void* stream) {
  VST_REQUIRE(jobs && njobs > 0 && nblocks > 0 && nblocks < (1L << 31), "weight_pack_batch: bad args");
  constexpr int kind = 2;  // 0: per element, 1: 4 elements per lane, 2: + the tiled OK / IK / IKF path
  const PackJob* J = reinterpret_cast<const PackJob*>(jobs);
  if (kind == 0)
    hipLaunchKernelGGL(weight_pack_batch1_k, dim3((unsigned)nblocks), dim3(256), 0, (hipStream_t)stream, J, njobs);
  else if (kind == 1)
    hipLaunchKernelGGL(weight_pack_batch_k<false>, dim3((unsigned)nblocks), dim3(64), 0, (hipStream_t)stream, J, njobs);
  else
    hipLaunchKernelGGL(weight_pack_batch_k<true>, dim3((unsigned)nblocks), dim3(64), 0, (hipStream_t)stream, J, njobs);
  return check_launch("weight_pack_batch");
}

extern "C" int vst_adam_step(float* p, const float* g, float* m, float* v, long n, float lr,
                             float beta1, float beta2, float eps, int step, void* stream) {
  VST_REQUIRE(p && g && m && v && step >= 1, "adam_step: bad args");
  const double bc1 = 1.0 - pow((double)beta1, step);
  const double bc2 = 1.0 - pow((double)beta2, step);
  hipLaunchKernelGGL(adam_k, dim3(ceil_div(n, 256)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n,
                     lr, beta1, beta2, eps, (float)bc1, (float)sqrt(bc2));
  return check_launch("adam_step");
}

extern "C" int vst_axpby(const float* x, float* y, long n, float a, float b, void* stream) {
  VST_REQUIRE(x && y, "axpby: bad args");
  hipLaunchKernelGGL(axpby_k, dim3(ceil_div(n, 256)), dim3(256), 0, (hipStream_t)stream, x, y, n, a, b);
  return check_launch("axpby");
}
