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
// target number of (slice, sample) blocks of a reduction pass over N*HW pixels
#ifndef IN_TARGET_BLOCKS
#define IN_TARGET_BLOCKS 512
#endif

struct RedGeom {
  int LP, PG, SP, nsplit;  // lanes per pixel (C/4), pixel groups, pixels per slice, slices
};

static bool red_geom(int N, int HW, int C, RedGeom& g) {
  if (C % 4) return false;
  g.LP = C / 4;
  if (g.LP > NRED) return false;
  g.PG = NRED / g.LP;  // threads beyond LP*PG idle when LP does not divide NRED
  long sp = ((long)N * HW + IN_TARGET_BLOCKS - 1) / IN_TARGET_BLOCKS;
  if (sp < 2L * g.PG) sp = 2L * g.PG;
  sp = (sp + g.PG - 1) / g.PG * g.PG;
  if (sp > HW) sp = HW;
  g.SP = (int)sp;
  g.nsplit = ceil_div(HW, g.SP);
  return true;
}

#ifndef IN_UNROLL
#define IN_UNROLL 4
#endif

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
  // one pixel row's float4 (x, and g for MODE 1) into the fp64 partials
  auto accum = [&](const float4 v, const float4 gv) {
    const float xv[4] = {v.x, v.y, v.z, v.w};
    if (MODE == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[0][j] += xv[j];
        acc[1][j] += (double)xv[j] * xv[j];
      }
    } else {
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
  };
  // the thread's rows p, p + PG, p + 2 PG, ... accumulated in that order; UR rows' loads are
  // issued together ahead of their (serial, order-preserving) fp64 accumulation
  constexpr int UR = IN_UNROLL;
  if (pg < PG) {
    int p = p0 + pg;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    for (; p + (UR - 1) * PG < p1; p += UR * PG) {
      float4 v[UR], gv[UR];
#pragma unroll
      for (int k = 0; k < UR; ++k) {
        v[k] = xb[(long)(p + k * PG) * LP];
        gv[k] = MODE == 1 ? gb[(long)(p + k * PG) * LP] : z4;
      }
#pragma unroll
      for (int k = 0; k < UR; ++k) accum(v[k], gv[k]);
    }
    for (; p < p1; p += PG) accum(xb[(long)p * LP], MODE == 1 ? gb[(long)p * LP] : z4);
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

// Fold the per-slice partials of one (n, CPB-channel group): G = 256 / CPB thread groups stride the
// slices (coalesced over c), then combine through LDS in a fixed order.  out[v] = sum_z
// part[n][z][c][v].  CPB = 16 for the IN finalizes (4x the blocks of CPB = 64: these small kernels are
// latency-bound, their slice chains 4x shorter).
template <int NV, int CPB = 64>
__device__ __forceinline__ bool fold_slices(const double* __restrict__ part, int n, int C, int nsplit,
                                            double (&out)[NV]) {
  constexpr int G = 256 / CPB;
  __shared__ double red[NV][G][CPB];
  const int cl = threadIdx.x % CPB, q = threadIdx.x / CPB;
  const int c = blockIdx.x * CPB + cl;
  // 4 independent accumulator chains per thread (slices q, q+G, q+2G, q+3G, then +4G ...) so the
  // loads overlap instead of serialising on the fp64 add chain; combined in a fixed order.
  double acc[NV], acc4[4][NV];
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int v = 0; v < NV; ++v) acc4[u][v] = 0.0;
  if (c < C) {
    const long zs = (long)C * NV;
    const double* base = part + (((long)n * nsplit) * C + c) * NV;
    int z = q;
    for (; z + 3 * G < nsplit; z += 4 * G) {
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < NV; ++v) acc4[u][v] += base[(long)(z + G * u) * zs + v];
    }
    for (; z < nsplit; z += G)
#pragma unroll
      for (int v = 0; v < NV; ++v) acc4[0][v] += base[(long)z * zs + v];
  }
#pragma unroll
  for (int v = 0; v < NV; ++v) acc[v] = (acc4[0][v] + acc4[1][v]) + (acc4[2][v] + acc4[3][v]);
#pragma unroll
  for (int v = 0; v < NV; ++v) red[v][q][cl] = acc[v];
  __syncthreads();
  if (q != 0 || c >= C) return false;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    double o = 0.0;
#pragma unroll
    for (int g = 0; g < G; ++g) o += red[v][g][cl];
    out[v] = o;
  }
  return true;
}

// Channels per finalize block: 16, or 4 when (C / 16) x N blocks would leave most CUs idle over many
// slices (the first conv's 64 channels x 8 images over 2048 slices: 32 blocks, 14 us; B=1 inference's
// 256 channels: 16 blocks) — 4x the blocks, each thread's slice chain 4x shorter.
static constexpr bool g_fin_narrow = true;
static int fin_cpb(int C, int N, int nsplit) {
  return (!g_fin_narrow || (long)((C + 15) / 16) * N >= 128 || nsplit < 64) ? 16 : 4;
}

// grid (C/CPB, N), 256 threads
template <int CPB>
__global__ void in_finalize_k(const double* __restrict__ part, float* __restrict__ stats, int N,
                              int HW, int C, int nsplit, float eps) {
  double sq[2];
  const int n = blockIdx.y;
  if (!fold_slices<2, CPB>(part, n, C, nsplit, sq)) return;
  const int idx = n * C + blockIdx.x * CPB + (threadIdx.x % CPB);
  const double mean = sq[0] / HW;
  double var = sq[1] / HW - mean * mean;
  if (var < 0) var = 0;
  stats[2 * idx] = (float)mean;
  stats[2 * idx + 1] = (float)(1.0 / sqrt(var + (double)eps));
}

// coef[(n*C+c)] = {mean(g), mean(g*xhat)}; dbn[n*C+c] = sum_p dx = rstd*((sum g - HW*mean g)
// - mean(g xhat)*sum xhat)  (the exact per-channel sum of the IN input gradient).
template <int CPB>
__global__ void in_bwd_finalize_k(const double* __restrict__ part, const float* __restrict__ stats,
                                  float2* __restrict__ coef, double* __restrict__ dbn, int N, int HW,
                                  int C, int nsplit) {
  double a[3];
  const int n = blockIdx.y;
  if (!fold_slices<3, CPB>(part, n, C, nsplit, a)) return;
  const int idx = n * C + blockIdx.x * CPB + (threadIdx.x % CPB);
  const double mg = a[0] / HW, mgx = a[1] / HW;
  coef[idx] = make_float2((float)mg, (float)mgx);
  const double rstd = stats[2 * idx + 1];
  dbn[idx] = rstd * ((a[0] - HW * mg) - mgx * a[2]);
}


__device__ __forceinline__ void store_planes4(__bf16* __restrict__ pl, long pps, long e, float4 v);

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

// RNE bf16 pair (the split of vst_weight_split / nhwc_to_cp_planes_k)
__device__ __forceinline__ uint32_t bf16_pack2(float a, float b) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef __bf16 b2 __attribute__((ext_vector_type(2)));
  const f2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, b2));
}

// v's three bf16 planes (hi, mid, lo: the RNE split of nhwc_to_cp_planes_k / split8) at element e of planes
// [3][pps] — the NHWC A-operand planes of an x6 data gradient that takes its A operand pre-split (APRE_BWD)
__device__ __forceinline__ void store_planes4(__bf16* __restrict__ pl, long pps, long e, float4 v) {
  float r[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    const uint32_t q0 = bf16_pack2(r[0], r[1]), q1 = bf16_pack2(r[2], r[3]);
    *reinterpret_cast<uint2*>(pl + p * pps + e) = make_uint2(q0, q1);
    if (p < 2) {
      r[0] -= __uint_as_float(q0 << 16);
      r[1] -= __uint_as_float(q0 & 0xffff0000u);
      r[2] -= __uint_as_float(q1 << 16);
      r[3] -= __uint_as_float(q1 & 0xffff0000u);
    }
  }
}

// in_apply_k fused with the weight gradient's A-operand image of the conv that consumes the result:
// a = act(IN(y)) (+ residual) written NHWC (the next conv's input) AND as the padded channel-major
// copy [C][N][H+2p][W+2p] (reflect or zero border; phase: stride-2 column-phase rows) that
// nhwc_to_cp_pad_k would make from a in the backward pass — the backward's read of a and its
// launch are gone.  Walks padded pixels in 64 x 64 LDS tiles (as nhwc_to_cp_pad_k); the interior
// positions also store a.  grid (ceil(N (H+2p)(W+2p+wx) / 64), ceil(C / 64)), 256 threads.
// planes != null: the image goes out as three bf16 planes [3][C][ld] (the RNE split of
// nhwc_to_cp_planes_k) instead of fp32 — the x6 weight gradient's B operand when a is the "output"
// side of the GEMM (tap_wgrad_swap) — and each padded row carries wx more zero columns.
__global__ __launch_bounds__(256) void in_apply_cp_pad_k(const float* __restrict__ x, const float* __restrict__ stats,
                                                          const float* __restrict__ res, float* __restrict__ a,
                                                          float* __restrict__ xt, int N, int H, int W, int C,
                                                          int pad, int reflect, int phase, long ld, int act,
                                                          float slope, int wx = 0, __bf16* __restrict__ planes = nullptr) {
  __shared__ float tile[64][65];
  const int Hp = H + 2 * pad, Wp = W + 2 * pad, Wq = Wp + wx;
  const long P = (long)N * Hp * Wq;
  const long p0 = (long)blockIdx.x * 64;
  const int c0 = blockIdx.y * 64;
  const int t = threadIdx.x;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int idx = t + 256 * it, pr = idx >> 4, c4 = (idx & 15) * 4;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    const long q = p0 + pr;
    if (q < P && c0 + c4 < C) {
      const int n = (int)(q / ((long)Hp * Wq));
      const int rem = (int)(q - (long)n * Hp * Wq);
      int h = rem / Wq - pad, w = rem % Wq;
      const bool xcol = w >= Wp;  // one of the wx zero columns
      if (phase) {
        const int wh = Wp >> 1;
        w = w < wh ? 2 * w : 2 * (w - wh) + 1;
      }
      w -= pad;
      const bool inner = (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
      bool ok = inner;
      if (reflect && !xcol) {
        h = reflect_idx(h, H);
        w = reflect_idx(w, W);
        ok = true;
      }
      if (ok) {
        const long e = (((long)n * H + h) * W + w) * C + c0 + c4;
        const float4 s0 = reinterpret_cast<const float4*>(stats)[((long)n * C + c0 + c4) / 2];
        const float4 s1 = reinterpret_cast<const float4*>(stats)[((long)n * C + c0 + c4) / 2 + 1];
        v = *reinterpret_cast<const float4*>(x + e);
        v.x = apply_act((v.x - s0.x) * s0.y, act, slope);
        v.y = apply_act((v.y - s0.z) * s0.w, act, slope);
        v.z = apply_act((v.z - s1.x) * s1.y, act, slope);
        v.w = apply_act((v.w - s1.z) * s1.w, act, slope);
        if (res) add_f4(v, *reinterpret_cast<const float4*>(res + e));
        if (inner) *reinterpret_cast<float4*>(a + e) = v;
      }
    }
    tile[pr][c4] = v.x;
    tile[pr][c4 + 1] = v.y;
    tile[pr][c4 + 2] = v.z;
    tile[pr][c4 + 3] = v.w;
  }
  __syncthreads();
  if (planes) {
    const long plane = (long)C * ld;
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int idx = t + 256 * it, cr = idx >> 4, p4 = (idx & 15) * 4;
      if (c0 + cr >= C || p0 + p4 >= P) continue;
      float r[4] = {tile[p4][cr], tile[p4 + 1][cr], tile[p4 + 2][cr], tile[p4 + 3][cr]};
      __bf16* dst = planes + (long)(c0 + cr) * ld + p0 + p4;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
        const uint32_t q0 = bf16_pack2(r[0], r[1]), q1 = bf16_pack2(r[2], r[3]);
        if (p0 + p4 + 3 < P) {
          *reinterpret_cast<uint2*>(dst + pl * plane) = make_uint2(q0, q1);
        } else {
          const uint16_t h[4] = {(uint16_t)q0, (uint16_t)(q0 >> 16), (uint16_t)q1, (uint16_t)(q1 >> 16)};
          for (int e = 0; e < 4 && p0 + p4 + e < P; ++e) reinterpret_cast<uint16_t*>(dst + pl * plane)[e] = h[e];
        }
        if (pl < 2) {
          r[0] -= __uint_as_float(q0 << 16);
          r[1] -= __uint_as_float(q0 & 0xffff0000u);
          r[2] -= __uint_as_float(q1 << 16);
          r[3] -= __uint_as_float(q1 & 0xffff0000u);
        }
      }
    }
    return;
  }
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int idx = t + 256 * it, cr = idx >> 4, p4 = (idx & 15) * 4;
    if (c0 + cr >= C || p0 + p4 >= P) continue;
    float* dst = xt + (long)(c0 + cr) * ld + p0 + p4;
    if (p0 + p4 + 3 < P && (ld & 3) == 0) {
      *reinterpret_cast<float4*>(dst) = make_float4(tile[p4][cr], tile[p4 + 1][cr], tile[p4 + 2][cr], tile[p4 + 3][cr]);
    } else {
      for (int e = 0; e < 4 && p0 + p4 + e < P; ++e) dst[e] = tile[p4 + e][cr];
    }
  }
}

__device__ __forceinline__ float in_bwd1(float gy, float x, float mean, float rstd, float2 k, int act,
                                         float slope) {
  const float xh = (x - mean) * rstd;
  float d = 1.f;
  if (act == VST_ACT_RELU) d = xh > 0.f ? 1.f : 0.f;
  else if (act == VST_ACT_LRELU) d = xh > 0.f ? 1.f : slope;
  return rstd * (gy * d - k.x - xh * k.y);
}

// db[c] (+)= sum_n dbn[n][c] in a fixed order (the conv-bias gradient), by the first blocks of the
// apply pass that follows in_bwd_finalize_k (replaces a launch of its own)
__device__ __forceinline__ void in_bias_grad_blocks(const double* __restrict__ dbn, float* __restrict__ db, int N,
                                                    int C, int accumulate, int c) {
  if (c >= C) return;
  double s = 0.0;
  for (int n = 0; n < N; ++n) s += dbn[(long)n * C + c];
  db[c] = accumulate ? db[c] + (float)s : (float)s;
}

__global__ void in_bwd_apply_k(const float4* __restrict__ gy, const float4* __restrict__ x,
                               const float* __restrict__ stats, const float2* __restrict__ coef,
                               float4* __restrict__ dx, long total4, int HW, int C4, int act,
                               float slope, const double* __restrict__ dbn, float* __restrict__ db, int N,
                               int accumulate_db, __bf16* __restrict__ apl = nullptr) {
  if (db && blockIdx.x * blockDim.x < 4 * C4)
    in_bias_grad_blocks(dbn, db, N, 4 * C4, accumulate_db, blockIdx.x * blockDim.x + threadIdx.x);
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
  if (apl)  // dx as its NHWC planes only (the data gradient's pre-split A operand and the NHWC weight gradient's B)
    store_planes4(apl, total4 * 4, i * 4, o);
  else
    dx[i] = o;
}

// in_bwd_apply_k fused with the weight gradient's B-operand image: dx = the IN(+act) input gradient
// written NHWC (the data gradient's A operand) AND as three bf16 planes [3][C][ldp] (hi, mid, lo;
// the RNE split of vst_weight_split / nhwc_to_cp_planes_k) through a 64-pixel x 64-channel LDS
// transpose tile — the conv below the IN consumes dx both ways, so the plane copy's extra read of dx
// is gone.  grid (ceil(P / 64), ceil(C / 64)), 256 threads.

__global__ __launch_bounds__(256) void in_bwd_apply_planes_k(const float* __restrict__ gy, const float* __restrict__ x,
                                                              const float* __restrict__ stats,
                                                              const float2* __restrict__ coef, float* __restrict__ dx,
                                                              __bf16* __restrict__ planes, long P, int HW, int C,
                                                              long ldp, int act, float slope,
                                                              const double* __restrict__ dbn, float* __restrict__ db,
                                                              int N, int accumulate_db, __bf16* __restrict__ apl = nullptr) {
  __shared__ float tile[64][65];
  const long p0 = (long)blockIdx.x * 64;
  const int c0 = blockIdx.y * 64;
  const int t = threadIdx.x;
  if (db && blockIdx.x == 0 && t < 64) in_bias_grad_blocks(dbn, db, N, C, accumulate_db, c0 + t);
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int idx = t + 256 * it, pr = idx >> 4, c4 = (idx & 15) * 4;
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
    const long q = p0 + pr;
    if (q < P && c0 + c4 < C) {
      const long nc = (q / HW) * C + c0 + c4;
      const float4 s0 = reinterpret_cast<const float4*>(stats)[nc / 2];
      const float4 s1 = reinterpret_cast<const float4*>(stats)[nc / 2 + 1];
      const float4 k01 = reinterpret_cast<const float4*>(coef)[nc / 2];
      const float4 k23 = reinterpret_cast<const float4*>(coef)[nc / 2 + 1];
      const float4 g = *reinterpret_cast<const float4*>(gy + q * C + c0 + c4);
      const float4 v = *reinterpret_cast<const float4*>(x + q * C + c0 + c4);
      o.x = in_bwd1(g.x, v.x, s0.x, s0.y, make_float2(k01.x, k01.y), act, slope);
      o.y = in_bwd1(g.y, v.y, s0.z, s0.w, make_float2(k01.z, k01.w), act, slope);
      o.z = in_bwd1(g.z, v.z, s1.x, s1.y, make_float2(k23.x, k23.y), act, slope);
      o.w = in_bwd1(g.w, v.w, s1.z, s1.w, make_float2(k23.z, k23.w), act, slope);
      if (apl) store_planes4(apl, P * C, q * C + c0 + c4, o);  // dx as its NHWC planes only
      else *reinterpret_cast<float4*>(dx + q * C + c0 + c4) = o;
    }
    tile[pr][c4] = o.x;
    tile[pr][c4 + 1] = o.y;
    tile[pr][c4 + 2] = o.z;
    tile[pr][c4 + 3] = o.w;
  }
  __syncthreads();
  const long plane = (long)C * ldp;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int idx = t + 256 * it, cr = idx >> 4, p4 = (idx & 15) * 4;
    if (c0 + cr >= C || p0 + p4 >= P) continue;
    float r[4] = {tile[p4][cr], tile[p4 + 1][cr], tile[p4 + 2][cr], tile[p4 + 3][cr]};
    __bf16* dst = planes + (long)(c0 + cr) * ldp + p0 + p4;
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) {
      const uint32_t q0 = bf16_pack2(r[0], r[1]), q1 = bf16_pack2(r[2], r[3]);
      if (p0 + p4 + 3 < P) {
        *reinterpret_cast<uint2*>(dst + pl * plane) = make_uint2(q0, q1);
      } else {
        const uint16_t h[4] = {(uint16_t)q0, (uint16_t)(q0 >> 16), (uint16_t)q1, (uint16_t)(q1 >> 16)};
        for (int e = 0; e < 4 && p0 + p4 + e < P; ++e) reinterpret_cast<uint16_t*>(dst + pl * plane)[e] = h[e];
      }
      if (pl < 2) {
        r[0] -= __uint_as_float(q0 << 16);
        r[1] -= __uint_as_float(q0 & 0xffff0000u);
        r[2] -= __uint_as_float(q1 << 16);
        r[3] -= __uint_as_float(q1 & 0xffff0000u);
      }
    }
  }
}

__global__ void act_bwd_k(const float* __restrict__ gy, const float* __restrict__ y,
                          float* __restrict__ dx, long n, int act, float slope) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dx[i] = gy[i] * act_grad_from_out(y[i], act, slope);
}

// per-channel sum (bias gradient of a layer without a following IN), same geometry as in_partial.
// Channels wider than 4*NRED run as chunks of LP float4 lanes: chunk lanes [c4off, c4off + nl) of a
// row of CS4 float4s; part rows are CS4*4 doubles wide so one final pass folds every chunk.
__global__ __launch_bounds__(NRED) void chsum_partial_k(const float* __restrict__ x,
                                                        double* __restrict__ part, long NHW, int LP,
                                                        int PG, int SP, int CS4, int c4off, int nl) {
  __shared__ double red[4][NRED];
  const int t = threadIdx.x, c4 = t % LP, pg = t / LP;
  const long p0 = (long)blockIdx.x * SP, p1 = min(NHW, p0 + SP);
  double acc[4] = {0, 0, 0, 0};
  const float4* xb = reinterpret_cast<const float4*>(x) + c4off + c4;
  for (long p = p0 + pg; pg < PG && c4 < nl && p < p1; p += PG) {
    const float4 v = xb[p * CS4];
    acc[0] += v.x; acc[1] += v.y; acc[2] += v.z; acc[3] += v.w;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) red[j][t] = acc[j];
  __syncthreads();
  if (pg == 0 && c4 < nl)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      double s = 0.0;
      for (int q = 0; q < PG; ++q) s += red[j][q * LP + c4];
      part[(long)blockIdx.x * CS4 * 4 + 4 * (c4off + c4) + j] = s;
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


// ---- affine InstanceNorm (nn.InstanceNorm2d(affine=True), learning-based network.py:147-261) ---
// y = s * act(gamma[c] * xhat + beta[c]) + residual, xhat = (x - mean) * rstd, computed as ATen's
// CPU batch-norm transform does: z = x * alpha + (beta - mean * alpha), alpha = rstd * gamma.
// s = 1, or the ResidualBlock gate s = 2|u| / (1 + |u|), u = gate_mult * gate[0]
// (network.py:241-245 layer_strength).
__device__ __forceinline__ float gate_scale(const float* gate, float mult) {
  if (!gate) return 1.f;
  const float u = fabsf(mult * gate[0]);
  return 2.f * u / (1.f + u);
}

__global__ void in_aff_apply_k(const float4* __restrict__ x, const float* __restrict__ stats,
                               const float* __restrict__ gamma, const float* __restrict__ beta,
                               const float* __restrict__ gate, float gate_mult,
                               const float4* __restrict__ res, float4* __restrict__ y, long total4,
                               int HW, int C4, int act, float slope) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total4) return;
  const int c4 = i % C4;
  const int n = (i / C4) / HW;
  const float sc = gate_scale(gate, gate_mult);
  const float* st = stats + ((long)n * C4 + c4) * 8;
  const float4 v = x[i];
  const float xv[4] = {v.x, v.y, v.z, v.w};
  float o[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = 4 * c4 + j;
    const float al = st[2 * j + 1] * gamma[c];
    const float be = beta[c] - st[2 * j] * al;
    float z = apply_act(xv[j] * al + be, act, slope);
    o[j] = gate ? sc * z : z;
  }
  float4 r = make_float4(o[0], o[1], o[2], o[3]);
  if (res) add_f4(r, res[i]);
  y[i] = r;
}

// backward partials per (n, c) slice: {sum gz, sum gz*xhat, sum xhat, sum gy*a},
// gz = s * gy * act'(z), a = act(z) (the gate-input activation)
__global__ __launch_bounds__(NRED) void in_aff_partial_k(const float* __restrict__ x,
                                                         const float* __restrict__ gy,
                                                         const float* __restrict__ stats,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ beta,
                                                         const float* __restrict__ gate, float gate_mult,
                                                         double* __restrict__ part, int HW, int C,
                                                         int LP, int PG, int SP, int nsplit, int act,
                                                         float slope) {
  constexpr int NV = 4;
  __shared__ double red[NV * 4][NRED];
  const int t = threadIdx.x, c4 = t % LP, pg = t / LP;
  const int n = blockIdx.y, z = blockIdx.x;
  const int p0 = z * SP, p1 = min(HW, p0 + SP);
  const float sc = gate_scale(gate, gate_mult);
  double acc[NV][4];
#pragma unroll
  for (int v = 0; v < NV; ++v)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[v][j] = 0.0;
  float mean[4], rstd[4], ga[4], be[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = 4 * c4 + j < C ? 4 * c4 + j : 0;
    mean[j] = stats[2 * ((long)n * C + c)];
    rstd[j] = stats[2 * ((long)n * C + c) + 1];
    ga[j] = gamma[c];
    be[j] = beta[c];
  }
  const float4* xb = reinterpret_cast<const float4*>(x) + (long)n * HW * LP + c4;
  const float4* gb = reinterpret_cast<const float4*>(gy) + (long)n * HW * LP + c4;
  for (int p = p0 + pg; pg < PG && p < p1; p += PG) {
    const float4 v = xb[(long)p * LP];
    const float4 gv = gb[(long)p * LP];
    const float xv[4] = {v.x, v.y, v.z, v.w};
    const float gg[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float xh = (xv[j] - mean[j]) * rstd[j];
      const float al = rstd[j] * ga[j];
      const float zz = xv[j] * al + (be[j] - mean[j] * al);
      float d = 1.f;
      if (act == VST_ACT_RELU) d = zz > 0.f ? 1.f : 0.f;
      else if (act == VST_ACT_LRELU) d = zz > 0.f ? 1.f : slope;
      const float g = sc * gg[j] * d;
      acc[0][j] += g;
      acc[1][j] += (double)g * xh;
      acc[2][j] += xh;
      acc[3][j] += (double)gg[j] * apply_act(zz, act, slope);
    }
  }
#pragma unroll
  for (int v = 0; v < NV; ++v)
#pragma unroll
    for (int j = 0; j < 4; ++j) red[v * 4 + j][t] = acc[v][j];
  __syncthreads();
  if (pg == 0) {
    double* dst = part + (((long)n * nsplit + z) * C + 4 * c4) * NV;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        double s = 0.0;
        for (int q = 0; q < PG; ++q) s += red[v * 4 + j][q * LP + c4];
        dst[j * NV + v] = s;
      }
  }
}

// coef[n*C+c] = {mean gz, mean gz*xhat}; sums[n*C+c] = {sum gz, sum gz*xhat, sum gy*a, dbias}
__global__ void in_aff_finalize_k(const double* __restrict__ part, const float* __restrict__ stats,
                                  const float* __restrict__ gamma, float2* __restrict__ coef,
                                  double* __restrict__ sums, int N, int HW, int C, int nsplit) {
  double a[4];
  const int n = blockIdx.y;
  if (!fold_slices<4>(part, n, C, nsplit, a)) return;
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int idx = n * C + c;
  const double mg = a[0] / HW, mgx = a[1] / HW;
  coef[idx] = make_float2((float)mg, (float)mgx);
  const double rstd = stats[2 * idx + 1];
  sums[4 * idx + 0] = a[0];
  sums[4 * idx + 1] = a[1];
  sums[4 * idx + 2] = a[3];
  sums[4 * idx + 3] = rstd * gamma[c] * ((a[0] - HW * mg) - mgx * a[2]);
}

// one block: dgamma/dbeta/dbias per channel (sum over n, fixed order) and the gate gradient
__global__ void in_aff_param_grad_k(const double* __restrict__ sums, float* __restrict__ dgamma,
                                    float* __restrict__ dbeta, float* __restrict__ dbias,
                                    const float* __restrict__ gate, float gate_mult,
                                    float* __restrict__ dgate, int N, int C, int accumulate) {
  __shared__ double red[4];
  double ds = 0.0;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    double sg = 0.0, sgx = 0.0, sb = 0.0;
    for (int n = 0; n < N; ++n) {
      const double* q = sums + 4 * ((long)n * C + c);
      sg += q[0];
      sgx += q[1];
      ds += q[2];
      sb += q[3];
    }
    if (dgamma) dgamma[c] = accumulate ? dgamma[c] + (float)sgx : (float)sgx;
    if (dbeta) dbeta[c] = accumulate ? dbeta[c] + (float)sg : (float)sg;
    if (dbias) dbias[c] = accumulate ? dbias[c] + (float)sb : (float)sb;
  }
  if (!gate || !dgate) return;
  ds = wave_sum_d(ds);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ds;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double tot = red[0] + red[1] + red[2] + red[3];
    const float u = gate_mult * gate[0];
    const float au = fabsf(u);
    const float du = 2.f / ((1.f + au) * (1.f + au)) * (u > 0.f ? 1.f : (u < 0.f ? -1.f : 0.f));
    const float g = (float)tot * du * gate_mult;
    dgate[0] = accumulate ? dgate[0] + g : g;
  }
}

__global__ void in_aff_bwd_apply_k(const float4* __restrict__ gy, const float4* __restrict__ x,
                                   const float* __restrict__ stats, const float* __restrict__ gamma,
                                   const float* __restrict__ beta, const float* __restrict__ gate,
                                   float gate_mult, const float2* __restrict__ coef,
                                   float4* __restrict__ dx, long total4, int HW, int C4, int act,
                                   float slope) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total4) return;
  const int c4 = i % C4;
  const int n = (i / C4) / HW;
  const float sc = gate_scale(gate, gate_mult);
  const long nc = (long)n * C4 * 4 + 4 * c4;
  const float4 g4 = gy[i], v = x[i];
  const float gg[4] = {g4.x, g4.y, g4.z, g4.w}, xv[4] = {v.x, v.y, v.z, v.w};
  float o[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = 4 * c4 + j;
    const float mean = stats[2 * (nc + j)], rstd = stats[2 * (nc + j) + 1];
    const float al = rstd * gamma[c];
    const float zz = xv[j] * al + (beta[c] - mean * al);
    float d = 1.f;
    if (act == VST_ACT_RELU) d = zz > 0.f ? 1.f : 0.f;
    else if (act == VST_ACT_LRELU) d = zz > 0.f ? 1.f : slope;
    const float g = sc * gg[j] * d;
    const float xh = (xv[j] - mean) * rstd;
    const float2 k = coef[nc + j];
    o[j] = al * (g - k.x - xh * k.y);
  }
  dx[i] = make_float4(o[0], o[1], o[2], o[3]);
}


// ---- running statistics (nn.InstanceNorm2d(track_running_stats=True), StarGAN model.py:13-16) ---
// ATen instance_norm: batch_norm over (1, N*C, HW) with the running buffers repeated N times, then
// the N copies averaged: rm = (1-m) rm + m * mean_n(mean_nc); rv = (1-m) rv + m * mean_n(var_nc *
// HW/(HW-1)) (unbiased).  var_nc is recovered from rstd: 1/rstd^2 - eps.
__global__ void in_running_update_k(const float* __restrict__ stats, float* __restrict__ rm,
                                    float* __restrict__ rv, int N, int C, int HW, float momentum,
                                    float eps) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double sm = 0.0, sv = 0.0;
  const double unb = HW > 1 ? (double)HW / (HW - 1) : 1.0;
  for (int n = 0; n < N; ++n) {
    const float mean = stats[2 * ((long)n * C + c)], rstd = stats[2 * ((long)n * C + c) + 1];
    const double var = 1.0 / ((double)rstd * rstd) - eps;
    sm += (1.0 - momentum) * rm[c] + (double)momentum * mean;
    sv += (1.0 - momentum) * rv[c] + (double)momentum * var * unb;
  }
  rm[c] = (float)(sm / N);
  rv[c] = (float)(sv / N);
}

// eval mode: stats[n][c] = {running_mean, 1/sqrt(running_var + eps)} for every n
__global__ void in_stats_from_running_k(const float* __restrict__ rm, const float* __restrict__ rv,
                                        float* __restrict__ stats, int N, int C, float eps) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)N * C) return;
  const int c = i % C;
  stats[2 * i] = rm[c];
  stats[2 * i + 1] = 1.f / sqrtf(rv[c] + eps);
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
  if (fin_cpb(C, N, g.nsplit) == 4)
    hipLaunchKernelGGL(in_finalize_k<4>, dim3(ceil_div(C, 4), N), dim3(256), 0, s, part, stats, N, HW, C, g.nsplit, eps);
  else
    hipLaunchKernelGGL(in_finalize_k<16>, dim3(ceil_div(C, 16), N), dim3(256), 0, s, part, stats, N, HW, C, g.nsplit,
                       eps);
  return check_launch("instnorm_stats");
}

extern "C" int vst_instnorm_finalize(const double* part, float* stats, int N, int HW, int C, int nsplit,
                                     float eps, void* stream) {
  VST_REQUIRE(part && stats && N > 0 && HW > 0 && C > 0 && nsplit > 0, "instnorm_finalize: bad args");
  if (fin_cpb(C, N, nsplit) == 4)
    hipLaunchKernelGGL(in_finalize_k<4>, dim3(ceil_div(C, 4), N), dim3(256), 0, (hipStream_t)stream, part, stats, N,
                       HW, C, nsplit, eps);
  else
    hipLaunchKernelGGL(in_finalize_k<16>, dim3(ceil_div(C, 16), N), dim3(256), 0, (hipStream_t)stream, part, stats,
                       N, HW, C, nsplit, eps);
  return check_launch("instnorm_finalize");
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

extern "C" int vst_instnorm_act_bwd_planes(const float* gy, const float* x, const float* stats, float* dx,
                                           float* db, float* ws, int N, int HW, int C, int act, float slope,
                                           int accumulate_db, void* planes, long ldp, void* stream);

extern "C" int vst_instnorm_act_fwd_cp(const float* x, const float* stats, const float* residual, float* y,
                                       float* xt, int N, int H, int W, int C, int act, float slope, int pad,
                                       int pad_mode, int stride, void* stream) {
  VST_REQUIRE(x && stats && y && xt && C % 4 == 0 && pad >= 0 && (stride == 1 || stride == 2),
              "instnorm_act_fwd_cp: bad args");
  VST_REQUIRE(pad_mode == VST_PAD_ZERO || (pad < H && pad < W), "instnorm_act_fwd_cp: reflect pad >= size");
  VST_REQUIRE(stride == 1 || (W + 2 * pad) % 2 == 0, "instnorm_act_fwd_cp: stride 2 needs W + 2 pad even");
  const long P = (long)N * (H + 2 * pad) * (W + 2 * pad);
  hipLaunchKernelGGL(in_apply_cp_pad_k, dim3(ceil_div(P, 64), ceil_div(C, 64)), dim3(256), 0, (hipStream_t)stream,
                     x, stats, residual, y, xt, N, H, W, C, pad, pad_mode == VST_PAD_REFLECT, stride == 2,
                     rk_cp_ld(P), act, slope);
  return check_launch("instnorm_act_fwd_cp");
}

extern "C" int vst_instnorm_act_fwd_planes(const float* x, const float* stats, const float* residual, float* y,
                                           void* planes, int N, int H, int W, int C, int act, float slope, int pad,
                                           int pad_mode, int wx, void* stream) {
  VST_REQUIRE(x && stats && y && planes && C % 4 == 0 && pad >= 0 && wx >= 0, "instnorm_act_fwd_planes: bad args");
  VST_REQUIRE(pad_mode == VST_PAD_ZERO || (pad < H && pad < W), "instnorm_act_fwd_planes: reflect pad >= size");
  const long P = (long)N * (H + 2 * pad) * (W + 2 * pad + wx);
  hipLaunchKernelGGL(in_apply_cp_pad_k, dim3(ceil_div(P, 64), ceil_div(C, 64)), dim3(256), 0, (hipStream_t)stream,
                     x, stats, residual, y, nullptr, N, H, W, C, pad, pad_mode == VST_PAD_REFLECT, 0, rk_cp_ld(P), act,
                     slope, wx, reinterpret_cast<__bf16*>(planes));
  return check_launch("instnorm_act_fwd_planes");
}

extern "C" int vst_instnorm_act_bwd(const float* gy, const float* x, const float* stats, float* dx,
                                    float* db, float* ws, int N, int HW, int C, int act, float slope,
                                    int accumulate_db, void* stream) {
  return vst_instnorm_act_bwd_planes(gy, x, stats, dx, db, ws, N, HW, C, act, slope, accumulate_db, nullptr,
                                     0, stream);
}

// IN backward after its partials are in ws: finalize, bias gradient, apply (+ planes).
static int in_bwd_tail(const float* gy, const float* x, const float* stats, float* dx, float* db, float* ws,
                       int N, int HW, int C, int act, float slope, int accumulate_db, void* planes, long ldp,
                       const RedGeom& g, hipStream_t s, void* apl = nullptr);

extern "C" int vst_instnorm_act_bwd_planes(const float* gy, const float* x, const float* stats, float* dx,
                                           float* db, float* ws, int N, int HW, int C, int act, float slope,
                                           int accumulate_db, void* planes, long ldp, void* stream) {
  RedGeom g;
  VST_REQUIRE(gy && x && stats && dx && ws && red_geom(N, HW, C, g), "instnorm_act_bwd: bad args");
  VST_REQUIRE(!planes || ldp >= (long)N * HW, "instnorm_act_bwd: plane stride %ld < N*HW", ldp);
  hipStream_t s = (hipStream_t)stream;
  double* part = reinterpret_cast<double*>(ws);
  hipLaunchKernelGGL(in_partial_k<1>, dim3(g.nsplit, N), dim3(NRED), 0, s, x, gy, stats, part, HW, C,
                     g.LP, g.PG, g.SP, g.nsplit, act, slope);
  return in_bwd_tail(gy, x, stats, dx, db, ws, N, HW, C, act, slope, accumulate_db, planes, ldp, g, s);
}

// vst_instnorm_act_bwd_planes that writes dx ONLY as its NHWC bf16 planes apl [3][N*HW*C] (the A operand of the x6
// data gradient that consumes dx, pre-split: vst_conv2d_dgrad_refl_epi_part's apl; and the B operand of
// vst_conv2d_wgrad_nhwc) — with planes (!= NULL) the channel-major planes [3][C][ldp] too, without them none
extern "C" int vst_instnorm_act_bwd_planes_apre(const float* gy, const float* x, const float* stats, float* dx,
                                                float* db, float* ws, int N, int HW, int C, int act, float slope,
                                                int accumulate_db, void* planes, long ldp, void* apl, void* stream) {
  RedGeom g;
  VST_REQUIRE(gy && x && stats && dx && ws && apl && red_geom(N, HW, C, g), "instnorm_act_bwd_apre: bad args");
  VST_REQUIRE(!planes || ldp >= (long)N * HW, "instnorm_act_bwd_apre: plane stride %ld < N*HW", ldp);
  hipStream_t s = (hipStream_t)stream;
  double* part = reinterpret_cast<double*>(ws);
  hipLaunchKernelGGL(in_partial_k<1>, dim3(g.nsplit, N), dim3(NRED), 0, s, x, gy, stats, part, HW, C,
                     g.LP, g.PG, g.SP, g.nsplit, act, slope);
  return in_bwd_tail(gy, x, stats, dx, db, ws, N, HW, C, act, slope, accumulate_db, planes, ldp, g, s, apl);
}

// ReflectionPad2d(1) + 3x3 conv data gradient (vst_conv2d_dgrad_refl) and the InstanceNorm(+act) backward of the
// layer below it, with the IN-backward partials taken by the data gradient itself: the interior GEMM's epilogue
// (per 32-row group) and the border add (its correction slices) write them, so no partial pass (a read of g and z
// and a launch) is needed; then the finalize / apply (+ dy planes).  Workspace: the
// IN partials [N][ns][C][3] + coefficients, then the data gradient's.  x6 arithmetic, H W % 32 == 0.
static size_t in_epi_ws_bytes_al(int N, int H, int W, int C) {
  const size_t ns = bf_dgrad_refl1_inb_slices(H, W);
  return ((size_t)N * ns * C * 3 * sizeof(double) + (size_t)N * C * (sizeof(float2) + sizeof(double)) + 256 + 255) /
         256 * 256;
}

extern "C" size_t vst_conv2d_dgrad_refl_in_epi_ws_bytes(int N, int H, int W, int Cy, int Cx, int math) {
  if (Cx % 4 || !bf_dgrad_refl1_inb_ok(N, H, W, Cy, Cx, math)) return 0;
  return in_epi_ws_bytes_al(N, H, W, Cx) + bf_dgrad_refl1_ws_floats(N, H, W, Cy, Cx, math) * sizeof(float);
}

// the two halves (the data gradient can then be timed on its own): the data gradient + partials, the tail
extern "C" int vst_conv2d_dgrad_refl_epi_part(const float* dy, const void* dy_apl, const void* wsplit,
                                              const float* addend, float* gout, const float* x, const float* stats,
                                              float* ws, size_t ws_bytes, int N, int H, int W, int Cy, int Cx, int act,
                                              float slope, int math, void* stream) {
  const size_t need = vst_conv2d_dgrad_refl_in_epi_ws_bytes(N, H, W, Cy, Cx, math);
  VST_REQUIRE(dy && wsplit && gout && x && stats && ws, "conv2d_dgrad_refl_in_epi: null pointer");
  VST_REQUIRE(need > 0 && ws_bytes >= need,
              "conv2d_dgrad_refl_in_epi: unsupported shape or workspace too small (%zu of %zu bytes)", ws_bytes, need);
  const size_t inb = in_epi_ws_bytes_al(N, H, W, Cx);
  float* dws = reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + inb);
  return bf_dgrad_refl1_inb_launch(dy, wsplit, (long)Cx * 9 * Cy, addend, gout, N, H, W, Cy, Cx, math,
                                   (hipStream_t)stream, dws, (ws_bytes - inb) / sizeof(float), x, stats,
                                   reinterpret_cast<double*>(ws), act, slope, reinterpret_cast<const __bf16*>(dy_apl),
                                   (long)N * H * W * Cy);
}

extern "C" int vst_instnorm_act_bwd_epi_tail(const float* gout, const float* x, const float* stats, float* dx,
                                             float* db, float* ws, int N, int H, int W, int Cx, int act, float slope,
                                             int accumulate_db, void* planes, long ldp, void* apl, void* stream) {
  VST_REQUIRE(gout && x && stats && dx && ws && Cx % 4 == 0 && (H * W) % 32 == 0, "instnorm_act_bwd_epi_tail: bad args");
  VST_REQUIRE(!planes || ldp >= (long)N * H * W, "instnorm_act_bwd_epi_tail: plane stride %ld < N*HW", ldp);
  RedGeom g{};
  g.nsplit = bf_dgrad_refl1_inb_slices(H, W);
  return in_bwd_tail(gout, x, stats, dx, db, ws, N, H * W, Cx, act, slope, accumulate_db, planes, ldp, g,
                     (hipStream_t)stream, apl);
}

extern "C" int vst_conv2d_dgrad_refl_in_epi(const float* dy, const void* wsplit, const float* addend, float* gout,
                                            const float* x, const float* stats, float* dx, float* db, float* ws,
                                            size_t ws_bytes, int N, int H, int W, int Cy, int Cx, int act, float slope,
                                            int accumulate_db, void* planes, long ldp, int math, void* stream) {
  VST_REQUIRE(dx, "conv2d_dgrad_refl_in_epi: null pointer");
  if (int e = vst_conv2d_dgrad_refl_epi_part(dy, nullptr, wsplit, addend, gout, x, stats, ws, ws_bytes, N, H, W, Cy,
                                             Cx, act, slope, math, stream))
    return e;
  return vst_instnorm_act_bwd_epi_tail(gout, x, stats, dx, db, ws, N, H, W, Cx, act, slope, accumulate_db, planes, ldp,
                                       nullptr, stream);
}

static int in_bwd_tail(const float* gy, const float* x, const float* stats, float* dx, float* db, float* ws,
                       int N, int HW, int C, int act, float slope, int accumulate_db, void* planes, long ldp,
                       const RedGeom& g, hipStream_t s, void* apl) {
  double* part = reinterpret_cast<double*>(ws);
  float2* coef = reinterpret_cast<float2*>(reinterpret_cast<char*>(ws) +
                                           (size_t)N * g.nsplit * C * 3 * sizeof(double));
  double* dbn = reinterpret_cast<double*>(reinterpret_cast<char*>(coef) + (size_t)N * C * sizeof(float2));
  if (fin_cpb(C, N, g.nsplit) == 4)
    hipLaunchKernelGGL(in_bwd_finalize_k<4>, dim3(ceil_div(C, 4), N), dim3(256), 0, s, part, stats, coef, dbn,
                     N, HW, C, g.nsplit);
  else
    hipLaunchKernelGGL(in_bwd_finalize_k<16>, dim3(ceil_div(C, 16), N), dim3(256), 0, s, part, stats, coef, dbn,
                     N, HW, C, g.nsplit);
  // the bias gradient (sum over n of dbn) is taken by the apply pass's first blocks
  if (planes) {
    const long P = (long)N * HW;
    hipLaunchKernelGGL(in_bwd_apply_planes_k, dim3(ceil_div(P, 64), ceil_div(C, 64)), dim3(256), 0, s, gy, x, stats,
                       coef, dx, reinterpret_cast<__bf16*>(planes), P, HW, C, ldp, act, slope, dbn, db, N,
                       accumulate_db, reinterpret_cast<__bf16*>(apl));
    return check_launch("instnorm_act_bwd_planes");
  }
  const long total4 = (long)N * HW * C / 4;
  VST_REQUIRE(!db || total4 >= C, "instnorm_act_bwd: fewer elements than channels");
  hipLaunchKernelGGL(in_bwd_apply_k, dim3(ceil_div(total4, 256)), dim3(256), 0, s,
                     reinterpret_cast<const float4*>(gy), reinterpret_cast<const float4*>(x), stats,
                     coef, reinterpret_cast<float4*>(dx), total4, HW, C / 4, act, slope, dbn, db, N,
                     accumulate_db, reinterpret_cast<__bf16*>(apl));
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
  if (Cs % 4 || !red_geom(1, (int)NHW, std::min(Cs, 4 * NRED), g)) return 0;
  return (size_t)g.nsplit * Cs * sizeof(double);
}

extern "C" int vst_channel_sum(const float* x, float* db, float* ws, long NHW, int Cs, int Cl,
                               int accumulate, void* stream) {
  RedGeom g;
  VST_REQUIRE(x && db && ws && Cl <= Cs && NHW > 0 && Cs % 4 == 0 &&
                  red_geom(1, (int)NHW, std::min(Cs, 4 * NRED), g),
              "channel_sum: bad args");
  hipStream_t s = (hipStream_t)stream;
  double* part = reinterpret_cast<double*>(ws);
  const int cs4 = Cs / 4;
  for (int c4off = 0; c4off < cs4; c4off += g.LP)
    hipLaunchKernelGGL(chsum_partial_k, dim3(g.nsplit), dim3(NRED), 0, s, x, part, NHW, g.LP, g.PG, g.SP, cs4,
                       c4off, std::min(g.LP, cs4 - c4off));
  hipLaunchKernelGGL(chsum_final_k, dim3(ceil_div(Cs, 64)), dim3(256), 0, s, part, db, g.nsplit, Cs, Cl,
                     accumulate);
  return check_launch("channel_sum");
}

extern "C" size_t vst_instnorm_affine_ws_bytes(int N, int HW, int C) {
  RedGeom g;
  if (!red_geom(N, HW, C, g)) return 0;
  return (size_t)N * g.nsplit * C * 4 * sizeof(double) + (size_t)N * C * (sizeof(float2) + 4 * sizeof(double)) +
         256;
}

extern "C" int vst_instnorm_affine_fwd(const float* x, const float* stats, const float* gamma,
                                       const float* beta, const float* gate, float gate_mult,
                                       const float* residual, float* y, int N, int HW, int C, int act,
                                       float slope, void* stream) {
  VST_REQUIRE(x && stats && gamma && beta && y && C % 4 == 0 && N > 0 && HW > 0,
              "instnorm_affine_fwd: bad args");
  const long total4 = (long)N * HW * C / 4;
  hipLaunchKernelGGL(in_aff_apply_k, dim3(ceil_div(total4, 256)), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const float4*>(x), stats, gamma, beta, gate, gate_mult,
                     reinterpret_cast<const float4*>(residual), reinterpret_cast<float4*>(y), total4, HW,
                     C / 4, act, slope);
  return check_launch("instnorm_affine_fwd");
}

extern "C" int vst_instnorm_affine_bwd(const float* gy, const float* x, const float* stats,
                                       const float* gamma, const float* beta, const float* gate,
                                       float gate_mult, float* dx, float* dgamma, float* dbeta,
                                       float* dgate, float* dbias, float* ws, int N, int HW, int C,
                                       int act, float slope, int accumulate, void* stream) {
  RedGeom g;
  VST_REQUIRE(gy && x && stats && gamma && beta && dx && ws && red_geom(N, HW, C, g),
              "instnorm_affine_bwd: bad args (C must be 4*2^k <= 1024)");
  hipStream_t s = (hipStream_t)stream;
  double* part = reinterpret_cast<double*>(ws);
  char* p = reinterpret_cast<char*>(ws) + (size_t)N * g.nsplit * C * 4 * sizeof(double);
  float2* coef = reinterpret_cast<float2*>(p);
  double* sums = reinterpret_cast<double*>(p + (size_t)N * C * sizeof(float2));
  hipLaunchKernelGGL(in_aff_partial_k, dim3(g.nsplit, N), dim3(NRED), 0, s, x, gy, stats, gamma, beta,
                     gate, gate_mult, part, HW, C, g.LP, g.PG, g.SP, g.nsplit, act, slope);
  hipLaunchKernelGGL(in_aff_finalize_k, dim3(ceil_div(C, 64), N), dim3(256), 0, s, part, stats, gamma,
                     coef, sums, N, HW, C, g.nsplit);
  hipLaunchKernelGGL(in_aff_param_grad_k, dim3(1), dim3(256), 0, s, sums, dgamma, dbeta, dbias, gate,
                     gate_mult, dgate, N, C, accumulate);
  const long total4 = (long)N * HW * C / 4;
  hipLaunchKernelGGL(in_aff_bwd_apply_k, dim3(ceil_div(total4, 256)), dim3(256), 0, s,
                     reinterpret_cast<const float4*>(gy), reinterpret_cast<const float4*>(x), stats, gamma,
                     beta, gate, gate_mult, coef, reinterpret_cast<float4*>(dx), total4, HW, C / 4, act,
                     slope);
  return check_launch("instnorm_affine_bwd");
}

extern "C" int vst_instnorm_running_update(const float* stats, float* running_mean, float* running_var,
                                           int N, int C, int HW, float momentum, float eps,
                                           void* stream) {
  VST_REQUIRE(stats && running_mean && running_var && N > 0 && C > 0, "instnorm_running_update: bad args");
  hipLaunchKernelGGL(in_running_update_k, dim3(ceil_div(C, 256)), dim3(256), 0, (hipStream_t)stream, stats,
                     running_mean, running_var, N, C, HW, momentum, eps);
  return check_launch("instnorm_running_update");
}

extern "C" int vst_instnorm_stats_from_running(const float* running_mean, const float* running_var,
                                               float* stats, int N, int C, float eps, void* stream) {
  VST_REQUIRE(running_mean && running_var && stats && N > 0 && C > 0, "instnorm_stats_from_running: bad args");
  hipLaunchKernelGGL(in_stats_from_running_k, dim3(ceil_div((long)N * C, 256)), dim3(256), 0,
                     (hipStream_t)stream, running_mean, running_var, stats, N, C, eps);
  return check_launch("instnorm_stats_from_running");
}
