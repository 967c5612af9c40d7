// Tap-GEMM form of the convolutions with 4 (padded) output channels — the generators' last layer
// (c7s1-3 + tanh, CycleGAN networks.py:365-367; StarGAN model.py:53-54; MoGAN's motion nets).
//
// A 4-wide output makes the implicit GEMM N = 4: a 32x32 MFMA tile would be 1/8 useful, so the
// direct form ran on the VALU at ~10 TFLOP/s.  Instead the contraction over input channels runs
// first for every tap at once, as a 1x1 conv with N = R*S*4 on the MFMA fprop kernel:
//     Z[q][(r,s,co)] = sum_ci x[q][ci] * w[co][ci][r][s]            (weights = VST_PACK_CK pack)
// and the taps are summed afterwards by a gather over source pixels:
//     y[p][co] = act(bias[co] + sum_{r,s} Z[src(p, r, s)][(r,s,co)])  (vst_tapsum_fwd)
// The weight gradient mirrors it: the adjoint of the gather folds dy into
//     D[q][(r,s,co)] = sum_{p : src(p,r,s) = q} dy[p][co]            (vst_tapfold)
// (with reflect padding a source pixel can be hit by up to 2 positions per axis), the MFMA wgrad
// kernel contracts D with x over pixels (a 1x1 wgrad, M = R*S*4, N = Ci), and vst_tap_wgrad_scatter
// writes the [R*S*4][Ci] result back into the [Co][Ci][R][S] gradient.
// Streaming kernels; Z / D are N*H*W*R*S*16 bytes, each element written once and read once.
#include "common.h"

namespace vst {

__device__ __forceinline__ int src_index(int x, int n, int reflect) {
  if (!reflect) return (x >= 0 && x < n) ? x : -1;
  if (x < 0) return -x;
  if (x >= n) return 2 * (n - 1) - x;
  return x;
}

__global__ void tapsum_k(const float4* __restrict__ z, int zcs4, const float* __restrict__ bias,
                         float4* __restrict__ y, int H, int W, int R, int S, int pad, int reflect, int act,
                         float slope, long P) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const int w = p % W;
  const long t = p / W;
  const int h = t % H;
  const long n = t / H;
  float4 acc = bias ? make_float4(bias[0], bias[1], bias[2], bias[3]) : make_float4(0.f, 0.f, 0.f, 0.f);
  for (int r = 0; r < R; ++r) {
    const int hh = src_index(h + r - pad, H, reflect);
    if (hh < 0) continue;
    const float4* zr = z + ((n * H + hh) * (long)W) * zcs4 + r * S;
    for (int s = 0; s < S; ++s) {
      const int ww = src_index(w + s - pad, W, reflect);
      if (ww < 0) continue;
      const float4 v = zr[(long)ww * zcs4 + s];
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
  }
  y[p] = make_float4(apply_act(acc.x, act, slope), apply_act(acc.y, act, slope), apply_act(acc.z, act, slope),
                     apply_act(acc.w, act, slope));
}

// preimages along one axis: positions pos in [0, n) with src_index(pos + k - pad) == q (k = tap)
__device__ __forceinline__ int preimages(int q, int k, int pad, int n, int reflect, int (&out)[3]) {
  const int cand[3] = {q - k + pad, pad - k - q, 2 * (n - 1) - q - k + pad};
  int m = 0;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int c = cand[j];
    if (c < 0 || c >= n) continue;
    if (src_index(c + k - pad, n, reflect) != q) continue;
    bool dup = false;
    for (int e = 0; e < m; ++e) dup |= out[e] == c;
    if (!dup) out[m++] = c;
  }
  return m;
}

__global__ void tapfold_k(const float4* __restrict__ g, float4* __restrict__ d, int H, int W, int R, int S,
                          int pad, int reflect, long total) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int RS = R * S;
  const int rs = i % RS;
  const long q = i / RS;
  const int qw = q % W;
  const long t = q / W;
  const int qh = t % H;
  const long n = t / H;
  const int r = rs / S, s = rs - r * S;
  int ph[3], pw[3];
  const int mh = preimages(qh, r, pad, H, reflect, ph);
  const int mw = preimages(qw, s, pad, W, reflect, pw);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int a = 0; a < mh; ++a)
    for (int b = 0; b < mw; ++b) {
      const float4 v = g[(n * H + ph[a]) * (long)W + pw[b]];
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
  d[i] = acc;
}

// tapfold_k writing D straight as the x6 weight gradient's B operand: three bf16 planes
// [3][R*S*4][ldp] (hi, mid, lo; RNE splits as vst_weight_split), channel-major over the P pixels, so
// the fp32 D (N*H*W*R*S*16 bytes) and its plane copy are never materialised.  grid (ceil(P / 256),
// R*S): a thread owns one pixel q and one tap (r, s), i.e. the 4 channels (r, s, 0..3).
__device__ __forceinline__ uint32_t tap_bf16x2(float a, float b) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef __bf16 b2 __attribute__((ext_vector_type(2)));
  const f2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, b2));
}

__global__ __launch_bounds__(256) void tapfold_planes_k(const float4* __restrict__ g, uint16_t* __restrict__ planes,
                                                        int H, int W, int R, int S, int pad, int reflect, long P,
                                                        long ldp) {
  const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= P) return;
  const int rs = blockIdx.y;
  const int qw = q % W;
  const long t = q / W;
  const int qh = t % H;
  const long n = t / H;
  const int r = rs / S, s = rs - r * S;
  int ph[3], pw[3];
  const int mh = preimages(qh, r, pad, H, reflect, ph);
  const int mw = preimages(qw, s, pad, W, reflect, pw);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int a = 0; a < mh; ++a)
    for (int b = 0; b < mw; ++b) {
      const float4 v = g[(n * H + ph[a]) * (long)W + pw[b]];
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
  float v[4] = {acc.x, acc.y, acc.z, acc.w};
  const long plane = (long)R * S * 4 * ldp;
  uint16_t* dst = planes + (long)rs * 4 * ldp + q;
#pragma unroll
  for (int pl = 0; pl < 3; ++pl) {
    const uint32_t q0 = tap_bf16x2(v[0], v[1]), q1 = tap_bf16x2(v[2], v[3]);
    dst[pl * plane] = (uint16_t)q0;
    dst[pl * plane + ldp] = (uint16_t)(q0 >> 16);
    dst[pl * plane + 2 * ldp] = (uint16_t)q1;
    dst[pl * plane + 3 * ldp] = (uint16_t)(q1 >> 16);
    if (pl < 2) {
      v[0] -= __uint_as_float(q0 << 16);
      v[1] -= __uint_as_float(q0 & 0xffff0000u);
      v[2] -= __uint_as_float(q1 << 16);
      v[3] -= __uint_as_float(q1 & 0xffff0000u);
    }
  }
}

// Row-segment form of tapsum: a 64-lane block owns 64 consecutive output pixels of one row; for
// each filter row r it stages the S taps of that row for the 64 + S - 1 source pixels in LDS
// (each pixel's S float4 are contiguous in Z), then every lane sums its S taps from LDS.  Every Z
// element is read once, in 16*S-byte contiguous runs.
template <int S>
__global__ __launch_bounds__(64) void tapsum_row_k(const float4* __restrict__ z, const float* __restrict__ bias,
                                                   float4* __restrict__ y, int H, int W, int R, int pad,
                                                   int reflect, int act, float slope) {
  constexpr int SEG = 64, NSRC = SEG + S - 1;
  __shared__ float4 lds[NSRC * S];
  const int lane = threadIdx.x;
  const int segs = (W + SEG - 1) / SEG;
  const long row = blockIdx.x / segs;  // (n, h)
  const int w0 = (blockIdx.x % segs) * SEG;
  const int h = row % H;
  const long n = row / H;
  const int zcs4 = R * S;
  const int w = w0 + lane;
  float4 acc = bias ? make_float4(bias[0], bias[1], bias[2], bias[3]) : make_float4(0.f, 0.f, 0.f, 0.f);
  for (int r = 0; r < R; ++r) {
    const int hh = src_index(h + r - pad, H, reflect);
    if (hh < 0) continue;  // whole row zero-padded (uniform over the block)
    const float4* zr = z + (n * H + hh) * (long)W * zcs4 + r * S;
    __syncthreads();
    for (int e = lane; e < NSRC * S; e += SEG) {
      const int j = e / S, s = e - j * S;
      const int ww = src_index(w0 - pad + j, W, reflect);
      lds[e] = (ww >= 0 && w0 - pad + j < W + pad) ? zr[(long)ww * zcs4 + s] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const float4 v = lds[(lane + s) * S + s];
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
  }
  if (w < W)
    y[row * W + w] = make_float4(apply_act(acc.x, act, slope), apply_act(acc.y, act, slope),
                                 apply_act(acc.z, act, slope), apply_act(acc.w, act, slope));
}

// Data-gradient gather (adjoint of the tap gather): y[q] = sum_{r,s} sum_{p: src(p,r,s) = q} Z[p][(r,s)]
__global__ void tapgather_k(const float4* __restrict__ z, float4* __restrict__ y, int H, int W, int R, int S,
                            int pad, int reflect, long P) {
  const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= P) return;
  const int qw = q % W;
  const long t = q / W;
  const int qh = t % H;
  const long n = t / H;
  const int zcs4 = R * S;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int r = 0; r < R; ++r) {
    int ph[3];
    const int mh = preimages(qh, r, pad, H, reflect, ph);
    for (int a = 0; a < mh; ++a) {
      const float4* zr = z + (n * H + ph[a]) * (long)W * zcs4 + r * S;
      for (int s = 0; s < S; ++s) {
        int pw[3];
        const int mw = preimages(qw, s, pad, W, reflect, pw);
        for (int b = 0; b < mw; ++b) {
          const float4 v = zr[(long)pw[b] * zcs4 + s];
          acc.x += v.x;
          acc.y += v.y;
          acc.z += v.z;
          acc.w += v.w;
        }
      }
    }
  }
  y[q] = acc;
}

// Stride-2 transposed conv as four sub-pixel phase convolutions (see vst_interleave_phases):
// y[n][2i+a][2j+b][c] = P_ab[n][i+a][j+b][c], P_ab of size (H+a) x (W+b).
__global__ void interleave_phases_k(const float4* __restrict__ p00, const float4* __restrict__ p01,
                                    const float4* __restrict__ p10, const float4* __restrict__ p11,
                                    float4* __restrict__ y, int H, int W, int C4, long total, int full) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int c4 = idx % C4;
  long q = idx / C4;
  const int X = q % (2 * W);
  q /= 2 * W;
  const int Y = q % (2 * H);
  const long n = q / (2 * H);
  const int a = Y & 1, b = X & 1, i = Y >> 1, j = X >> 1;
  const float4* src = a ? (b ? p11 : p10) : (b ? p01 : p00);
  const int Wp = W + (full ? 1 : b), Hp = H + (full ? 1 : a);  // full: every phase is (H+1) x (W+1)
  y[idx] = src[((n * Hp + i + a) * (long)Wp + j + b) * C4 + c4];
}

// Row-segment form of tapgather: a 64-lane block owns output pixels [w0, w0+64) of row qh; for each
// filter row r and each source row ph mapping onto qh, it stages Z[ph][w0-2pad .. w0+64+2pad) taps
// (r, 0..S-1) in LDS and each lane adds its direct column preimages pw = qw - s + pad from LDS; the
// reflected column preimages (lanes within pad of a border) are read from global memory.
template <int S>
__global__ __launch_bounds__(64) void tapgather_row_k(const float4* __restrict__ z, float4* __restrict__ y, int H,
                                                      int W, int R, int pad, int reflect) {
  constexpr int SEG = 64;
  __shared__ float4 lds[(SEG + 2 * (S - 1)) * S];
  const int nsrc = SEG + 4 * pad;
  const int lane = threadIdx.x;
  const int segs = (W + SEG - 1) / SEG;
  const long row = blockIdx.x / segs;
  const int w0 = (blockIdx.x % segs) * SEG;
  const int qh = row % H;
  const long n = row / H;
  const int zcs4 = R * S;
  const int qw = w0 + lane;
  const int base = w0 - 2 * pad;  // source column held at lds slot 0
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int r = 0; r < R; ++r) {
    int ph[3];
    const int mh = preimages(qh, r, pad, H, reflect, ph);  // uniform over the block
    for (int a = 0; a < mh; ++a) {
      const float4* zr = z + (n * H + ph[a]) * (long)W * zcs4 + r * S;
      __syncthreads();
      for (int e = lane; e < nsrc * S; e += SEG) {
        const int j = e / S, s = e - j * S;
        const int pw = base + j;
        lds[e] = (pw >= 0 && pw < W) ? zr[(long)pw * zcs4 + s] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      __syncthreads();
      if (qw < W) {
#pragma unroll
        for (int s = 0; s < S; ++s) {
          int pw[3];
          const int mw = preimages(qw, s, pad, W, reflect, pw);
          for (int b = 0; b < mw; ++b) {
            const int j = pw[b] - base;
            const float4 v = (pw[b] == qw - s + pad && j >= 0 && j < nsrc) ? lds[j * S + s]
                                                                          : zr[(long)pw[b] * zcs4 + s];
            acc.x += v.x;
            acc.y += v.y;
            acc.z += v.z;
            acc.w += v.w;
          }
        }
      }
    }
  }
  if (qw < W) y[row * W + qw] = acc;
}

// dw[co][ci][rs] (+)= t[(rs*4 + co)][ci], co < Co
// y[p][co] = act(bias[co] + sum_s z[(n, h, src(w + s - pad))][s*4 + co]): the column taps of
// vst_tapconv_h_fwd (z rows of Wz pixels x S float4s, y rows of Wo pixels).  One thread per pixel,
// s in order.
template <int S>
__global__ __launch_bounds__(256) void tapsum_h_k(const float4* __restrict__ z, const float* __restrict__ bias,
                                                  float4* __restrict__ y, int Wz, int Wo, int pad, int reflect,
                                                  int act, float slope, long P) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const long row = p / Wo;
  const int w = (int)(p - row * Wo);
  const float4* zr = z + row * Wz * S;
  float4 v[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int ww = src_index(w + s - pad, Wz, reflect);
    v[s] = ww >= 0 ? zr[(long)ww * S + s] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  float4 acc = bias ? make_float4(bias[0], bias[1], bias[2], bias[3]) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int s = 0; s < S; ++s) {
    acc.x += v[s].x;
    acc.y += v[s].y;
    acc.z += v[s].z;
    acc.w += v[s].w;
  }
  y[p] = make_float4(apply_act(acc.x, act, slope), apply_act(acc.y, act, slope), apply_act(acc.z, act, slope),
                     apply_act(acc.w, act, slope));
}

// dy of the R x 1 weight-gradient form of a reflect 'same' conv with 4 (padded) outputs
// (vst_tapshift_planes): over the (H+2) x (W+S+1) output frame of the R x 1 conv with padding
// pad+1, channel (s, co) of pixel (ho, wo) is g[ho-1][wo-1-s][co] (zero outside), written as the x6
// wgrad's three bf16 planes [3][S*4][ldp].  grid (ceil(P / 256), S): thread = (frame pixel, column tap).
__global__ __launch_bounds__(256) void tapshift_planes_k(const float4* __restrict__ g, uint16_t* __restrict__ planes,
                                                         int H, int W, int S, long P, long ldp) {
  const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= P) return;
  const int s = blockIdx.y;
  const int Wf = W + S + 1, Hf = H + 2;
  const int wo = q % Wf;
  const long t = q / Wf;
  const int ho = t % Hf;
  const long n = t / Hf;
  const int h = ho - 1, w = wo - 1 - s;
  const float4 a = ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W) ? g[(n * H + h) * (long)W + w]
                                                                            : make_float4(0.f, 0.f, 0.f, 0.f);
  float v[4] = {a.x, a.y, a.z, a.w};
  const long plane = (long)S * 4 * ldp;
  uint16_t* dst = planes + (long)s * 4 * ldp + q;
#pragma unroll
  for (int pl = 0; pl < 3; ++pl) {
    const uint32_t q0 = tap_bf16x2(v[0], v[1]), q1 = tap_bf16x2(v[2], v[3]);
    dst[pl * plane] = (uint16_t)q0;
    dst[pl * plane + ldp] = (uint16_t)(q0 >> 16);
    dst[pl * plane + 2 * ldp] = (uint16_t)q1;
    dst[pl * plane + 3 * ldp] = (uint16_t)(q1 >> 16);
    if (pl < 2) {
      v[0] -= __uint_as_float(q0 << 16);
      v[1] -= __uint_as_float(q0 & 0xffff0000u);
      v[2] -= __uint_as_float(q1 << 16);
      v[3] -= __uint_as_float(q1 & 0xffff0000u);
    }
  }
}

// dw[co][ci][r][s] (+)= t[((s*4 + co)*Ci + ci)*R + r] (the R x 1 wgrad's [(s, co)][ci][r] result)
__global__ void tap_wgrad_scatter_h_k(const float* __restrict__ t, float* __restrict__ dw, int Ci, int R, int S,
                                      int accumulate, long total) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int s = i % S;
  const long u = i / S;
  const int r = u % R;
  const long u2 = u / R;
  const int ci = u2 % Ci;
  const int co = u2 / Ci;
  const float v = t[(((long)s * 4 + co) * Ci + ci) * R + r];
  dw[i] = accumulate ? dw[i] + v : v;
}

// The swapped weight-gradient form (vst_tap_wgrad_swap): the first cx (3 or 4) channels of dy (NHWC4) as
// the zero-padded channel-major fp32 image [cx][ld] of an Hp x Wp frame (pad rows / columns before, the
// rest after), the "x" side of the GEMM.  grid (ceil(N Hp Wp / 256)), one thread per frame pixel
// (coalesced along each channel row).
// part != null: the block's per-channel sums of g (the bias gradient of the conv, in fp64), folded in
// thread order: wave butterflies (a fixed tree) then the 4 waves in order -> part[block][4].
__global__ __launch_bounds__(256) void tap_swap_dy_cp_k(const float4* __restrict__ g, float* __restrict__ xt, int H,
                                                        int W, int pad, int Hp, int Wp, long P, long ld, int cx,
                                                        double* __restrict__ part) {
  const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (q < P) {
    const int wp = q % Wp;
    const long t = q / Wp;
    const int h = (int)(t % Hp) - pad, w = wp - pad;
    const long n = t / Hp;
    if ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W) a = g[(n * H + h) * (long)W + w];
    xt[q] = a.x;
    xt[ld + q] = a.y;
    xt[2 * ld + q] = a.z;
    if (cx == 4) xt[3 * ld + q] = a.w;
  }
  if (!part) return;
  double v[4] = {a.x, a.y, a.z, a.w};
  __shared__ double red[4][4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    v[c] = wave_sum_d(v[c]);
    if (lane == 0) red[wv][c] = v[c];
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    const int c = threadIdx.x;
    part[(long)blockIdx.x * 4 + c] = ((red[0][c] + red[1][c]) + red[2][c]) + red[3][c];
  }
}

// dw[co][ci][tap] (+)= t[co][ci][RS-1-tap]: the swapped GEMM's taps run rotated by 180 degrees.  db != null:
// the grid's last block folds the tap_swap_dy_cp_k block sums into db[c < Co] (thread c*64 + l sums blocks
// l, l + 64, ... in order; then the 64 lanes' butterfly, a fixed tree).
__global__ void tap_wgrad_scatter_flip_k(const float* __restrict__ t, float* __restrict__ dw, int RS, int accumulate,
                                         long total, const double* __restrict__ part, int nblk,
                                         float* __restrict__ db, int Co) {
  if (db && blockIdx.x == gridDim.x - 1) {
    const int c = threadIdx.x >> 6, l = threadIdx.x & 63;
    double s = 0.0;
    if (c < Co)
      for (int b = l; b < nblk; b += 64) s += part[(long)b * 4 + c];
    s = wave_sum_d(s);
    if (c < Co && l == 0) db[c] = accumulate ? db[c] + (float)s : (float)s;
    return;
  }
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int tap = i % RS;
  const float v = t[i - tap + (RS - 1 - tap)];
  dw[i] = accumulate ? dw[i] + v : v;
}

__global__ void tap_wgrad_scatter_k(const float* __restrict__ t, float* __restrict__ dw, int Co, int Ci, int RS,
                                    int accumulate, long total) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int rs = i % RS;
  const long u = i / RS;
  const int ci = u % Ci;
  const int co = u / Ci;
  const float v = t[((long)rs * 4 + co) * Ci + ci];
  dw[i] = accumulate ? dw[i] + v : v;
}

}  // namespace vst

using namespace vst;

extern "C" int vst_tapconv_h_fwd(const float* x, const float* wp, const void* wsplit, const float* bias, float* z,
                                 float* y, int N, int H, int W, int Cx, int R, int pad, int pad_mode, int act,
                                 float slope, int math, void* stream) {
  VST_REQUIRE(x && wp && z && y && N > 0 && H > 0 && W > 0 && Cx % 8 == 0 && pad >= 0 && pad < R,
              "tapconv_h_fwd: bad args (Cx %% 8 == 0, 0 <= pad < R)");
  VST_REQUIRE(R == 3 || R == 5 || R == 7, "tapconv_h_fwd: R in {3, 5, 7}");
  VST_REQUIRE(pad_mode == VST_PAD_ZERO || (2 * pad == R - 1 && pad < H && pad < W),
              "tapconv_h_fwd: reflect padding needs a 'same' conv with pad < size");
  const int Ho = H + 2 * pad - R + 1, Wo = W + 2 * pad - R + 1;
  // 64 channels, 7 x 7, split-bf16: the R x 1 conv and the column taps as one direct kernel (conv_tap64.hip)
  if (wsplit && tap64_ok(Cx, R, W, math))
    return tap64_launch(x, wsplit, (long)4 * R * R * Cx, bias, y, N, H, W, pad, pad_mode == VST_PAD_REFLECT, act,
                        slope, math, (hipStream_t)stream);
  // the R x 1 conv: rows padded by `pad`, the columns by 0 (their taps are summed below)
  if (int e = vst_conv2d_fwd_hwp(x, wp, wsplit, nullptr, z, N, H, W, Cx, 4 * R, R, 1, 1, pad, 0, pad_mode,
                                 VST_ACT_NONE, 0.f, math, stream))
    return e;
  const long P = (long)N * Ho * Wo;
  const int refl = pad_mode == VST_PAD_REFLECT;
  hipStream_t st = (hipStream_t)stream;
  const float4* z4 = reinterpret_cast<const float4*>(z);
  float4* y4 = reinterpret_cast<float4*>(y);
  const dim3 g((unsigned)ceil_div(P, 256));
  if (R == 3)
    hipLaunchKernelGGL(tapsum_h_k<3>, g, dim3(256), 0, st, z4, bias, y4, W, Wo, pad, refl, act, slope, P);
  else if (R == 5)
    hipLaunchKernelGGL(tapsum_h_k<5>, g, dim3(256), 0, st, z4, bias, y4, W, Wo, pad, refl, act, slope, P);
  else
    hipLaunchKernelGGL(tapsum_h_k<7>, g, dim3(256), 0, st, z4, bias, y4, W, Wo, pad, refl, act, slope, P);
  return check_launch("tapconv_h_fwd");
}

extern "C" int vst_tapsum_fwd(const float* z, int zcs, const float* bias, float* y, int N, int H, int W, int R,
                              int S, int pad, int pad_mode, int act, float slope, void* stream) {
  VST_REQUIRE(z && y && N > 0 && H > 0 && W > 0 && R > 0 && S > 0 && zcs == R * S * 4 && pad >= 0,
              "tapsum_fwd: bad args");
  VST_REQUIRE(pad_mode == VST_PAD_ZERO || (pad < H && pad < W), "tapsum_fwd: reflect pad >= size");
  VST_REQUIRE(2 * pad == R - 1 && 2 * pad == S - 1, "tapsum_fwd: 'same' convolutions only (2*pad == k-1)");
  const long P = (long)N * H * W;
  const int refl = pad_mode == VST_PAD_REFLECT;
  hipStream_t st = (hipStream_t)stream;
  const dim3 rows((unsigned)((long)N * H * ceil_div(W, 64)));
  switch (S) {
    case 3: hipLaunchKernelGGL(tapsum_row_k<3>, rows, dim3(64), 0, st, reinterpret_cast<const float4*>(z), bias,
                               reinterpret_cast<float4*>(y), H, W, R, pad, refl, act, slope); break;
    case 5: hipLaunchKernelGGL(tapsum_row_k<5>, rows, dim3(64), 0, st, reinterpret_cast<const float4*>(z), bias,
                               reinterpret_cast<float4*>(y), H, W, R, pad, refl, act, slope); break;
    case 7: hipLaunchKernelGGL(tapsum_row_k<7>, rows, dim3(64), 0, st, reinterpret_cast<const float4*>(z), bias,
                               reinterpret_cast<float4*>(y), H, W, R, pad, refl, act, slope); break;
    default:
      hipLaunchKernelGGL(tapsum_k, dim3(ceil_div(P, 256)), dim3(256), 0, st, reinterpret_cast<const float4*>(z),
                         zcs / 4, bias, reinterpret_cast<float4*>(y), H, W, R, S, pad, refl, act, slope, P);
  }
  return check_launch("tapsum_fwd");
}

extern "C" int vst_tapfold(const float* g, float* d, int N, int H, int W, int R, int S, int pad, int pad_mode,
                           void* stream) {
  VST_REQUIRE(g && d && N > 0 && H > 0 && W > 0 && R > 0 && S > 0 && pad >= 0, "tapfold: bad args");
  VST_REQUIRE(pad_mode == VST_PAD_ZERO || (pad < H && pad < W), "tapfold: reflect pad >= size");
  VST_REQUIRE(2 * pad == R - 1 && 2 * pad == S - 1, "tapfold: 'same' convolutions only (2*pad == k-1)");
  const long total = (long)N * H * W * R * S;
  hipLaunchKernelGGL(tapfold_k, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const float4*>(g), reinterpret_cast<float4*>(d), H, W, R, S, pad,
                     pad_mode == VST_PAD_REFLECT, total);
  return check_launch("tapfold");
}

extern "C" int vst_tapfold_planes(const float* g, void* planes, long ldp, int N, int H, int W, int R, int S, int pad,
                                  int pad_mode, void* stream) {
  const long P = (long)N * H * W;
  VST_REQUIRE(g && planes && N > 0 && H > 0 && W > 0 && R > 0 && S > 0 && pad >= 0 && ldp >= P,
              "tapfold_planes: bad args");
  hipLaunchKernelGGL(tapfold_planes_k, dim3(ceil_div(P, 256), R * S), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const float4*>(g), reinterpret_cast<uint16_t*>(planes), H, W, R, S, pad,
                     pad_mode == VST_PAD_REFLECT, P, ldp);
  return check_launch("tapfold_planes");
}

extern "C" int vst_tapshift_planes(const float* g, void* planes, long ldp, int N, int H, int W, int S, void* stream) {
  const long P = (long)N * (H + 2) * (W + S + 1);
  VST_REQUIRE(g && planes && N > 0 && H > 0 && W > 0 && S > 0 && S <= 8 && ldp >= P, "tapshift_planes: bad args");
  hipLaunchKernelGGL(tapshift_planes_k, dim3(ceil_div(P, 256), S), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const float4*>(g), reinterpret_cast<uint16_t*>(planes), H, W, S, P, ldp);
  return check_launch("tapshift_planes");
}

extern "C" int vst_tap_wgrad_scatter_h(const float* t, float* dw, int Co, int Ci, int R, int S, int accumulate,
                                       void* stream) {
  VST_REQUIRE(t && dw && Co > 0 && Co <= 4 && Ci > 0 && R > 0 && S > 0, "tap_wgrad_scatter_h: bad args");
  const long total = (long)Co * Ci * R * S;
  hipLaunchKernelGGL(tap_wgrad_scatter_h_k, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, t, dw, Ci,
                     R, S, accumulate, total);
  return check_launch("tap_wgrad_scatter_h");
}

// The swapped form's geometry: frame Hf x (Wf + wx) with wx zero columns so rows are whole 8-pixel chunks.
static void tap_swap_geom(int N, int H, int W, int R, int* Hf, int* Wq, int* wx) {
  *Hf = H + R - 1;
  *wx = (8 - (W + R - 1) % 8) % 8;
  *Wq = W + R - 1 + *wx;
}

extern "C" long vst_tap_wgrad_swap_ld(int N, int H, int W, int R) {
  int Hf, Wq, wx;
  tap_swap_geom(N, H, W, R, &Hf, &Wq, &wx);
  return rk_cp_ld((long)N * Hf * Wq);
}

extern "C" size_t vst_tap_wgrad_swap_ws_bytes(int N, int H, int W, int Ci, int R) {
  int Hf, Wq, wx;
  tap_swap_geom(N, H, W, R, &Hf, &Wq, &wx);
  const int pad = R - 1;
  const long ldx = rk_cp_ld((long)N * (H + 2 * pad) * (W + wx + 2 * pad));
  // the GEMM runs over 3 or 4 dy channels (Co <= 3 or not, see vst_tap_wgrad_swap): size for either plan
  const size_t wg = std::max(vst_conv2d_wgrad_ws_bytes(N, H, W + wx, 4, Hf, Wq, Ci, R, R, 1),
                             vst_conv2d_wgrad_ws_bytes(N, H, W + wx, 3, Hf, Wq, Ci, R, R, 1));
  // + the bias gradient's block sums (vst_tap_wgrad_swap_db: ceil(Pp / 256) x 4 doubles, 8-byte aligned)
  const long Pp = (long)N * (H + 2 * pad) * (W + wx + 2 * pad);
  return (size_t)(4 * ldx + 4 * (long)Ci * R * R + 2) * sizeof(float) + (size_t)ceil_div(Pp, 256) * 4 * sizeof(double) +
         wg;
}

extern "C" int vst_tap_wgrad_swap_db(const float* g, const void* x_planes, float* dw, float* db, float* ws,
                                     size_t ws_bytes, int N, int H, int W, int Ci, int R, int Co, int accumulate,
                                     int math, void* stream);

extern "C" int vst_tap_wgrad_swap(const float* g, const void* x_planes, float* dw, float* ws, size_t ws_bytes, int N,
                                  int H, int W, int Ci, int R, int Co, int accumulate, int math, void* stream) {
  return vst_tap_wgrad_swap_db(g, x_planes, dw, nullptr, ws, ws_bytes, N, H, W, Ci, R, Co, accumulate, math, stream);
}

extern "C" int vst_tap_wgrad_swap_db(const float* g, const void* x_planes, float* dw, float* db, float* ws,
                                     size_t ws_bytes, int N, int H, int W, int Ci, int R, int Co, int accumulate,
                                     int math, void* stream) {
  VST_REQUIRE(g && x_planes && dw && ws && N > 0 && H > 0 && W > 0 && Co > 0 && Co <= 4 && R % 2 == 1 &&
                  Ci % 4 == 0 && (R - 1) / 2 < H && (R - 1) / 2 < W,
              "tap_wgrad_swap: bad args");
  VST_REQUIRE(ws_bytes >= vst_tap_wgrad_swap_ws_bytes(N, H, W, Ci, R), "tap_wgrad_swap: workspace too small");
  int Hf, Wq, wx;
  tap_swap_geom(N, H, W, R, &Hf, &Wq, &wx);
  const int pad = R - 1, Hp = H + 2 * pad, Wp = W + wx + 2 * pad;
  const long Pp = (long)N * Hp * Wp, ldx = rk_cp_ld(Pp);
  hipStream_t s = (hipStream_t)stream;
  float* xt = ws;
  float* t = xt + 4 * ldx;
  const int nblk = ceil_div(Pp, 256);
  double* bpart = reinterpret_cast<double*>(((uintptr_t)(t + 4 * (long)Ci * R * R) + 7) & ~(uintptr_t)7);
  float* wsg = reinterpret_cast<float*>(bpart + (long)nblk * 4);
  // Co <= 3: only three dy channels become GEMM rows (M = 3 R^2: 147 rows = 3 tiles of 64 at R = 7, not 4)
  const int cx = Co <= 3 ? 3 : 4;
  hipLaunchKernelGGL(tap_swap_dy_cp_k, dim3(nblk), dim3(256), 0, s, reinterpret_cast<const float4*>(g), xt, H, W, pad,
                     Hp, Wp, Pp, ldx, cx, db ? bpart : nullptr);
  int rc = check_launch("tap_wgrad_swap");
  if (rc) return rc;
  // t[c][ci][tap'] = sum_q dyP[q + tap'][c] * xf[q][ci]  (the frame's "output" channels ci: so = R*R, si = Ci*R*R)
  const size_t wsb = ws_bytes - (size_t)((char*)wsg - (char*)ws);
  rc = vst_conv2d_wgrad_pre(g, xt, g, x_planes, t, wsg, wsb, N, H, W + wx, cx, Hf, Wq, Ci, R, R, 1, pad, VST_PAD_ZERO,
                            Ci, cx, (long)R * R, (long)Ci * R * R, 0, math, stream);
  if (rc) return rc;
  const long total = (long)Co * Ci * R * R;
  hipLaunchKernelGGL(tap_wgrad_scatter_flip_k, dim3(ceil_div(total, 256) + (db ? 1 : 0)), dim3(256), 0, s, t, dw,
                     R * R, accumulate, total, bpart, nblk, db, Co);
  return check_launch("tap_wgrad_swap");
}

extern "C" int vst_tap_wgrad_scatter(const float* t, float* dw, int Co, int Ci, int R, int S, int accumulate,
                                     void* stream) {
  VST_REQUIRE(t && dw && Co > 0 && Co <= 4 && Ci > 0 && R > 0 && S > 0, "tap_wgrad_scatter: bad args");
  const long total = (long)Co * Ci * R * S;
  hipLaunchKernelGGL(tap_wgrad_scatter_k, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, t, dw, Co,
                     Ci, R * S, accumulate, total);
  return check_launch("tap_wgrad_scatter");
}

extern "C" int vst_tapgather(const float* z, float* y, int N, int H, int W, int R, int S, int pad, int pad_mode,
                             void* stream) {
  VST_REQUIRE(z && y && N > 0 && H > 0 && W > 0 && R > 0 && S > 0 && pad >= 0, "tapgather: bad args");
  VST_REQUIRE(pad_mode == VST_PAD_ZERO || (pad < H && pad < W), "tapgather: reflect pad >= size");
  VST_REQUIRE(2 * pad == R - 1 && 2 * pad == S - 1, "tapgather: 'same' convolutions only (2*pad == k-1)");
  const long P = (long)N * H * W;
  const int refl = pad_mode == VST_PAD_REFLECT;
  hipStream_t st = (hipStream_t)stream;
  const dim3 rows((unsigned)((long)N * H * ceil_div(W, 64)));
  const float4* zz = reinterpret_cast<const float4*>(z);
  float4* yy = reinterpret_cast<float4*>(y);
  switch (S) {
    case 3: hipLaunchKernelGGL(tapgather_row_k<3>, rows, dim3(64), 0, st, zz, yy, H, W, R, pad, refl); break;
    case 5: hipLaunchKernelGGL(tapgather_row_k<5>, rows, dim3(64), 0, st, zz, yy, H, W, R, pad, refl); break;
    case 7: hipLaunchKernelGGL(tapgather_row_k<7>, rows, dim3(64), 0, st, zz, yy, H, W, R, pad, refl); break;
    default:
      hipLaunchKernelGGL(tapgather_k, dim3(ceil_div(P, 256)), dim3(256), 0, st, zz, yy, H, W, R, S, pad, refl, P);
  }
  return check_launch("tapgather");
}

extern "C" int vst_interleave_phases(const float* p00, const float* p01, const float* p10, const float* p11, float* y,
                                     int N, int H, int W, int C, void* stream) {
  VST_REQUIRE(p00 && p01 && p10 && p11 && y && N > 0 && H > 0 && W > 0 && C % 4 == 0, "interleave_phases: bad args");
  const long total = (long)N * 4 * H * W * (C / 4);
  hipLaunchKernelGGL(interleave_phases_k, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const float4*>(p00), reinterpret_cast<const float4*>(p01),
                     reinterpret_cast<const float4*>(p10), reinterpret_cast<const float4*>(p11),
                     reinterpret_cast<float4*>(y), H, W, C / 4, total, 0);
  return check_launch("interleave_phases");
}

extern "C" int vst_interleave_phases_full(const float* p00, const float* p01, const float* p10, const float* p11,
                                          float* y, int N, int H, int W, int C, void* stream) {
  VST_REQUIRE(p00 && p01 && p10 && p11 && y && N > 0 && H > 0 && W > 0 && C % 4 == 0,
              "interleave_phases_full: bad args");
  const long total = (long)N * 4 * H * W * (C / 4);
  hipLaunchKernelGGL(interleave_phases_k, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const float4*>(p00), reinterpret_cast<const float4*>(p01),
                     reinterpret_cast<const float4*>(p10), reinterpret_cast<const float4*>(p11),
                     reinterpret_cast<float4*>(y), H, W, C / 4, total, 1);
  return check_launch("interleave_phases_full");
}
