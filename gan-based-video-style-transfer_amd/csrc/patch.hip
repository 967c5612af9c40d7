// The PatchGAN head — Conv2d(8*ndf, 1, kernel 4, stride 1, padding 1), the last layer of the reference
// NLayerDiscriminator (methods/GAN-based/CycleGAN/models/networks.py:576-578) — forward, weight gradient
// and data gradient, each reading its wide operand (the 512-channel 31x31 activation, or writing its
// gradient) ONCE from HBM.
//
// The head has one real output channel (padded to 4 in NHWC), so its convolution is not a GEMM that
// fills an MFMA tile: per output pixel it is a 16-tap x Cin dot product, and the whole layer moves
// ~16 MB for 0.12 GFLOP.  The generic VALU path (skinny.hip) re-gathered the input once per output
// pixel (16x the bytes through L2: 50 us at N = 8) and its weight gradient ran 128 split-K slabs of
// 4 x Mw floats.  Here every kernel walks the activation row by row:
//
//   head_fwd_k      block = (image, output row, column segment); wave r takes input row h - pad + r and
//                   computes its S tap dot products z[r][col][s] for the segment's columns (KS lanes per
//                   column split the channels; the row's weights are staged in LDS); the block then
//                   sums z over (r, s) in a fixed order.  An input row is read by R blocks (L2 / MALL),
//                   never re-gathered per tap.
//   head_wgrad_k    block = (image, group of input rows): each thread owns 4 channels and accumulates
//                   all R*S taps' products x[i][j][c] * dy[i+pad-r][j+pad-s] (dy wave-uniform), so the
//                   activation is read once; the per-block partials [R*S][Cin] are summed by
//                   head_wgrad_reduce_k in a fixed slab order (deterministic) into the reference
//                   [Co][Ci][R][S] layout.
//   head_dgrad_k    block = (image, input row): dx[i][j][c] = sum_{r,s} dy[i+pad-r][j+pad-s] * w[r][s][c]
//                   with the thread's 4-channel weight column for all taps in registers; a write-bound
//                   pass.
// fp32 arithmetic throughout (fma chains; only the summation order differs from the reference's).
#include "common.h"

namespace vst {
namespace patch {

constexpr int RMAX = 4, SMAX = 4;  // kernel taps per dimension (the head is 4 x 4)

// ---- forward -------------------------------------------------------------------------------------
// wp: the VST_PACK_OK pack [Cop][R][S][Cin]; only output channel 0 is computed (co_real = 1), the
// padded channels get act(bias[c]) like the 4-channel path's zero sums.
template <int KS>
__global__ __launch_bounds__(256) void head_fwd_k(const float* __restrict__ x, const float* __restrict__ wp,
                                                  const float* __restrict__ bias, float* __restrict__ out, int Hi,
                                                  int Wi, int Cin, int Ho, int Wo, int R, int S, int pad, int act,
                                                  float slope, int seg) {
  constexpr int NCOL = 64 / KS;
  extern __shared__ float lds[];
  float* wl = lds;                        // [R][S][Cin]
  float* z = lds + RMAX * SMAX * Cin;     // [RMAX][NCOL][SMAX]
  const int t = threadIdx.x, lane = t & 63;
  const int r = __builtin_amdgcn_readfirstlane(t >> 6);
  const int n = blockIdx.z, h = blockIdx.y, w0 = blockIdx.x * seg;
  const long wn = (long)R * S * Cin;
  for (long e = 4 * t; e < wn; e += 4 * 256)
    *reinterpret_cast<float4*>(wl + e) = *reinterpret_cast<const float4*>(wp + e);
  __syncthreads();
  const int col = lane / KS, k = lane % KS;
  const int hi = h - pad + r, wi = w0 - pad + col;
  const int ncol = seg + S - 1;
  float acc[SMAX] = {0.f, 0.f, 0.f, 0.f};
  if (r < R && (unsigned)hi < (unsigned)Hi && col < ncol && (unsigned)wi < (unsigned)Wi) {
    // lane k of a column takes the channel range [k * Cin / KS, (k + 1) * Cin / KS): a contiguous stream
    const int cw = Cin / KS, c0 = k * cw;
    const float* src = x + (((long)n * Hi + hi) * Wi + wi) * Cin + c0;
    const float* wr = wl + (long)r * S * Cin + c0;
    if (S == 4) {
#pragma unroll 4
      for (int c = 0; c < cw; c += 4) {
        const float4 v = *reinterpret_cast<const float4*>(src + c);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const float4 w = *reinterpret_cast<const float4*>(wr + s * Cin + c);
          acc[s] = fmaf(v.x, w.x, acc[s]);
          acc[s] = fmaf(v.y, w.y, acc[s]);
          acc[s] = fmaf(v.z, w.z, acc[s]);
          acc[s] = fmaf(v.w, w.w, acc[s]);
        }
      }
    } else {
      for (int c = 0; c < cw; c += 4) {
        const float4 v = *reinterpret_cast<const float4*>(src + c);
#pragma unroll
        for (int s = 0; s < SMAX; ++s) {
          if (s >= S) break;
          const float4 w = *reinterpret_cast<const float4*>(wr + s * Cin + c);
          acc[s] = fmaf(v.x, w.x, acc[s]);
          acc[s] = fmaf(v.y, w.y, acc[s]);
          acc[s] = fmaf(v.z, w.z, acc[s]);
          acc[s] = fmaf(v.w, w.w, acc[s]);
        }
      }
    }
  }
#pragma unroll
  for (int s = 0; s < SMAX; ++s)
#pragma unroll
    for (int o = KS / 2; o > 0; o >>= 1) acc[s] += __shfl_xor(acc[s], o, 64);
  if (k == 0 && r < RMAX) {
#pragma unroll
    for (int s = 0; s < SMAX; ++s) z[(r * NCOL + col) * SMAX + s] = acc[s];
  }
  __syncthreads();
  if (t < seg && w0 + t < Wo) {
    float v = 0.f;
    for (int rr = 0; rr < R; ++rr)
      for (int s = 0; s < S; ++s) v += z[(rr * NCOL + t + s) * SMAX + s];
    const float4 b4 = bias ? *reinterpret_cast<const float4*>(bias) : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 o;
    o.x = apply_act(v + b4.x, act, slope);
    o.y = apply_act(b4.y, act, slope);
    o.z = apply_act(b4.z, act, slope);
    o.w = apply_act(b4.w, act, slope);
    *reinterpret_cast<float4*>(out + (((long)n * Ho + h) * Wo + w0 + t) * 4) = o;
  }
}

// ---- weight gradient -----------------------------------------------------------------------------
// part[zb][(r*S + s)*Cin + c] = sum over the block's input rows i and columns j of
// x[n][i][j][c] * dy[n][i+pad-r][j+pad-s][0]   (zero outside dy).  Thread: channel quad q = t % Q
// (Q = Cin / 4), column group g = t / Q (NG = 256 / Q groups stride the row's columns).
__global__ __launch_bounds__(256) void head_wgrad_k(const float* __restrict__ x, const float* __restrict__ dy,
                                                    float* __restrict__ part, int Hi, int Wi, int Cin, int Ho,
                                                    int Wo, int R, int S, int pad, int G) {
  extern __shared__ float lds[];
  // dl[r][SMAX + ww]: dy row i + pad - r (channel 0), zero outside the image, so the tap loop has no
  // bounds tests; then the cross-group partials [NG - 1][R*S][Cin]
  const int DW = Wo + 2 * SMAX;
  float* dl = lds;
  float* xg = lds + RMAX * DW;
  const int t = threadIdx.x, Q = Cin / 4, NG = 256 / Q;
  const int q = t % Q, g = t / Q;
  const int n = blockIdx.y, i0 = blockIdx.x * G;
  float4 acc[RMAX * SMAX];
#pragma unroll
  for (int e = 0; e < RMAX * SMAX; ++e) acc[e] = make_float4(0.f, 0.f, 0.f, 0.f);
  const float* dyn = dy + (long)n * Ho * Wo * 4;
  for (int i = i0; i < i0 + G && i < Hi; ++i) {
    __syncthreads();
    for (int e = t; e < RMAX * DW; e += 256) {
      const int r = e / DW, ww = e - r * DW - SMAX, hh = i + pad - r;
      dl[e] = (r < R && (unsigned)hh < (unsigned)Ho && (unsigned)ww < (unsigned)Wo) ? dyn[((long)hh * Wo + ww) * 4]
                                                                                     : 0.f;
    }
    __syncthreads();
    const float* xr = x + ((long)n * Hi + i) * Wi * Cin + 4 * q;
    for (int j = g; j < Wi; j += NG) {
      const float4 v = *reinterpret_cast<const float4*>(xr + (long)j * Cin);
      const float* dj = dl + SMAX + j + pad;
#pragma unroll
      for (int r = 0; r < RMAX; ++r)
#pragma unroll
        for (int s = 0; s < SMAX; ++s) {
          const float d = dj[r * DW - s];
          float4& a = acc[r * SMAX + s];
          a.x = fmaf(v.x, d, a.x);
          a.y = fmaf(v.y, d, a.y);
          a.z = fmaf(v.z, d, a.z);
          a.w = fmaf(v.w, d, a.w);
        }
    }
  }
  const int RS = R * S;
  if (g > 0) {
#pragma unroll
    for (int r = 0; r < RMAX; ++r)
#pragma unroll
      for (int s = 0; s < SMAX; ++s)
        if (r < R && s < S)
          *reinterpret_cast<float4*>(xg + ((long)(g - 1) * RS + r * S + s) * Cin + 4 * q) = acc[r * SMAX + s];
  }
  __syncthreads();
  if (g == 0) {
    float* dst = part + (long)(blockIdx.y * gridDim.x + blockIdx.x) * RS * Cin + 4 * q;
#pragma unroll
    for (int r = 0; r < RMAX; ++r)
#pragma unroll
      for (int s = 0; s < SMAX; ++s) {
        if (r >= R || s >= S) continue;
        float4 a = acc[r * SMAX + s];
        for (int gg = 1; gg < NG; ++gg)
          add_f4(a, *reinterpret_cast<const float4*>(xg + ((long)(gg - 1) * RS + r * S + s) * Cin + 4 * q));
        *reinterpret_cast<float4*>(dst + (long)(r * S + s) * Cin) = a;
      }
  }
}

// Fixed-order sum of the 256 threads' values v (the block's, in thread order of 16-groups) -> thread 0.
__device__ __forceinline__ float block_sum_fixed(float v, float* red) {
  red[threadIdx.x] = v;
  __syncthreads();
  float s = 0.f;
  if (threadIdx.x < 16) {
    for (int k = 0; k < 16; ++k) s += red[threadIdx.x * 16 + k];
  }
  __syncthreads();
  if (threadIdx.x < 16) red[threadIdx.x] = s;
  __syncthreads();
  s = 0.f;
  if (threadIdx.x == 0)
    for (int k = 0; k < 16; ++k) s += red[k];
  return s;
}

// db[0] (+)= sum_p dy[p][0] over P pixels of a 4-channel dy, in a fixed order (one block).
__device__ void bias_sum_c0(const float* __restrict__ dy, long P, float* __restrict__ db, int accumulate) {
  __shared__ float red[256];
  float a = 0.f;
  for (long p = threadIdx.x; p < P; p += 256) a += dy[p * 4];
  const float s = block_sum_fixed(a, red);
  if (threadIdx.x == 0) db[0] = accumulate ? db[0] + s : s;
}

// dw[ci*si + rs] (+)= sum_z part[z][rs*Cin + ci] in a fixed order: block = 16 outputs x 16 slab
// groups (group u sums slabs u, u + 16, ... in order), the 16 group sums are then added in order.
// db != null: one more block sums dy's channel 0 (the bias gradient).
__global__ __launch_bounds__(256) void head_wgrad_reduce_k(const float* __restrict__ part, float* __restrict__ dw,
                                                           int Mw, int Cin, int Ci, int RS, long si,
                                                           int accumulate, int nz, const float* __restrict__ dy,
                                                           long P, float* __restrict__ db) {
  if (db && blockIdx.x == gridDim.x - 1) {
    bias_sum_c0(dy, P, db, accumulate);
    return;
  }
  __shared__ float red[16][17];
  const int t = threadIdx.x, o = t & 15, u = t >> 4;
  const int m = blockIdx.x * 16 + o;
  float a = 0.f;
  if (m < Mw) {
    int zz = u;
    for (; zz + 48 < nz; zz += 64) {
      const float p0 = part[(long)zz * Mw + m], p1 = part[(long)(zz + 16) * Mw + m];
      const float p2 = part[(long)(zz + 32) * Mw + m], p3 = part[(long)(zz + 48) * Mw + m];
      a += p0;
      a += p1;
      a += p2;
      a += p3;
    }
    for (; zz < nz; zz += 16) a += part[(long)zz * Mw + m];
  }
  red[u][o] = a;
  __syncthreads();
  const int rs = m / Cin, ci = m - rs * Cin;
  if (u == 0 && m < Mw && ci < Ci) {
    float s = red[0][o];
    for (int k = 1; k < 16; ++k) s += red[k][o];
    float* d = dw + (long)ci * si + rs;
    *d = accumulate ? *d + s : s;
  }
}

// ---- data gradient -------------------------------------------------------------------------------
// dx[n][i][j][c] = sum_{r,s} dy[n][i+pad-r][j+pad-s][0] * w[c][r][s][0] (+ addend): wp = the VST_PACK_IK
// pack [Cx][R][S][Cy] with Cy = 4 of which only channel 0 is real (co_real = 1).
__global__ __launch_bounds__(256) void head_dgrad_k(const float* __restrict__ dy, const float* __restrict__ wp,
                                                    const float* __restrict__ addend, float* __restrict__ dx,
                                                    int Hd, int Wd, int Cx, int H, int W, int R, int S, int pad) {
  extern __shared__ float dl[];  // dl[r][SMAX + ww] = dy row i + pad - r (channel 0), zero outside
  const int DW = Wd + 2 * SMAX;
  const int t = threadIdx.x, Q = Cx / 4, NG = 256 / Q;
  const int q = t % Q, g = t / Q;
  const int n = blockIdx.y, i = blockIdx.x;
  const float* dyn = dy + (long)n * Hd * Wd * 4;
  for (int e = t; e < RMAX * DW; e += 256) {
    const int r = e / DW, ww = e - r * DW - SMAX, hh = i + pad - r;
    dl[e] = (r < R && (unsigned)hh < (unsigned)Hd && (unsigned)ww < (unsigned)Wd) ? dyn[((long)hh * Wd + ww) * 4]
                                                                                  : 0.f;
  }
  float4 wv[RMAX * SMAX];
  const long cs = (long)R * S * 4;  // between input channels of the IK pack
#pragma unroll
  for (int r = 0; r < RMAX; ++r)
#pragma unroll
    for (int s = 0; s < SMAX; ++s) {
      float4 w = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r < R && s < S) {
        const float* p = wp + (long)(4 * q) * cs + (r * S + s) * 4;  // [c][r][s][0], c = 4q..4q+3
        w = make_float4(p[0], p[cs], p[2 * cs], p[3 * cs]);
      }
      wv[r * SMAX + s] = w;
    }
  __syncthreads();
  for (int j = g; j < W; j += NG) {
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    const float* dj = dl + SMAX + j + pad;
#pragma unroll
    for (int r = 0; r < RMAX; ++r)
#pragma unroll
      for (int s = 0; s < SMAX; ++s) {
        const float d = dj[r * DW - s];
        const float4 w = wv[r * SMAX + s];
        a.x = fmaf(d, w.x, a.x);
        a.y = fmaf(d, w.y, a.y);
        a.z = fmaf(d, w.z, a.z);
        a.w = fmaf(d, w.w, a.w);
      }
    const long o = (((long)n * H + i) * W + j) * Cx + 4 * q;
    if (addend) add_f4(a, *reinterpret_cast<const float4*>(addend + o));
    *reinterpret_cast<float4*>(dx + o) = a;
  }
}


// ---- image-input weight gradient (the PatchGAN first layer Conv2d(3, ndf, 4, 2, 1), networks.py:556) ----
// C[co][j] = sum_p dy[p][co] * X[p][j] over the output pixels p, j = (r*S + s)*4 + c, X[p][j] =
// x[n][st*ho - pad + r][st*wo - pad + s][c] (zero outside; c < Ci real, the rest zero) and, when the
// bias gradient is wanted, X[p][3] = 1 (tap 0's padding channel): row j = 3 of C is then sum_p dy[p][co].
// On v_mfma_f32_32x32x2_f32 — the exact fp32 products (no bf16 split: this GEMM is 64 x 64 x P,
// HBM-bound on the fp32 dy stream, which is read once and never converted to planes).  Lane l = (i =
// l % 32, k = l / 32) feeds pixel p0 + k of a pair: A block mi takes co = 2i + mi (one float2 load of dy's
// row), B block nj takes j = 2i + nj (one float2 of x: tap i / 2, channels 2 (i % 2) + {0, 1}).  A wave
// walks a contiguous run of pixel pairs; the block's waves add their 64 x 64 tiles in LDS in a fixed
// order into one partial slab part[block][j][co], reduced by img_wgrad_reduce_k.
constexpr int IW_WAVES = 8;

__global__ __launch_bounds__(64 * IW_WAVES) void img_wgrad_k(const float* __restrict__ x, const float* __restrict__ dy,
                                                            float* __restrict__ part, int H, int W, int Ho, int Wo,
                                                            int Cyp, int R, int S, int st, int pad, int Ci,
                                                            int want_db, long P, int ppw) {
  extern __shared__ float tl[];  // [IW_WAVES - 1][64][64] wave tiles (j-major: [j][co])
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int i = lane & 31, kk = lane >> 5;
  const int rs = i >> 1, c0 = 2 * (i & 1);
  const int r = rs / S, s = rs - (rs / S) * S;
  const bool tap_ok = rs < R * S;
  const bool co_ok = 2 * i < Cyp;
  // which of this lane's two B channels are real / the bias slot
  const bool cx_ok = c0 < Ci, cy_ok = c0 + 1 < Ci;
  const float cy_bias = (want_db && rs == 0 && c0 + 1 == 3) ? 1.f : 0.f;
  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;
  const long wid = (long)blockIdx.x * IW_WAVES + wave;
  const long p0 = wid * ppw, p1 = p0 + ppw < P ? p0 + ppw : P;
  const long HWo = (long)Ho * Wo;
  for (long p = p0 + kk; p - kk < p1; p += 2) {
    float2 av = make_float2(0.f, 0.f), bv = make_float2(0.f, cy_bias);
    if (p < p1) {
      const long n = p / HWo;
      const int rem = (int)(p - n * HWo), ho = rem / Wo, wo = rem - (rem / Wo) * Wo;
      if (co_ok) av = *reinterpret_cast<const float2*>(dy + p * Cyp + 2 * i);
      const int hi = st * ho - pad + r, wi = st * wo - pad + s;
      if (tap_ok && (unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W) {
        const float2 v = *reinterpret_cast<const float2*>(x + (((n * H + hi) * W + wi) << 2) + c0);
        bv.x = cx_ok ? v.x : 0.f;
        if (cy_ok) bv.y = v.y;
      }
    } else {
      bv.y = 0.f;
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(a ? av.y : av.x, b ? bv.y : bv.x, acc[a][b], 0, 0, 0);
  }
  // C block (a, b): lane column jj = i, rows ii = 8 (e / 4) + 4 kk + e % 4  ->  co = 2 ii + a, j = 2 jj + b
  if (wave > 0) {
    float* d = tl + (long)(wave - 1) * 4096;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int ii = 8 * (e >> 2) + 4 * kk + (e & 3);
          d[(2 * i + b) * 64 + 2 * ii + a] = acc[a][b][e];
        }
  }
  __syncthreads();
  if (wave == 0) {
    float* dst = part + (long)blockIdx.x * 4096;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int ii = 8 * (e >> 2) + 4 * kk + (e & 3);
          const int o = (2 * i + b) * 64 + 2 * ii + a;
          float v = acc[a][b][e];
          for (int w = 0; w < IW_WAVES - 1; ++w) v += tl[(long)w * 4096 + o];
          dst[o] = v;
        }
  }
}

// dw[co*so + ci*si + rs] (+)= sum_z part[z][rs*4 + ci][co] (ci < Ci, co < Co), db[co] (+)= sum_z
// part[z][3][co]; fixed order: block = 16 outputs x 16 slab groups.
__global__ __launch_bounds__(256) void img_wgrad_reduce_k(const float* __restrict__ part, float* __restrict__ dw,
                                                          float* __restrict__ db, int RS, int Co, int Ci, long so,
                                                          long si, int accumulate, int nz) {
  __shared__ float red[16][17];
  const int t = threadIdx.x, o = t & 15, u = t >> 4;
  const int m = blockIdx.x * 16 + o;  // (j, co) = (m / 64, m % 64)
  float a = 0.f;
  {
    int zz = u;
    for (; zz + 48 < nz; zz += 64) {
      const float p0 = part[(long)zz * 4096 + m], p1 = part[(long)(zz + 16) * 4096 + m];
      const float p2 = part[(long)(zz + 32) * 4096 + m], p3 = part[(long)(zz + 48) * 4096 + m];
      a += p0;
      a += p1;
      a += p2;
      a += p3;
    }
    for (; zz < nz; zz += 16) a += part[(long)zz * 4096 + m];
  }
  red[u][o] = a;
  __syncthreads();
  const int j = m >> 6, co = m & 63, rs = j >> 2, ci = j & 3;
  if (u != 0 || co >= Co) return;
  float v = red[0][o];
  for (int k = 1; k < 16; ++k) v += red[k][o];
  if (ci < Ci && rs < RS) {
    float* d = dw + (long)co * so + (long)ci * si + rs;
    *d = accumulate ? *d + v : v;
  } else if (db && j == 3) {
    db[co] = accumulate ? db[co] + v : v;
  }
}

}  // namespace patch

using namespace patch;

bool head_ok(int Cin, int R, int S, int st, int reflect, int Wo) {
  // Cin / 4 must divide the 256 threads (the channel quads x column groups layout); the LDS images
  // (the forward's weights, the weight gradient's cross-group partials + dy rows) must fit
  if (!(st == 1 && !reflect && R >= 1 && R <= RMAX && S >= 1 && S <= SMAX && Cin % 4 == 0 && Cin >= 4 &&
        256 % (Cin / 4) == 0 && Wo >= 1 && Wo <= 4096))
    return false;
  const long fwd = (long)RMAX * SMAX * Cin + RMAX * 64 * SMAX;
  const long wg = (long)(256 / (Cin / 4) - 1) * R * S * Cin + RMAX * (Wo + 2 * SMAX);
  return (fwd > wg ? fwd : wg) * 4 <= 160 * 1024;
}

int head_fwd_launch(const float* x, const float* wp, const float* bias, float* out, int N, int Hi, int Wi, int Cin,
                    int Ho, int Wo, int R, int S, int pad, int act, float slope, hipStream_t s) {
  // KS = 2 lanes per column when the row's columns fit 32 lanes, else one lane per column and
  // segments of 64 - S + 1 outputs
  const int ks = (Wo + S - 1 <= 32 && Cin % 8 == 0) ? 2 : 1;
  const int seg = ks == 2 ? Wo : (Wo + S - 1 <= 64 ? Wo : 64 - S + 1);
  const size_t lds = ((size_t)RMAX * SMAX * Cin + RMAX * (64 / ks) * SMAX) * sizeof(float);
  const dim3 grid(ceil_div(Wo, seg), Ho, N);
  if (ks == 2)
    hipLaunchKernelGGL(head_fwd_k<2>, grid, dim3(256), lds, s, x, wp, bias, out, Hi, Wi, Cin, Ho, Wo, R, S, pad, act,
                       slope, seg);
  else
    hipLaunchKernelGGL(head_fwd_k<1>, grid, dim3(256), lds, s, x, wp, bias, out, Hi, Wi, Cin, Ho, Wo, R, S, pad, act,
                       slope, seg);
  return check_launch("head_fwd");
}

// rows per weight-gradient block: about 160 blocks (the partial slabs stay small)
static int head_wgrad_rows(int N, int Hi) {
  const int G = ceil_div((long)N * Hi, 160);
  return G < 1 ? 1 : G;
}

size_t head_wgrad_ws_floats(int N, int Hi, int Cin, int R, int S) {
  const int G = head_wgrad_rows(N, Hi);
  return (size_t)N * ceil_div(Hi, G) * R * S * Cin;
}

int head_wgrad_launch(const float* x, const float* dy, float* dw, float* ws, int N, int Hi, int Wi, int Cin, int Ci,
                      int Ho, int Wo, int R, int S, int pad, long si, int accumulate, hipStream_t s, float* db) {
  const int G = head_wgrad_rows(N, Hi), nb = ceil_div(Hi, G);
  const int NG = 256 / (Cin / 4);
  const size_t lds = ((size_t)(NG - 1) * R * S * Cin + RMAX * (Wo + 2 * SMAX)) * sizeof(float);
  hipLaunchKernelGGL(head_wgrad_k, dim3(nb, N), dim3(256), lds, s, x, dy, ws, Hi, Wi, Cin, Ho, Wo, R, S, pad, G);
  int rc = check_launch("head_wgrad");
  if (rc) return rc;
  const int Mw = R * S * Cin;
  hipLaunchKernelGGL(head_wgrad_reduce_k, dim3(ceil_div(Mw, 16) + (db ? 1 : 0)), dim3(256), 0, s, ws, dw, Mw, Cin, Ci,
                     R * S, si, accumulate, N * nb, dy, (long)N * Ho * Wo, db);
  return check_launch("head_wgrad_reduce");
}

int head_dgrad_launch(const float* dy, const float* wp, const float* addend, float* dx, int N, int Hd, int Wd, int Cx,
                      int H, int W, int R, int S, int pad, hipStream_t s) {
  const size_t lds = (size_t)RMAX * (Wd + 2 * SMAX) * sizeof(float);
  hipLaunchKernelGGL(head_dgrad_k, dim3(H, N), dim3(256), lds, s, dy, wp, addend, dx, Hd, Wd, Cx, H, W, R, S, pad);
  return check_launch("head_dgrad");
}

}  // namespace vst

namespace vst {

// VST_IMG_WGRAD=0: image-input weight gradients on the split-bf16 GEMM (conv.hip) instead
const bool g_img_wgrad = [] {
  const char* e = getenv("VST_IMG_WGRAD");
  return !(e && e[0] == '0');
}();

bool img_wgrad_ok(int Cx, int Cyp, int R, int S, int st, int reflect, int Ci, int Wo) {
  return Cx == 4 && Ci <= 3 && Cyp % 2 == 0 && Cyp <= 64 && R * S <= 16 && st >= 1 && !reflect && Wo >= 1;
}

static long img_wgrad_blocks(long P) {
  // ~2 pixel-pair runs of >= 32 pairs per wave, at most 256 blocks (the partial slabs stay <= 4 MB)
  long b = (P + 64L * IW_WAVES - 1) / (64L * IW_WAVES);
  return b < 1 ? 1 : (b > 256 ? 256 : b);
}

size_t img_wgrad_ws_floats(int N, int Ho, int Wo) { return (size_t)img_wgrad_blocks((long)N * Ho * Wo) * 4096; }

int img_wgrad_launch(const float* x, const float* dy, float* dw, float* db, float* ws, int N, int H, int W, int Ho,
                     int Wo, int Cyp, int R, int S, int st, int pad, int Co, int Ci, long so, long si, int accumulate,
                     hipStream_t s) {
  const long P = (long)N * Ho * Wo;
  const long nb = img_wgrad_blocks(P);
  long ppw = (P + nb * IW_WAVES - 1) / (nb * IW_WAVES);
  ppw += ppw & 1;  // whole pixel pairs per wave
  const size_t lds = (size_t)(IW_WAVES - 1) * 4096 * sizeof(float);
  hipLaunchKernelGGL(img_wgrad_k, dim3((unsigned)nb), dim3(64 * IW_WAVES), lds, s, x, dy, ws, H, W, Ho, Wo, Cyp, R, S,
                     st, pad, Ci, db ? 1 : 0, P, (int)ppw);
  int rc = check_launch("img_wgrad");
  if (rc) return rc;
  hipLaunchKernelGGL(img_wgrad_reduce_k, dim3(256), dim3(256), 0, s, ws, dw, db, R * S, Co, Ci, so, si, accumulate,
                     (int)nb);
  return check_launch("img_wgrad_reduce");
}

}  // namespace vst
