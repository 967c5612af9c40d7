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

// Every kernel here issues its global loads in explicit batches before using them: on gfx950 a
// vector load waited on right after issue costs a full memory latency (~1 us under load), and a wait
// inside a loop that also stores drains the stores too (loads and stores share vmcnt).

// ---- forward -------------------------------------------------------------------------------------
// wp: the VST_PACK_OK pack [Cop][R][S][Cin]; only output channel 0 is computed (co_real = 1), the
// padded channels get act(bias[c]) like the 4-channel path's zero sums.  1024 threads: wave w takes
// input row h - pad + (w & 3) and channel quarter w >> 2; KS lanes per column split the quarter.
constexpr int HF_THREADS = 1024, HF_NQ = 4, HF_B = 16;

template <int KS>
__global__ __launch_bounds__(HF_THREADS) void head_fwd_k(const float* __restrict__ x, const float* __restrict__ wp,
                                                         const float* __restrict__ bias, float* __restrict__ out,
                                                         int Hi, int Wi, int Cin, int Ho, int Wo, int R, int S,
                                                         int pad, int act, float slope, int seg) {
  constexpr int NCOL = 64 / KS;
  extern __shared__ float lds[];
  float* wl = lds;                     // [R][S][Cin]
  float* zq = lds + RMAX * SMAX * Cin;  // [HF_NQ][RMAX][NCOL][SMAX]
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int r = wave & 3, qq = wave >> 2;
  const int n = blockIdx.z, h = blockIdx.y, w0 = blockIdx.x * seg;
  const int wn = R * S * Cin;
  for (int e = 4 * t; e < wn; e += 4 * HF_THREADS)
    *reinterpret_cast<float4*>(wl + e) = *reinterpret_cast<const float4*>(wp + e);
  __syncthreads();
  const int col = lane / KS, k = lane % KS;
  const int hi = h - pad + r, wi = w0 - pad + col;
  const int ncol = seg + S - 1;
  const bool valid = r < R && (unsigned)hi < (unsigned)Hi && col < ncol && (unsigned)wi < (unsigned)Wi;
  // channel slice (quarter qq, lane k): a contiguous run of cw channels
  const int cw = Cin / (HF_NQ * KS), c0 = (qq * KS + k) * cw;
  const float* src = x + (valid ? (((long)n * Hi + hi) * Wi + wi) * Cin : 0) + c0;
  const float* wr = wl + r * S * Cin + c0;
  float acc[SMAX] = {0.f, 0.f, 0.f, 0.f};
  if (r < R) {
    for (int cb = 0; cb < cw; cb += 4 * HF_B) {
      float4 v[HF_B];
#pragma unroll
      for (int u = 0; u < HF_B; ++u)
        if (cb + 4 * u < cw) v[u] = *reinterpret_cast<const float4*>(src + cb + 4 * u);
#pragma unroll
      for (int u = 0; u < HF_B; ++u) {
        if (cb + 4 * u >= cw) break;
#pragma unroll
        for (int s = 0; s < SMAX; ++s) {
          if (s >= S) break;
          const float4 w = *reinterpret_cast<const float4*>(wr + s * Cin + cb + 4 * u);
          acc[s] = fmaf(v[u].x, w.x, acc[s]);
          acc[s] = fmaf(v[u].y, w.y, acc[s]);
          acc[s] = fmaf(v[u].z, w.z, acc[s]);
          acc[s] = fmaf(v[u].w, w.w, acc[s]);
        }
      }
    }
  }
#pragma unroll
  for (int s = 0; s < SMAX; ++s) {
    acc[s] = valid ? acc[s] : 0.f;
#pragma unroll
    for (int o = KS / 2; o > 0; o >>= 1) acc[s] += __shfl_xor(acc[s], o, 64);
  }
  if (k == 0) {
#pragma unroll
    for (int s = 0; s < SMAX; ++s) zq[((qq * RMAX + r) * NCOL + col) * SMAX + s] = acc[s];
  }
  __syncthreads();
  if (t < seg && w0 + t < Wo) {
    float v = 0.f;
    for (int rr = 0; rr < R; ++rr)
      for (int s = 0; s < S; ++s)
#pragma unroll
        for (int q4 = 0; q4 < HF_NQ; ++q4) v += zq[((q4 * RMAX + rr) * NCOL + t + s) * SMAX + s];
    const float4 b4 = bias ? *reinterpret_cast<const float4*>(bias) : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 o;
    o.x = apply_act(v + b4.x, act, slope);
    o.y = apply_act(b4.y, act, slope);
    o.z = apply_act(b4.z, act, slope);
    o.w = apply_act(b4.w, act, slope);
    *reinterpret_cast<float4*>(out + (((long)n * Ho + h) * Wo + w0 + t) * 4) = o;
  }
}

// The forward as a tap GEMM over each input row, read ONCE (the row kernel above reads every input row
// once per kernel row r, i.e. R times, and is bound by that traffic):
//   head_tap_k     block = (input row i, image n): the row (JC columns at a time) and the channel-0
//                  weights [R*S][Cin] are staged in LDS with every load issued up front, then
//                  z[n][i][j][tap] = sum_c x[n][i][j][c] * w[tap][c] on v_mfma_f32_16x16x4_f32 (exact fp32
//                  products): M = 16 columns per block, N = the 16 taps, K = Cin split over the waves.
//                  A lane's ds_read_b128 of 4 consecutive channels feeds 4 MFMAs (channel c + 4(l>>4) + t
//                  to MFMA t, for both operands: the reduction order within a 16-channel group is free).
//   head_tapsum_k  out[n][h][w] = act(b + sum_{r,s} z[n][h-pad+r][w-pad+s][r*S+s]) in a fixed order.
constexpr int HT_THREADS = 256, HT_JC = 32;

__global__ __launch_bounds__(HT_THREADS) void head_tap_k(const float* __restrict__ x, const float* __restrict__ wp,
                                                         float* __restrict__ z, int Hi, int Wi, int Cin, int RS) {
  extern __shared__ float lds[];
  const int LD = Cin + 4;           // padded row stride (floats): the 16 rows of a read start 16 B apart
  float* xs = lds;                  // [HT_JC][LD]
  float* ws = lds + HT_JC * LD;     // [16][LD] (taps >= RS zero)
  float* zs = ws + 16 * LD;         // [4][HT_JC][16] per-wave partial z
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int n = blockIdx.y, i = blockIdx.x;
  const int Q = Cin / 4;
  // weights: 16 x Cin floats (rows >= RS zero), loads issued together
  {
    float4 v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = t + u * HT_THREADS, tap = e / Q, c4 = e - tap * Q;
      if (e < 16 * Q) v[u] = tap < RS ? *reinterpret_cast<const float4*>(wp + (long)tap * Cin + 4 * c4)
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = t + u * HT_THREADS, tap = e / Q, c4 = e - tap * Q;
      if (e < 16 * Q) *reinterpret_cast<float4*>(ws + tap * LD + 4 * c4) = v[u];
    }
  }
  const float* xr = x + ((long)n * Hi + i) * Wi * Cin;
  float* zr = z + ((long)n * Hi + i) * Wi * 16;
  const int l16 = lane & 15, kq = lane >> 4;
  for (int j0 = 0; j0 < Wi; j0 += HT_JC) {
    const int jn = Wi - j0 < HT_JC ? Wi - j0 : HT_JC;
    {
      float4 v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int e = t + u * HT_THREADS, j = e / Q, c4 = e - j * Q;
        if (e < HT_JC * Q) v[u] = j < jn ? *reinterpret_cast<const float4*>(xr + (long)(j0 + j) * Cin + 4 * c4)
                                         : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      __syncthreads();  // weights written / the previous chunk consumed
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int e = t + u * HT_THREADS, j = e / Q, c4 = e - j * Q;
        if (e < HT_JC * Q) *reinterpret_cast<float4*>(xs + j * LD + 4 * c4) = v[u];
      }
      __syncthreads();
    }
    // wave w: column block mb = w & 1 (16 columns), channel half kh = w >> 1
    const int mb = wave & 1, kh = wave >> 1, ch = Cin / 2;
    const float* pa = xs + (mb * 16 + l16) * LD + kh * ch + 4 * kq;
    const float* pb = ws + l16 * LD + kh * ch + 4 * kq;
    f32x4v acc = {0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < ch; c += 16) {
      const float4 a = *reinterpret_cast<const float4*>(pa + c);
      const float4 b = *reinterpret_cast<const float4*>(pb + c);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, acc, 0, 0, 0);
    }
    // C: column (tap) l & 15, rows (columns j) 4 (l >> 4) + reg
#pragma unroll
    for (int e = 0; e < 4; ++e) zs[(wave * HT_JC + mb * 16 + 4 * kq + e) * 16 + l16] = acc[e];
    __syncthreads();
    for (int e = t; e < jn * 16; e += HT_THREADS) {
      const int j = e >> 4, tap = e & 15, m = j >> 4;
      zr[(long)(j0 + j) * 16 + tap] = zs[(m * HT_JC + j) * 16 + tap] + zs[((2 + m) * HT_JC + j) * 16 + tap];
    }
  }
}

__global__ __launch_bounds__(256) void head_tapsum_k(const float* __restrict__ z, const float* __restrict__ bias,
                                                     float* __restrict__ out, int N, int Hi, int Wi, int Ho, int Wo,
                                                     int R, int S, int pad, int act, float slope) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= (long)N * Ho * Wo) return;
  const int w = (int)(p % Wo), h = (int)((p / Wo) % Ho), n = (int)(p / ((long)Wo * Ho));
  float zv[RMAX * SMAX];
#pragma unroll
  for (int r = 0; r < RMAX; ++r)
#pragma unroll
    for (int s = 0; s < SMAX; ++s) {
      const int hi = h - pad + r, wi = w - pad + s;
      const bool ok = r < R && s < S && (unsigned)hi < (unsigned)Hi && (unsigned)wi < (unsigned)Wi;
      zv[r * SMAX + s] = ok ? z[(((long)n * Hi + hi) * Wi + wi) * 16 + r * S + s] : 0.f;
    }
  float v = 0.f;
#pragma unroll
  for (int e = 0; e < RMAX * SMAX; ++e) v += zv[e];
  const float4 b4 = bias ? *reinterpret_cast<const float4*>(bias) : make_float4(0.f, 0.f, 0.f, 0.f);
  float4 o;
  o.x = apply_act(v + b4.x, act, slope);
  o.y = apply_act(b4.y, act, slope);
  o.z = apply_act(b4.z, act, slope);
  o.w = apply_act(b4.w, act, slope);
  *reinterpret_cast<float4*>(out + p * 4) = o;
}

// ---- weight gradient -----------------------------------------------------------------------------
// part[zb][(r*S + s)*Cin + c] = sum over input row i (block zb = (n, i)) and its columns j of
// x[n][i][j][c] * dy[n][i+pad-r][j+pad-s][0]   (zero outside dy).  1024 threads: channel quad q = t % Q
// (Q = Cin / 4), kernel row r = (t / Q) % 4, column group g = t / (4Q) (NG = 256 / Q groups).  The row
// is staged into LDS in chunks of JC columns (all of a thread's loads issued together), dy's rows
// i + pad - r too (zero outside the image, so the tap loop has no bounds tests).
constexpr int HW_THREADS = 1024;

__global__ __launch_bounds__(HW_THREADS) void head_wgrad_k(const float* __restrict__ x, const float* __restrict__ dy,
                                                           float* __restrict__ part, int Hi, int Wi, int Cin, int Ho,
                                                           int Wo, int R, int S, int pad, int JC) {
  extern __shared__ float lds[];
  const int DW = Wo + 2 * SMAX;
  const int Q = Cin / 4, NG = HW_THREADS / (4 * Q);
  float* xs = lds;                    // [JC][Cin]
  float* dl = xs + JC * Cin;          // [RMAX][DW]
  float* xg = dl + RMAX * DW;         // [NG - 1][RMAX*SMAX][Cin]
  const int t = threadIdx.x, q = t % Q, r = (t / Q) & 3, g = t / (4 * Q);
  const int n = blockIdx.y, i = blockIdx.x;
  const float* dyn = dy + (long)n * Ho * Wo * 4;
  for (int e = t; e < RMAX * DW; e += HW_THREADS) {
    const int rr = e / DW, ww = e - rr * DW - SMAX, hh = i + pad - rr;
    dl[e] = (rr < R && (unsigned)hh < (unsigned)Ho && (unsigned)ww < (unsigned)Wo) ? dyn[((long)hh * Wo + ww) * 4]
                                                                                   : 0.f;
  }
  float4 acc[SMAX];
#pragma unroll
  for (int s = 0; s < SMAX; ++s) acc[s] = make_float4(0.f, 0.f, 0.f, 0.f);
  const float* xr = x + ((long)n * Hi + i) * Wi * Cin;
  for (int j0 = 0; j0 < Wi; j0 += JC) {
    const int jn = Wi - j0 < JC ? Wi - j0 : JC;
    const int nf4 = jn * Q;  // float4s of this chunk: <= 4 per thread (JC * Cin <= 16384)
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (t + u * HW_THREADS < nf4) v[u] = *reinterpret_cast<const float4*>(xr + (long)j0 * Cin + 4 * (t + u * HW_THREADS));
    __syncthreads();  // the previous chunk is consumed
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (t + u * HW_THREADS < nf4) *reinterpret_cast<float4*>(xs + 4 * (t + u * HW_THREADS)) = v[u];
    __syncthreads();
    const float* dj = dl + r * DW + SMAX + j0 + pad;
    for (int j = g; j < jn; j += NG) {
      const float4 xv = *reinterpret_cast<const float4*>(xs + j * Cin + 4 * q);
#pragma unroll
      for (int s = 0; s < SMAX; ++s) {
        const float d = dj[j - s];
        acc[s].x = fmaf(xv.x, d, acc[s].x);
        acc[s].y = fmaf(xv.y, d, acc[s].y);
        acc[s].z = fmaf(xv.z, d, acc[s].z);
        acc[s].w = fmaf(xv.w, d, acc[s].w);
      }
    }
  }
  const int RS = R * S;
  if (g > 0 && r < R) {
#pragma unroll
    for (int s = 0; s < SMAX; ++s)
      if (s < S) *reinterpret_cast<float4*>(xg + ((long)(g - 1) * RS + r * S + s) * Cin + 4 * q) = acc[s];
  }
  __syncthreads();
  if (g == 0 && r < R) {
    float* dst = part + ((long)n * gridDim.x + i) * RS * Cin + 4 * q;
#pragma unroll
    for (int s = 0; s < SMAX; ++s) {
      if (s >= S) continue;
      float4 a = acc[s];
      for (int gg = 1; gg < NG; ++gg)
        add_f4(a, *reinterpret_cast<const float4*>(xg + ((long)(gg - 1) * RS + r * S + s) * Cin + 4 * q));
      *reinterpret_cast<float4*>(dst + (long)(r * S + s) * Cin) = a;
    }
  }
}

// Fixed-order sum of the 256 threads' values v (thread order in 16-groups) -> thread 0.
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
  long p = threadIdx.x;
  for (; p + 768 < P; p += 1024) {
    const float a0 = dy[p * 4], a1 = dy[(p + 256) * 4], a2 = dy[(p + 512) * 4], a3 = dy[(p + 768) * 4];
    a += a0;
    a += a1;
    a += a2;
    a += a3;
  }
  for (; p < P; p += 256) a += dy[p * 4];
  const float s = block_sum_fixed(a, red);
  if (threadIdx.x == 0) db[0] = accumulate ? db[0] + s : s;
}

// out[m] = sum_z part[z][m] for one output m of a 16-wide block column, slab group u = 0..15 (slabs
// u, u + 16, ... in order, loaded 8 at a time), then the 16 group sums in order.
__device__ __forceinline__ float slab_sum16(const float* __restrict__ part, long Mw, long m, int nz, bool ok,
                                            float (*red)[17]) {
  const int t = threadIdx.x, o = t & 15, u = t >> 4;
  float a = 0.f;
  if (ok) {
    for (int z0 = u; z0 < nz; z0 += 128) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (z0 + 16 * e < nz) v[e] = part[(long)(z0 + 16 * e) * Mw + m];
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (z0 + 16 * e < nz) a += v[e];
    }
  }
  red[u][o] = a;
  __syncthreads();
  float s = 0.f;
  if (u == 0) {
    s = red[0][o];
    for (int k = 1; k < 16; ++k) s += red[k][o];
  }
  return s;
}

// dw[ci*si + rs] (+)= sum_z part[z][rs*Cin + ci] in a fixed order (block = 16 outputs x 16 slab groups).
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
  const int m = blockIdx.x * 16 + (threadIdx.x & 15);
  const float s = slab_sum16(part, Mw, m, nz, m < Mw, red);
  const int rs = m / Cin, ci = m - rs * Cin;
  if (threadIdx.x < 16 && m < Mw && ci < Ci) {
    float* d = dw + (long)ci * si + rs;
    *d = accumulate ? *d + s : s;
  }
}

// ---- data gradient -------------------------------------------------------------------------------
// dx[n][i][j][c] = sum_{r,s} dy[n][i+pad-r][j+pad-s][0] * w[c][r][s][0] (+ addend): wp = the VST_PACK_IK
// pack [Cx][R][S][Cy] with Cy = 4 of which only channel 0 is real (co_real = 1).  Block = (input row i,
// image n): the channel-0 weights [R*S][Cx] and dy's rows i + pad - r go to LDS first (loads batched),
// each thread then holds its 4 channels' R*S weights in registers, so the column loop issues only LDS
// reads and the stores.
constexpr int HD_THREADS = 256;

__global__ __launch_bounds__(HD_THREADS) void head_dgrad_k(const float* __restrict__ dy, const float* __restrict__ wp,
                                                           const float* __restrict__ addend, float* __restrict__ dx,
                                                           int Hd, int Wd, int Cx, int H, int W, int R, int S,
                                                           int pad) {
  extern __shared__ float lds[];
  const int DW = Wd + 2 * SMAX, RS = R * S;
  float* wl = lds;                   // [RMAX*SMAX][Cx]
  float* dl = lds + RMAX * SMAX * Cx;  // [RMAX][DW]
  const int t = threadIdx.x, Q = Cx / 4, NG = HD_THREADS / Q;
  const int q = t % Q, g = t / Q;
  const int n = blockIdx.y, i = blockIdx.x;
  const float* dyn = dy + (long)n * Hd * Wd * 4;
  // weights: element e = c * RS + tap of the channel-0 column (IK pack stride 4 floats)
  const int nw = Cx * RS;
  for (int e0 = 0; e0 < nw; e0 += 16 * HD_THREADS) {
    float v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u)
      if (e0 + t + u * HD_THREADS < nw) v[u] = wp[(long)(e0 + t + u * HD_THREADS) * 4];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = e0 + t + u * HD_THREADS;
      if (e < nw) {
        const int c = e / RS, tap = e - c * RS;
        wl[tap * Cx + c] = v[u];
      }
    }
  }
  for (int e = t; e < RMAX * DW; e += HD_THREADS) {
    const int rr = e / DW, ww = e - rr * DW - SMAX, hh = i + pad - rr;
    dl[e] = (rr < R && (unsigned)hh < (unsigned)Hd && (unsigned)ww < (unsigned)Wd) ? dyn[((long)hh * Wd + ww) * 4]
                                                                                  : 0.f;
  }
  __syncthreads();
  float4 wv[RMAX * SMAX];
#pragma unroll
  for (int r = 0; r < RMAX; ++r)
#pragma unroll
    for (int s = 0; s < SMAX; ++s)
      wv[r * SMAX + s] = (r < R && s < S) ? *reinterpret_cast<const float4*>(wl + (r * S + s) * Cx + 4 * q)
                                          : make_float4(0.f, 0.f, 0.f, 0.f);
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
// walks a contiguous run of pixel pairs, IW_B pairs' loads issued before their MFMAs; the block's waves
// add their 64 x 64 tiles in LDS in a fixed order into one partial slab part[block][j][co], reduced by
// img_wgrad_reduce_k.
constexpr int IW_WAVES = 8, IW_B = 16;

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
  const float mx = c0 < Ci ? 1.f : 0.f, my = c0 + 1 < Ci ? 1.f : 0.f;
  const bool bias_slot = want_db && rs == 0 && c0 + 1 == 3;
  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;
  const long wid = (long)blockIdx.x * IW_WAVES + wave;
  const long p0 = wid * ppw, p1 = p0 + ppw < P ? p0 + ppw : P;
  // this lane's pixel cursor (n, ho, wo) for p = pb + kk, advanced 2 pixels per pair
  long p = p0 + kk;
  int cn, cho, cwo;
  {
    const long HWo = (long)Ho * Wo;
    const long pp = p < P ? p : P - 1;
    cn = (int)(pp / HWo);
    const int rem = (int)(pp - (long)cn * HWo);
    cho = rem / Wo;
    cwo = rem - cho * Wo;
  }
  for (long pb = p0; pb < p1; pb += 2 * IW_B) {
    float2 av[IW_B], bv[IW_B];
    float live[IW_B];
#pragma unroll
    for (int u = 0; u < IW_B; ++u) {
      const bool ok = p < p1;
      const int hi = st * cho - pad + r, wi = st * cwo - pad + s;
      const bool in = ok && tap_ok && (unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W;
      const long pd = ok ? p : p0;  // p0 < P: a valid row to read when this lane is past its run
      av[u] = co_ok ? *reinterpret_cast<const float2*>(dy + pd * Cyp + 2 * i) : make_float2(0.f, 0.f);
      bv[u] = in ? *reinterpret_cast<const float2*>(x + ((((long)cn * H + hi) * W + wi) << 2) + c0)
                 : make_float2(0.f, 0.f);
      live[u] = ok ? 1.f : 0.f;
      p += 2;
      cwo += 2;
      while (cwo >= Wo) {
        cwo -= Wo;
        if (++cho == Ho) {
          cho = 0;
          ++cn;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < IW_B; ++u) {
      const float a0 = av[u].x * live[u], a1 = av[u].y * live[u];
      const float b0 = bv[u].x * mx, b1 = bias_slot ? live[u] : bv[u].y * my;
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
  }
  // The block's 8 wave tiles are summed in register order (tl[w][(2a + b) * 16 + e][lane]: conflict-free
  // LDS rows) and the partial slab keeps that order; img_wgrad_reduce_k maps it to (co, j).
  if (wave > 0) {
    float* d = tl + (long)(wave - 1) * 4096 + lane;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int e = 0; e < 16; ++e) d[((2 * a + b) * 16 + e) * 64] = acc[a][b][e];
  }
  __syncthreads();
  if (wave == 0) {
    float* dst = part + (long)blockIdx.x * 4096 + lane;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int o = ((2 * a + b) * 16 + e) * 64;
          float v = acc[a][b][e];
          for (int w = 0; w < IW_WAVES - 1; ++w) v += tl[(long)w * 4096 + o + lane];
          dst[o] = v;
        }
  }
}

// dw[co*so + ci*si + rs] (+)= sum_z C[co][j] (j = rs*4 + ci, ci < Ci, co < Co), db[co] (+)= sum_z C[co][3];
// part[z] holds C in the MFMA register order [(2a + b) * 16 + e][lane]: lane = i + 32 kk, column j =
// 2 i + b, row co = 2 (8 (e / 4) + 4 kk + e % 4) + a.  Fixed order: block = 16 outputs x 16 slab groups.
__global__ __launch_bounds__(256) void img_wgrad_reduce_k(const float* __restrict__ part, float* __restrict__ dw,
                                                          float* __restrict__ db, int RS, int Co, int Ci, long so,
                                                          long si, int accumulate, int nz) {
  __shared__ float red[16][17];
  const int m = blockIdx.x * 16 + (threadIdx.x & 15);
  const float v = slab_sum16(part, 4096, m, nz, true, red);
  const int lane = m & 63, ab = m >> 10, e = (m >> 6) & 15;
  const int a = ab >> 1, b = ab & 1, i = lane & 31, kk = lane >> 5;
  const int j = 2 * i + b, co = 2 * (8 * (e >> 2) + 4 * kk + (e & 3)) + a;
  const int rs = j >> 2, ci = j & 3;
  if (threadIdx.x >= 16 || co >= Co) return;
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
  // Cin / 4 channel quads must divide the threads (quads x kernel rows x column groups), Cin % 16 for
  // the forward's channel quarters; the LDS images (weights, the weight gradient's row chunk and
  // cross-group partials, dy rows) must fit
  if (!(st == 1 && !reflect && R >= 1 && R <= RMAX && S >= 1 && S <= SMAX && Cin % 16 == 0 && Cin >= 16 &&
        Cin <= 1024 && (Cin & (Cin - 1)) == 0 && Wo >= 1 && Wo <= 2048))
    return false;
  const long fwd = (long)RMAX * SMAX * Cin + HF_NQ * RMAX * 64 * SMAX;
  const long wg = 16384 + RMAX * (Wo + 2 * SMAX) + (long)(HW_THREADS / Cin - 1) * RMAX * SMAX * Cin;
  const long dg = (long)RMAX * SMAX * Cin + RMAX * (Wo + 2 * SMAX);
  const long mx = fwd > wg ? (fwd > dg ? fwd : dg) : (wg > dg ? wg : dg);
  return mx * 4 <= 160 * 1024;
}

int head_fwd_launch(const float* x, const float* wp, const float* bias, float* out, int N, int Hi, int Wi, int Cin,
                    int Ho, int Wo, int R, int S, int pad, int act, float slope, hipStream_t s) {
  // KS = 2 lanes per column when the row's columns fit 32 lanes, else one lane per column and
  // segments of 64 - S + 1 outputs
  const int ks = (Wo + S - 1 <= 32 && Cin % 32 == 0) ? 2 : 1;
  const int seg = ks == 2 ? Wo : (Wo + S - 1 <= 64 ? Wo : 64 - S + 1);
  const size_t lds = ((size_t)RMAX * SMAX * Cin + HF_NQ * RMAX * (64 / ks) * SMAX) * sizeof(float);
  const dim3 grid(ceil_div(Wo, seg), Ho, N);
  if (ks == 2)
    hipLaunchKernelGGL(head_fwd_k<2>, grid, dim3(HF_THREADS), lds, s, x, wp, bias, out, Hi, Wi, Cin, Ho, Wo, R, S, pad,
                       act, slope, seg);
  else
    hipLaunchKernelGGL(head_fwd_k<1>, grid, dim3(HF_THREADS), lds, s, x, wp, bias, out, Hi, Wi, Cin, Ho, Wo, R, S, pad,
                       act, slope, seg);
  return check_launch("head_fwd");
}

size_t head_tap_ws_floats(int N, int Hi, int Wi) { return (size_t)N * Hi * Wi * 16; }

bool head_tap_ok(int Cin) {
  // K halves of whole 16-channel groups; the row chunk + weights + partials fit the LDS; head_tap_k stages a row
  // chunk (HT_JC pixels x Cin / 4 float4) in at most 16 passes of HT_THREADS lanes: Cin <= 512
  return Cin % 32 == 0 && HT_JC * Cin / 4 <= 16 * HT_THREADS &&
         ((size_t)(HT_JC + 16) * (Cin + 4) + 4 * HT_JC * 16) * 4 <= 160 * 1024;
}

int head_tap_fwd_launch(const float* x, const float* wp, const float* bias, float* out, float* ws, int N, int Hi,
                        int Wi, int Cin, int Ho, int Wo, int R, int S, int pad, int act, float slope, hipStream_t s) {
  const size_t lds = ((size_t)(HT_JC + 16) * (Cin + 4) + 4 * HT_JC * 16) * sizeof(float);
  hipLaunchKernelGGL(head_tap_k, dim3(Hi, N), dim3(HT_THREADS), lds, s, x, wp, ws, Hi, Wi, Cin, R * S);
  int rc = check_launch("head_tap");
  if (rc) return rc;
  hipLaunchKernelGGL(head_tapsum_k, dim3(ceil_div((long)N * Ho * Wo, 256)), dim3(256), 0, s, ws, bias, out, N, Hi, Wi,
                     Ho, Wo, R, S, pad, act, slope);
  return check_launch("head_tapsum");
}

size_t head_wgrad_ws_floats(int N, int Hi, int Cin, int R, int S) { return (size_t)N * Hi * R * S * Cin; }

int head_wgrad_launch(const float* x, const float* dy, float* dw, float* ws, int N, int Hi, int Wi, int Cin, int Ci,
                      int Ho, int Wo, int R, int S, int pad, long si, int accumulate, hipStream_t s, float* db) {
  int JC = 16384 / Cin;
  if (JC > Wi) JC = Wi;
  const int NG = HW_THREADS / Cin;  // column groups: 1024 threads / (Cin / 4 quads x 4 kernel rows)
  const size_t lds = ((size_t)JC * Cin + RMAX * (Wo + 2 * SMAX) + (size_t)(NG - 1) * R * S * Cin) * sizeof(float);
  hipLaunchKernelGGL(head_wgrad_k, dim3(Hi, N), dim3(HW_THREADS), lds, s, x, dy, ws, Hi, Wi, Cin, Ho, Wo, R, S, pad,
                     JC);
  int rc = check_launch("head_wgrad");
  if (rc) return rc;
  const int Mw = R * S * Cin;
  hipLaunchKernelGGL(head_wgrad_reduce_k, dim3(ceil_div(Mw, 16) + (db ? 1 : 0)), dim3(256), 0, s, ws, dw, Mw, Cin, Ci,
                     R * S, si, accumulate, N * Hi, dy, (long)N * Ho * Wo, db);
  return check_launch("head_wgrad_reduce");
}

int head_dgrad_launch(const float* dy, const float* wp, const float* addend, float* dx, int N, int Hd, int Wd, int Cx,
                      int H, int W, int R, int S, int pad, hipStream_t s) {
  const size_t lds = ((size_t)RMAX * SMAX * Cx + RMAX * (Wd + 2 * SMAX)) * sizeof(float);
  hipLaunchKernelGGL(head_dgrad_k, dim3(H, N), dim3(HD_THREADS), lds, s, dy, wp, addend, dx, Hd, Wd, Cx, H, W, R, S,
                     pad);
  return check_launch("head_dgrad");
}

}  // namespace vst

namespace vst {

// g_img_wgrad = false: image-input weight gradients on the split-bf16 GEMM (conv.hip) instead
const bool g_img_wgrad = true;

bool img_wgrad_ok(int Cx, int Cyp, int R, int S, int st, int reflect, int Ci, int Wo) {
  return Cx == 4 && Ci <= 3 && Cyp % 2 == 0 && Cyp <= 64 && R * S <= 16 && st >= 1 && !reflect && Wo >= 1;
}

static long img_wgrad_blocks(long P) {
  // 2 x IW_B pixel pairs (64 pixels) per wave, at most 512 blocks (the partial slabs stay <= 8 MB)
  long b = (P + 64L * IW_WAVES - 1) / (64L * IW_WAVES);
  return b < 1 ? 1 : (b > 512 ? 512 : b);
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
  hipLaunchKernelGGL(img_wgrad_reduce_k, dim3(4096 / 16), dim3(256), 0, s, ws, dw, db, R * S, Co, Ci, so, si,
                     accumulate, (int)nb);
  return check_launch("img_wgrad_reduce");
}

}  // namespace vst
