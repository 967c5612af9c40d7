// Implicit-GEMM convolution kernels on gfx950 fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// Replaces the cuDNN conv fprop / dgrad / wgrad that nn.Conv2d, nn.ConvTranspose2d and
// nn.ReflectionPad2d dispatch in the reference ResnetGenerator / NLayerDiscriminator
// (methods/GAN-based/CycleGAN/models/networks.py:340-367, 404-426, 556-578).
//
// All three kernels compute a tile C[BM x BN] = sum_k A[m][k] * B[k][n] with
//   * 256 threads = 4 waves, each wave owning a WM x WN sub-tile of 32x32 MFMA blocks,
//   * BK = 32 deep K-steps double-buffered in LDS (one barrier per K-step); both LDS operand
//     images are k-major ([k][row], row contiguous, +4 float pad) so every MFMA operand fetch is
//     a conflict-free ds_read_b32 over 32 consecutive rows,
//   * the next K-step's global loads issued into registers before the MFMAs of the current one
//     (register-staged pipeline), written to the other LDS buffer after them.
// Operand gathers fold the padding (zero or reflect) and the stride into address generation, so
// no im2col / padded copy is ever materialised.  fp32 MFMA is exact fp32 fma arithmetic, which is
// what keeps the path within the reference's fp32 tolerance.
//
//   conv_fprop_k  : y = conv(x, w)         m = output pixel, n = out channel, k = (r, s, ci)
//   conv_tconv_k  : transposed conv / dgrad, gathered per output-parity class (blockIdx.z), so a
//                   stride-2 layer only walks the taps that hit each class (no zero-insertion)
//   conv_wgrad_k  : dw = x_gather^T * dy    m = (r, s, ci) [+ one all-ones row -> bias grad],
//                   n = out channel, k = pixel; split-K over blockIdx.z into an fp32 slab,
//                   reduced deterministically by wgrad_reduce_k.
#include "common.h"

namespace vst {

constexpr int NT = 256;
constexpr int BK = 32;

template <int BM, int BN, int WM, int WN>
struct Tile {
  static constexpr int LDA = BM + 4;
  static constexpr int LDB = BN + 4;
  static constexpr int WAVES_N = BN / WN;
  static constexpr int MI = WM / 32;
  static constexpr int NI = WN / 32;
  static constexpr int A_ELEMS = BK * LDA;
  static constexpr int B_ELEMS = BK * LDB;
  static_assert((BM / WM) * (BN / WN) == 4, "4 waves per block");
  static_assert(WM % 32 == 0 && WN % 32 == 0, "32x32 MFMA blocks");
};

// MFMA over one BK-deep LDS stage.
template <int BM, int BN, int WM, int WN>
__device__ __forceinline__ void mma_stage(const float* __restrict__ As, const float* __restrict__ Bs,
                                          f32x16 (&acc)[WM / 32][WN / 32], int wm0, int wn0, int lane) {
  using T = Tile<BM, BN, WM, WN>;
  const int kh = lane >> 5, li = lane & 31;
#pragma unroll
  for (int kk = 0; kk < BK / 2; ++kk) {
    const int krow = 2 * kk + kh;
    float a[T::MI], b[T::NI];
#pragma unroll
    for (int i = 0; i < T::MI; ++i) a[i] = As[krow * T::LDA + wm0 + 32 * i + li];
#pragma unroll
    for (int j = 0; j < T::NI; ++j) b[j] = Bs[krow * T::LDB + wn0 + 32 * j + li];
#pragma unroll
    for (int i = 0; i < T::MI; ++i)
#pragma unroll
      for (int j = 0; j < T::NI; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
  }
}

// XCD-aware remap of the M-tile index: consecutive M tiles (neighbouring pixel rows, which share
// halo rows) land on the same XCD / L2 (blocks b and b+8 share an XCD under round-robin dispatch).
__device__ __forceinline__ int remap_mtile(int bx, int nx) {
  if ((nx & 7) != 0) return bx;
  return (bx & 7) * (nx >> 3) + (bx >> 3);
}

// ------------------------------------------------------------------------------------------ fprop
template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(NT, 2) void conv_fprop_k(
    const float* __restrict__ x, const float* __restrict__ wp, const float* __restrict__ bias,
    float* __restrict__ y, int H, int W, int C, int Ho, int Wo, int Cop, int S, int st, int pad,
    int reflect, int act, float slope, int M, int Ktot) {
  using T = Tile<BM, BN, WM, WN>;
  constexpr int KSTEP4 = NT / BM;             // k4 stride between a thread's A loads
  constexpr int A_LD = BK / 4 / KSTEP4;       // float4 A loads per thread per stage
  constexpr int BN4 = BN / 4;
  constexpr int KRSTEP = NT / BN4;
  constexpr int B_LD = BK / KRSTEP;
  static_assert(NT % BM == 0 && A_LD >= 1 && B_LD >= 1, "tile shape");
  __shared__ __attribute__((aligned(16))) float smem[2 * (T::A_ELEMS + T::B_ELEMS)];

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int mt = remap_mtile(blockIdx.x, gridDim.x);
  const int m0 = mt * BM, n0 = blockIdx.y * BN;

  // ---- A gather state: one output pixel per thread, A_LD k-offsets
  const int ml = t % BM, k4b = t / BM;
  const int m = m0 + ml;
  const bool mval = m < M;
  int hb = 0, wb = 0;
  long ibase = 0;
  if (mval) {
    const int hw = Ho * Wo;
    const int n = m / hw, rem = m - n * hw, ho = rem / Wo, wo = rem - (rem / Wo) * Wo;
    hb = ho * st - pad;
    wb = wo * st - pad;
    ibase = (long)n * H * W * C;
  }
  int ac[A_LD], as_[A_LD], ar[A_LD];
#pragma unroll
  for (int j = 0; j < A_LD; ++j) {
    const int k = 4 * (k4b + KSTEP4 * j);
    ac[j] = k % C;
    const int rs = k / C;
    ar[j] = rs / S;
    as_[j] = rs - ar[j] * S;
  }
  // ---- B state
  const int bn4 = t % BN4, bkr = t / BN4;
  const int bcol = n0 + 4 * bn4;
  const bool bcval = bcol < Cop;

  float4 ra[A_LD], rb[B_LD];
  auto load_a = [&](int k0) {
#pragma unroll
    for (int j = 0; j < A_LD; ++j) {
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      const int kk = k0 + 4 * (k4b + KSTEP4 * j);
      if (mval && kk < Ktot) {
        int hi = hb + ar[j], wi = wb + as_[j];
        bool ok = true;
        if (reflect) {
          hi = reflect_idx(hi, H);
          wi = reflect_idx(wi, W);
        } else {
          ok = (unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W;
        }
        if (ok) v = *reinterpret_cast<const float4*>(x + ibase + ((long)hi * W + wi) * C + ac[j]);
      }
      ra[j] = v;
    }
  };
  auto adv_a = [&]() {
#pragma unroll
    for (int j = 0; j < A_LD; ++j) {
      ac[j] += BK;
      while (ac[j] >= C) {
        ac[j] -= C;
        if (++as_[j] == S) { as_[j] = 0; ++ar[j]; }
      }
    }
  };
  auto load_b = [&](int k0) {
#pragma unroll
    for (int j = 0; j < B_LD; ++j) {
      const int kr = k0 + bkr + KRSTEP * j;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (bcval && kr < Ktot) v = *reinterpret_cast<const float4*>(wp + (long)kr * Cop + bcol);
      rb[j] = v;
    }
  };
  auto store = [&](int buf) {
    float* As = smem + buf * (T::A_ELEMS + T::B_ELEMS);
    float* Bs = As + T::A_ELEMS;
#pragma unroll
    for (int j = 0; j < A_LD; ++j) {
      const int kr = 4 * (k4b + KSTEP4 * j);
      As[(kr + 0) * T::LDA + ml] = ra[j].x;
      As[(kr + 1) * T::LDA + ml] = ra[j].y;
      As[(kr + 2) * T::LDA + ml] = ra[j].z;
      As[(kr + 3) * T::LDA + ml] = ra[j].w;
    }
#pragma unroll
    for (int j = 0; j < B_LD; ++j)
      *reinterpret_cast<float4*>(Bs + (bkr + KRSTEP * j) * T::LDB + 4 * bn4) = rb[j];
  };

  f32x16 acc[T::MI][T::NI];
#pragma unroll
  for (int i = 0; i < T::MI; ++i)
#pragma unroll
    for (int j = 0; j < T::NI; ++j)
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int wm0 = (wave / T::WAVES_N) * WM, wn0 = (wave % T::WAVES_N) * WN;
  const int nk = (Ktot + BK - 1) / BK;
  load_a(0);
  load_b(0);
  store(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      adv_a();
      load_a((kt + 1) * BK);
      load_b((kt + 1) * BK);
    }
    const float* As = smem + cur * (T::A_ELEMS + T::B_ELEMS);
    mma_stage<BM, BN, WM, WN>(As, As + T::A_ELEMS, acc, wm0, wn0, lane);
    if (kt + 1 < nk) store(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue: bias + activation, NHWC store (32 consecutive channels per half-wave)
#pragma unroll
  for (int i = 0; i < T::MI; ++i)
#pragma unroll
    for (int j = 0; j < T::NI; ++j) {
      const int n = n0 + wn0 + 32 * j + (lane & 31);
      if (n >= Cop) continue;
      const float bv = bias ? bias[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int mm = m0 + wm0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (mm < M) y[(long)mm * Cop + n] = apply_act(acc[i][j][r] + bv, act, slope);
      }
    }
}

// ------------------------------------------------------------------- transposed conv / dgrad
// out[n][h][w][cx] = sum in[n][ho][wo][cy] * wp[r][s][cy][cx] over h = ho*st - pad + r.
// blockIdx.z = parity class (a, b): h = a + st*hh, w = b + st*ww; only taps r = r0 + st*i with
// r0 = (a + pad) mod st contribute, at ho = (h + pad - r) / st (exact).
template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(NT, 2) void conv_tconv_k(
    const float* __restrict__ in, const float* __restrict__ wp, const float* __restrict__ bias,
    float* __restrict__ out, int Hi, int Wi, int Cy, int Ho, int Wo, int Cx, int R, int S, int st,
    int pad, int act, float slope, int Nimg) {
  using T = Tile<BM, BN, WM, WN>;
  constexpr int KSTEP4 = NT / BM;
  constexpr int A_LD = BK / 4 / KSTEP4;
  constexpr int BN4 = BN / 4;
  constexpr int KRSTEP = NT / BN4;
  constexpr int B_LD = BK / KRSTEP;
  __shared__ __attribute__((aligned(16))) float smem[2 * (T::A_ELEMS + T::B_ELEMS)];

  const int ca = blockIdx.z / st, cb = blockIdx.z % st;
  const int Hc = Ho > ca ? (Ho - ca + st - 1) / st : 0;
  const int Wc = Wo > cb ? (Wo - cb + st - 1) / st : 0;
  const int M = Nimg * Hc * Wc;
  const int mt = remap_mtile(blockIdx.x, gridDim.x);
  const int m0 = mt * BM, n0 = blockIdx.y * BN;
  if (m0 >= M) return;
  const int r0 = (ca + pad) % st, s0 = (cb + pad) % st;
  const int nr = r0 < R ? (R - r0 + st - 1) / st : 0;
  const int ns = s0 < S ? (S - s0 + st - 1) / st : 0;
  const int Ktot = nr * ns * Cy;

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int ml = t % BM, k4b = t / BM;
  const int m = m0 + ml;
  const bool mval = m < M;
  int hp = 0, wq = 0;
  long ibase = 0;
  if (mval) {
    const int hw = Hc * Wc;
    const int n = m / hw, rem = m - n * hw, hh = rem / Wc, ww = rem - hh * Wc;
    hp = ca + st * hh + pad;
    wq = cb + st * ww + pad;
    ibase = (long)n * Hi * Wi * Cy;
  }
  int ac[A_LD], ais[A_LD], air[A_LD];
#pragma unroll
  for (int j = 0; j < A_LD; ++j) {
    const int k = 4 * (k4b + KSTEP4 * j);
    ac[j] = Cy > 0 ? k % Cy : 0;
    const int tp = Cy > 0 ? k / Cy : 0;
    air[j] = ns > 0 ? tp / ns : 0;
    ais[j] = tp - air[j] * ns;
  }
  const int bn4 = t % BN4, bkr = t / BN4;
  const int bcol = n0 + 4 * bn4;
  const bool bcval = bcol < Cx;

  float4 ra[A_LD], rb[B_LD];
  auto load_a = [&](int k0) {
#pragma unroll
    for (int j = 0; j < A_LD; ++j) {
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      const int kk = k0 + 4 * (k4b + KSTEP4 * j);
      if (mval && kk < Ktot) {
        const int r = r0 + st * air[j], s = s0 + st * ais[j];
        const int ho = (hp - r) / st, wo = (wq - s) / st;
        if (hp - r >= 0 && wq - s >= 0 && ho < Hi && wo < Wi)
          v = *reinterpret_cast<const float4*>(in + ibase + ((long)ho * Wi + wo) * Cy + ac[j]);
      }
      ra[j] = v;
    }
  };
  auto adv_a = [&]() {
#pragma unroll
    for (int j = 0; j < A_LD; ++j) {
      ac[j] += BK;
      while (ac[j] >= Cy) {
        ac[j] -= Cy;
        if (++ais[j] == ns) { ais[j] = 0; ++air[j]; }
      }
    }
  };
  // B rows follow the same k decomposition (tap, cy) but index the full [R][S][Cy] row space.
  auto load_b = [&](int k0) {
#pragma unroll
    for (int j = 0; j < B_LD; ++j) {
      const int kk = k0 + bkr + KRSTEP * j;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (bcval && kk < Ktot) {
        const int cy = kk % Cy, tp = kk / Cy;
        const int ir = tp / ns, is = tp - ir * ns;
        const int row = ((r0 + st * ir) * S + (s0 + st * is)) * Cy + cy;
        v = *reinterpret_cast<const float4*>(wp + (long)row * Cx + bcol);
      }
      rb[j] = v;
    }
  };
  auto store = [&](int buf) {
    float* As = smem + buf * (T::A_ELEMS + T::B_ELEMS);
    float* Bs = As + T::A_ELEMS;
#pragma unroll
    for (int j = 0; j < A_LD; ++j) {
      const int kr = 4 * (k4b + KSTEP4 * j);
      As[(kr + 0) * T::LDA + ml] = ra[j].x;
      As[(kr + 1) * T::LDA + ml] = ra[j].y;
      As[(kr + 2) * T::LDA + ml] = ra[j].z;
      As[(kr + 3) * T::LDA + ml] = ra[j].w;
    }
#pragma unroll
    for (int j = 0; j < B_LD; ++j)
      *reinterpret_cast<float4*>(Bs + (bkr + KRSTEP * j) * T::LDB + 4 * bn4) = rb[j];
  };

  f32x16 acc[T::MI][T::NI];
#pragma unroll
  for (int i = 0; i < T::MI; ++i)
#pragma unroll
    for (int j = 0; j < T::NI; ++j)
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int wm0 = (wave / T::WAVES_N) * WM, wn0 = (wave % T::WAVES_N) * WN;
  const int nk = (Ktot + BK - 1) / BK;
  if (nk > 0) {
    load_a(0);
    load_b(0);
    store(0);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      adv_a();
      load_a((kt + 1) * BK);
      load_b((kt + 1) * BK);
    }
    const float* As = smem + cur * (T::A_ELEMS + T::B_ELEMS);
    mma_stage<BM, BN, WM, WN>(As, As + T::A_ELEMS, acc, wm0, wn0, lane);
    if (kt + 1 < nk) store(cur ^ 1);
    __syncthreads();
  }

  const int hw = Hc * Wc;
#pragma unroll
  for (int i = 0; i < T::MI; ++i)
#pragma unroll
    for (int j = 0; j < T::NI; ++j) {
      const int n = n0 + wn0 + 32 * j + (lane & 31);
      if (n >= Cx) continue;
      const float bv = bias ? bias[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int mm = m0 + wm0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (mm >= M) continue;
        const int nimg = mm / hw, rem = mm - nimg * hw, hh = rem / Wc, ww = rem - hh * Wc;
        const long o = (((long)nimg * Ho + (ca + st * hh)) * Wo + (cb + st * ww)) * Cx + n;
        out[o] = apply_act(acc[i][j][r] + bv, act, slope);
      }
    }
}

// ------------------------------------------------------------------------------------------ wgrad
// slab[z][m][n] = sum_{pixels p in split z} A[p][m] * dy[p][n],  A[p][m=(r,s,ci)] = x gathered;
// row m == Mw (if with_bias) is the all-ones row, giving the bias gradient sum_p dy[p][n].
template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(NT, 2) void conv_wgrad_k(
    const float* __restrict__ x, const float* __restrict__ dy, float* __restrict__ slab, int H,
    int W, int Cx, int Ho, int Wo, int Cyp, int S, int st, int pad, int reflect, int Mw, int Mtot,
    int P, int chunk) {
  using T = Tile<BM, BN, WM, WN>;
  constexpr int BM4 = BM / 4;
  constexpr int AKSTEP = NT / BM4;
  constexpr int A_LD = BK / AKSTEP;
  constexpr int BN4 = BN / 4;
  constexpr int KRSTEP = NT / BN4;
  constexpr int B_LD = BK / KRSTEP;
  static_assert(A_LD >= 1 && B_LD >= 1, "tile shape");
  __shared__ __attribute__((aligned(16))) float smem[2 * (T::A_ELEMS + T::B_ELEMS)];

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int pbeg = blockIdx.z * chunk;
  const int pend = min(P, pbeg + chunk);

  // A: this thread's 4 consecutive m (fixed tap), AKSTEP-strided pixel rows
  const int am4 = t % BM4, akb = t / BM4;
  const int am = m0 + 4 * am4;
  const int amode = am < Mw ? 0 : (am == Mw ? 1 : 2);  // 0 gather, 1 ones row, 2 zero
  int ar = 0, as_ = 0, aci = 0;
  if (amode == 0) {
    aci = am % Cx;
    const int rs = am / Cx;
    ar = rs / S;
    as_ = rs - ar * S;
  }
  // pixel decomposition for each of this thread's A rows (incremented by BK per stage)
  int pn[A_LD], pho[A_LD], pwo[A_LD];
#pragma unroll
  for (int j = 0; j < A_LD; ++j) {
    const int p = pbeg + akb + AKSTEP * j;
    const int hw = Ho * Wo;
    pn[j] = p / hw;
    const int rem = p - pn[j] * hw;
    pho[j] = rem / Wo;
    pwo[j] = rem - pho[j] * Wo;
  }
  const int bn4 = t % BN4, bkr = t / BN4;
  const int bcol = n0 + 4 * bn4;
  const bool bcval = bcol < Cyp;

  float4 ra[A_LD], rb[B_LD];
  auto load_a = [&](int p0) {
#pragma unroll
    for (int j = 0; j < A_LD; ++j) {
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      const int p = p0 + akb + AKSTEP * j;
      if (p < pend) {
        if (amode == 0) {
          int hi = pho[j] * st - pad + ar, wi = pwo[j] * st - pad + as_;
          bool ok = true;
          if (reflect) {
            hi = reflect_idx(hi, H);
            wi = reflect_idx(wi, W);
          } else {
            ok = (unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W;
          }
          if (ok)
            v = *reinterpret_cast<const float4*>(x + (((long)pn[j] * H + hi) * W + wi) * Cx + aci);
        } else if (amode == 1) {
          v.x = 1.f;
        }
      }
      ra[j] = v;
    }
  };
  auto adv_a = [&]() {
#pragma unroll
    for (int j = 0; j < A_LD; ++j) {
      pwo[j] += BK;
      while (pwo[j] >= Wo) {
        pwo[j] -= Wo;
        if (++pho[j] == Ho) { pho[j] = 0; ++pn[j]; }
      }
    }
  };
  auto load_b = [&](int p0) {
#pragma unroll
    for (int j = 0; j < B_LD; ++j) {
      const int p = p0 + bkr + KRSTEP * j;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (bcval && p < pend) v = *reinterpret_cast<const float4*>(dy + (long)p * Cyp + bcol);
      rb[j] = v;
    }
  };
  auto store = [&](int buf) {
    float* As = smem + buf * (T::A_ELEMS + T::B_ELEMS);
    float* Bs = As + T::A_ELEMS;
#pragma unroll
    for (int j = 0; j < A_LD; ++j)
      *reinterpret_cast<float4*>(As + (akb + AKSTEP * j) * T::LDA + 4 * am4) = ra[j];
#pragma unroll
    for (int j = 0; j < B_LD; ++j)
      *reinterpret_cast<float4*>(Bs + (bkr + KRSTEP * j) * T::LDB + 4 * bn4) = rb[j];
  };

  f32x16 acc[T::MI][T::NI];
#pragma unroll
  for (int i = 0; i < T::MI; ++i)
#pragma unroll
    for (int j = 0; j < T::NI; ++j)
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int wm0 = (wave / T::WAVES_N) * WM, wn0 = (wave % T::WAVES_N) * WN;
  const int nk = pend > pbeg ? (pend - pbeg + BK - 1) / BK : 0;
  if (nk > 0) {
    load_a(pbeg);
    load_b(pbeg);
    store(0);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      adv_a();
      load_a(pbeg + (kt + 1) * BK);
      load_b(pbeg + (kt + 1) * BK);
    }
    const float* As = smem + cur * (T::A_ELEMS + T::B_ELEMS);
    mma_stage<BM, BN, WM, WN>(As, As + T::A_ELEMS, acc, wm0, wn0, lane);
    if (kt + 1 < nk) store(cur ^ 1);
    __syncthreads();
  }

  float* sl = slab + (long)blockIdx.z * Mtot * Cyp;
#pragma unroll
  for (int i = 0; i < T::MI; ++i)
#pragma unroll
    for (int j = 0; j < T::NI; ++j) {
      const int n = n0 + wn0 + 32 * j + (lane & 31);
      if (n >= Cyp) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int mm = m0 + wm0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (mm < Mtot) sl[(long)mm * Cyp + n] = acc[i][j][r];
      }
    }
}

// dw[co*so + ci*si + rs] (+)= sum_z slab[z][rs*Cx + ci][co];  db[co] (+)= sum_z slab[z][Mw][co].
__global__ void wgrad_reduce_k(const float* __restrict__ slab, float* __restrict__ dw,
                               float* __restrict__ db, int nsplit, int Mtot, int Mw, int Cx, int Cyp,
                               int RS, int Co, int Ci, long so, long si, int accumulate) {
  const long total = (long)Co * Ci * RS;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx < total) {
    // idx enumerates (co, ci, rs) with rs fastest -> contiguous dw writes for so/si of PyTorch layout
    const int rs = idx % RS;
    const long q = idx / RS;
    const int ci = q % Ci;
    const int co = q / Ci;
    const long row = (long)rs * Cx + ci;
    float s = 0.f;
    for (int z = 0; z < nsplit; ++z) s += slab[((long)z * Mtot + row) * Cyp + co];
    float* d = dw + co * so + ci * si + rs;
    *d = accumulate ? *d + s : s;
  }
  if (db && idx < Co) {
    float s = 0.f;
    for (int z = 0; z < nsplit; ++z) s += slab[((long)z * Mtot + Mw) * Cyp + idx];
    db[idx] = accumulate ? db[idx] + s : s;
  }
}

// ------------------------------------------------------------------------------ reflect-pad fold
__global__ void reflect_fold_k(const float* __restrict__ dxp, const float* __restrict__ addend,
                               float* __restrict__ dx, int N, int H, int W, int C4, int p) {
  const long total = (long)N * H * W * C4;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int c4 = idx % C4;
  long q = idx / C4;
  const int w = q % W;
  q /= W;
  const int h = q % H;
  const int n = q / H;
  const int Hp = H + 2 * p, Wp = W + 2 * p;
  int hs[3], ws[3], nh = 0, nw = 0;
  hs[nh++] = h + p;
  if (h >= 1 && h <= p) hs[nh++] = p - h;
  if (h >= H - 1 - p && h <= H - 2) hs[nh++] = 2 * H - 2 - h + p;
  ws[nw++] = w + p;
  if (w >= 1 && w <= p) ws[nw++] = p - w;
  if (w >= W - 1 - p && w <= W - 2) ws[nw++] = 2 * W - 2 - w + p;
  const float4* src = reinterpret_cast<const float4*>(dxp);
  float4 acc = addend ? reinterpret_cast<const float4*>(addend)[idx] : make_float4(0.f, 0.f, 0.f, 0.f);
  for (int a = 0; a < nh; ++a)
    for (int b = 0; b < nw; ++b) {
      const float4 v = src[(((long)n * Hp + hs[a]) * Wp + ws[b]) * C4 + c4];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  reinterpret_cast<float4*>(dx)[idx] = acc;
}

// ---------------------------------------------------------------------------------- dispatch
template <int BM, int BN, int WM, int WN>
static int launch_fprop(const float* x, const float* wp, const float* bias, float* y, int N, int H,
                        int W, int C, int Ho, int Wo, int Cop, int R, int S, int st, int pad,
                        int reflect, int act, float slope, hipStream_t s) {
  const int M = N * Ho * Wo, K = R * S * C;
  dim3 grid(ceil_div(M, BM), ceil_div(Cop, BN));
  hipLaunchKernelGGL((conv_fprop_k<BM, BN, WM, WN>), grid, dim3(NT), 0, s, x, wp, bias, y, H, W, C,
                     Ho, Wo, Cop, S, st, pad, reflect, act, slope, M, K);
  return check_launch("conv2d_fwd");
}

template <int BM, int BN, int WM, int WN>
static int launch_tconv(const float* in, const float* wp, const float* bias, float* out, int N,
                        int Hi, int Wi, int Cy, int Ho, int Wo, int Cx, int R, int S, int st,
                        int pad, int act, float slope, hipStream_t s) {
  const int Hc = (Ho + st - 1) / st, Wc = (Wo + st - 1) / st;
  const int Mmax = N * Hc * Wc;
  dim3 grid(ceil_div(Mmax, BM), ceil_div(Cx, BN), st * st);
  hipLaunchKernelGGL((conv_tconv_k<BM, BN, WM, WN>), grid, dim3(NT), 0, s, in, wp, bias, out, Hi,
                     Wi, Cy, Ho, Wo, Cx, R, S, st, pad, act, slope, N);
  return check_launch("conv2d_tfwd");
}

// Tile choice: 128x128 when the channel dim allows and the grid has >= ~2 blocks/CU worth of
// work, otherwise narrower N tiles (skinny output channels: 3 or 1 logical, 4 padded).
enum TileKind { T128x128, T128x64, T256x32, T64x64 };

static TileKind pick_tile(long M, int Nc) {
  if (Nc <= 32) return T256x32;
  if (Nc <= 64) return M >= 128L * 256 ? T128x64 : T64x64;
  if (M / 128 * ((Nc + 127) / 128) >= 256) return T128x128;
  return T64x64;
}

struct WgradPlan {
  int Mw, Mtot, nsplit, chunk, gx, gy;
};

static WgradPlan plan_wgrad(int N, int Ho, int Wo, int Cx, int Cyp, int R, int S) {
  WgradPlan p;
  p.Mw = R * S * Cx;
  p.Mtot = p.Mw + 4;  // + ones row group for the bias gradient
  const int P = N * Ho * Wo;
  p.gx = ceil_div(p.Mtot, 128);
  p.gy = ceil_div(Cyp, Cyp <= 32 ? 32 : 64);
  const int tiles = p.gx * p.gy;
  int ns = ceil_div(1024, tiles);                     // aim for ~4 blocks per CU
  const int max_ns = ceil_div(P, 4 * BK);             // at least 4 K-steps per split
  if (ns > max_ns) ns = max_ns;
  if (ns < 1) ns = 1;
  p.chunk = ceil_div(ceil_div(P, ns), BK) * BK;
  p.nsplit = ceil_div(P, p.chunk);
  return p;
}

}  // namespace vst

using namespace vst;

extern "C" int vst_conv2d_fwd(const float* x, const float* wp, const float* bias, float* y, int N,
                              int H, int W, int Cx, int Cop, int R, int S, int stride, int pad,
                              int pad_mode, int act, float slope, void* stream) {
  VST_REQUIRE(x && wp && y, "conv2d_fwd: null pointer");
  VST_REQUIRE(N > 0 && H > 0 && W > 0 && R > 0 && S > 0 && stride > 0 && pad >= 0,
              "conv2d_fwd: bad shape");
  VST_REQUIRE(Cx % 4 == 0 && Cop % 4 == 0, "conv2d_fwd: channel strides must be multiples of 4");
  VST_REQUIRE(pad_mode == VST_PAD_ZERO || (pad < H && pad < W), "conv2d_fwd: reflect pad >= size");
  const int Ho = (H + 2 * pad - R) / stride + 1, Wo = (W + 2 * pad - S) / stride + 1;
  VST_REQUIRE(Ho > 0 && Wo > 0, "conv2d_fwd: empty output");
  const int refl = pad_mode == VST_PAD_REFLECT;
  hipStream_t s = (hipStream_t)stream;
  switch (pick_tile((long)N * Ho * Wo, Cop)) {
    case T128x128:
      return launch_fprop<128, 128, 64, 64>(x, wp, bias, y, N, H, W, Cx, Ho, Wo, Cop, R, S, stride, pad, refl, act, slope, s);
    case T128x64:
      return launch_fprop<128, 64, 64, 32>(x, wp, bias, y, N, H, W, Cx, Ho, Wo, Cop, R, S, stride, pad, refl, act, slope, s);
    case T256x32:
      return launch_fprop<256, 32, 64, 32>(x, wp, bias, y, N, H, W, Cx, Ho, Wo, Cop, R, S, stride, pad, refl, act, slope, s);
    default:
      return launch_fprop<64, 64, 32, 32>(x, wp, bias, y, N, H, W, Cx, Ho, Wo, Cop, R, S, stride, pad, refl, act, slope, s);
  }
}

extern "C" int vst_conv2d_tfwd(const float* in, const float* wp, const float* bias, float* out,
                               int N, int Hi, int Wi, int Cy, int Ho, int Wo, int Cx, int R, int S,
                               int stride, int pad, int act, float slope, void* stream) {
  VST_REQUIRE(in && wp && out, "conv2d_tfwd: null pointer");
  VST_REQUIRE(N > 0 && Hi > 0 && Wi > 0 && Ho > 0 && Wo > 0 && R > 0 && S > 0 && stride > 0 && pad >= 0,
              "conv2d_tfwd: bad shape");
  VST_REQUIRE(Cy % 4 == 0 && Cx % 4 == 0, "conv2d_tfwd: channel strides must be multiples of 4");
  hipStream_t s = (hipStream_t)stream;
  const long Mc = (long)N * ((Ho + stride - 1) / stride) * ((Wo + stride - 1) / stride);
  switch (pick_tile(Mc * stride * stride, Cx)) {
    case T128x128:
      return launch_tconv<128, 128, 64, 64>(in, wp, bias, out, N, Hi, Wi, Cy, Ho, Wo, Cx, R, S, stride, pad, act, slope, s);
    case T128x64:
      return launch_tconv<128, 64, 64, 32>(in, wp, bias, out, N, Hi, Wi, Cy, Ho, Wo, Cx, R, S, stride, pad, act, slope, s);
    case T256x32:
      return launch_tconv<256, 32, 64, 32>(in, wp, bias, out, N, Hi, Wi, Cy, Ho, Wo, Cx, R, S, stride, pad, act, slope, s);
    default:
      return launch_tconv<64, 64, 32, 32>(in, wp, bias, out, N, Hi, Wi, Cy, Ho, Wo, Cx, R, S, stride, pad, act, slope, s);
  }
}

extern "C" size_t vst_conv2d_wgrad_ws_bytes(int N, int H, int W, int Cx, int Ho, int Wo, int Cyp,
                                            int R, int S) {
  (void)H;
  (void)W;
  const WgradPlan p = plan_wgrad(N, Ho, Wo, Cx, Cyp, R, S);
  return (size_t)p.nsplit * p.Mtot * Cyp * sizeof(float);
}

extern "C" int vst_conv2d_wgrad(const float* x, const float* dy, float* dw, float* db, float* ws,
                                size_t ws_bytes, int N, int H, int W, int Cx, int Ho, int Wo,
                                int Cyp, int R, int S, int stride, int pad, int pad_mode, int Co,
                                int Ci, long so, long si, int accumulate, void* stream) {
  VST_REQUIRE(x && dy && dw && ws, "conv2d_wgrad: null pointer");
  VST_REQUIRE(Cx % 4 == 0 && Cyp % 4 == 0, "conv2d_wgrad: channel strides must be multiples of 4");
  VST_REQUIRE(Co <= Cyp && Ci <= Cx, "conv2d_wgrad: logical channels exceed strides");
  VST_REQUIRE(pad_mode == VST_PAD_ZERO || (pad < H && pad < W), "conv2d_wgrad: reflect pad >= size");
  const WgradPlan p = plan_wgrad(N, Ho, Wo, Cx, Cyp, R, S);
  VST_REQUIRE(ws_bytes >= (size_t)p.nsplit * p.Mtot * Cyp * sizeof(float),
              "conv2d_wgrad: workspace too small (%zu bytes)", ws_bytes);
  hipStream_t s = (hipStream_t)stream;
  const int P = N * Ho * Wo;
  const int refl = pad_mode == VST_PAD_REFLECT;
  if (Cyp <= 32) {
    dim3 grid(ceil_div(p.Mtot, 128), ceil_div(Cyp, 32), p.nsplit);
    hipLaunchKernelGGL((conv_wgrad_k<128, 32, 32, 32>), grid, dim3(NT), 0, s, x, dy, ws, H, W, Cx,
                       Ho, Wo, Cyp, S, stride, pad, refl, p.Mw, p.Mtot, P, p.chunk);
  } else {
    dim3 grid(ceil_div(p.Mtot, 128), ceil_div(Cyp, 64), p.nsplit);
    hipLaunchKernelGGL((conv_wgrad_k<128, 64, 64, 32>), grid, dim3(NT), 0, s, x, dy, ws, H, W, Cx,
                       Ho, Wo, Cyp, S, stride, pad, refl, p.Mw, p.Mtot, P, p.chunk);
  }
  int rc = check_launch("conv2d_wgrad");
  if (rc) return rc;
  const long total = (long)Co * Ci * R * S;
  const long threads = total > Co ? total : Co;
  hipLaunchKernelGGL(wgrad_reduce_k, dim3(ceil_div(threads, 256)), dim3(256), 0, s, ws, dw, db,
                     p.nsplit, p.Mtot, p.Mw, Cx, Cyp, R * S, Co, Ci, so, si, accumulate);
  return check_launch("conv2d_wgrad_reduce");
}

extern "C" int vst_reflect_fold(const float* dxp, const float* addend, float* dx, int N, int H,
                                int W, int C, int p, void* stream) {
  VST_REQUIRE(dxp && dx && C % 4 == 0 && p >= 0 && p < H && p < W, "reflect_fold: bad args");
  const long total = (long)N * H * W * (C / 4);
  hipLaunchKernelGGL(reflect_fold_k, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream,
                     dxp, addend, dx, N, H, W, C / 4, p);
  return check_launch("reflect_fold");
}
