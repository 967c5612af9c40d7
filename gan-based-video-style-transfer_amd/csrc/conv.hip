// Implicit-GEMM convolution kernels on gfx950 fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// Replaces the cuDNN conv fprop / dgrad / wgrad that nn.Conv2d, nn.ConvTranspose2d and
// nn.ReflectionPad2d dispatch in the reference ResnetGenerator / NLayerDiscriminator
// (methods/GAN-based/CycleGAN/models/networks.py:340-367, 404-426, 556-578).
//
// Every kernel computes C[BM x BN] = sum_k A[m][k] * B[k][n] per workgroup with
//   * NW = 4 or 8 waves (256/512 threads), each owning a WM x WN sub-tile of 32x32 MFMA blocks;
//     a 128x128 tile with 8 waves gives two waves per SIMD inside one workgroup, which is what the
//     CycleGAN shapes need (B=4: a 16384x256 output is exactly one 128x128 tile per CU);
//   * BK = 32 deep K-steps double-buffered in LDS, one barrier per K-step.  Both LDS operand images
//     are k-major ([k][row], +4 float pad) so every MFMA operand fetch is a conflict-free ds_read
//     over 32 consecutive rows; fragments of step kk+2 are fetched while step kk's MFMAs issue;
//   * the global loads of the NEXT K-step are interleaved into the MFMA sequence of the current
//     one (2 per MFMA group, so their address arithmetic runs in the shadow of the 64-cycle fp32
//     MFMAs) and written to the other LDS buffer after the last MFMA group;
// Operand gathers fold padding (zero or reflect), stride and transposition into address
// generation: no im2col, no padded copies, no zero-insertion.  fp32 MFMA is an exact fp32 fma
// chain, so results differ from the CPU reference only by summation order.
//
//   conv_fprop_k : y = conv(x, w)            m = output pixel, n = out channel, k = (r, s, ci)
//   conv_tconv_k : transposed conv / dgrad    gathered per output-parity class (blockIdx.z) so a
//                  stride-2 layer walks only the taps that hit each class; for stride 1 with
//                  reflect padding the gather adds the mirrored contributions of ReflectionPad2d's
//                  backward directly (no padded gradient buffer, no fold pass); optional residual
//                  addend fused in the epilogue
//   conv_wgrad_k : dw = x_gather^T * dy       m = (r, s, ci), n = out channel, k = pixel;
//                  split-K over blockIdx.z into an fp32 slab, summed in a fixed split order
//                  (deterministic) and written to [Co][Ci][R][S] by wgrad_reduce_store_k.
#include "common.h"

namespace vst {

constexpr int BK = 32;

template <int BM, int BN, int WM, int WN>
struct Tile {
  static constexpr int NW = (BM / WM) * (BN / WN);
  static constexpr int NT = 64 * NW;
  static constexpr int LDA = BM + 4;
  static constexpr int LDB = BN + 4;
  static constexpr int WAVES_N = BN / WN;
  static constexpr int MI = WM / 32;
  static constexpr int NI = WN / 32;
  static constexpr int A_ELEMS = BK * LDA;
  static constexpr int B_ELEMS = BK * LDB;
  static constexpr int STAGE = A_ELEMS + B_ELEMS;
  static_assert(NW == 4 || NW == 8, "4 or 8 waves per block");
  static_assert(WM % 32 == 0 && WN % 32 == 0, "32x32 MFMA blocks");
};

// MFMA over one BK-deep LDS stage (8 groups of 2 k-pairs).  hook(g) runs at the start of group g
// (global loads of the next stage); fragments for the next group are fetched during this one.
template <int BM, int BN, int WM, int WN, class Hook>
__device__ __forceinline__ void mma_stage(const float* __restrict__ As, const float* __restrict__ Bs,
                                          f32x16 (&acc)[WM / 32][WN / 32], int wm0, int wn0, int lane,
                                          Hook hook) {
  using T = Tile<BM, BN, WM, WN>;
  const int kh = lane >> 5, li = lane & 31;
  const float* pa = As + kh * T::LDA + wm0 + li;
  const float* pb = Bs + kh * T::LDB + wn0 + li;
  float a0[T::MI], b0[T::NI], a1[T::MI], b1[T::NI];
#pragma unroll
  for (int i = 0; i < T::MI; ++i) a0[i] = pa[32 * i];
#pragma unroll
  for (int j = 0; j < T::NI; ++j) b0[j] = pb[32 * j];
#pragma unroll
  for (int g = 0; g < BK / 4; ++g) {
    const int kk = 2 * g;
    hook(g);
#pragma unroll
    for (int i = 0; i < T::MI; ++i) a1[i] = pa[(2 * kk + 2) * T::LDA + 32 * i];
#pragma unroll
    for (int j = 0; j < T::NI; ++j) b1[j] = pb[(2 * kk + 2) * T::LDB + 32 * j];
#pragma unroll
    for (int i = 0; i < T::MI; ++i)
#pragma unroll
      for (int j = 0; j < T::NI; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[i], b0[j], acc[i][j], 0, 0, 0);
    if (g + 1 < BK / 4) {
#pragma unroll
      for (int i = 0; i < T::MI; ++i) a0[i] = pa[(2 * kk + 4) * T::LDA + 32 * i];
#pragma unroll
      for (int j = 0; j < T::NI; ++j) b0[j] = pb[(2 * kk + 4) * T::LDB + 32 * j];
    }
#pragma unroll
    for (int i = 0; i < T::MI; ++i)
#pragma unroll
      for (int j = 0; j < T::NI; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[i], b1[j], acc[i][j], 0, 0, 0);
  }
}

template <int MI, int NI>
__device__ __forceinline__ void zero_acc(f32x16 (&acc)[MI][NI]) {
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
}

// Double-buffered K loop shared by all kernels.  load_one(i, k0) issues global load number i
// (0 <= i < NLOAD, compile-time after unrolling) of the stage starting at k0 into registers;
// adv() steps the incremental index state by BK; store(buf) writes the staged registers to LDS.
template <int BM, int BN, int WM, int WN, int NLOAD, class LoadOne, class Adv, class Store>
__device__ __forceinline__ void main_loop(float* smem, int nk, int kbase,
                                          f32x16 (&acc)[WM / 32][WN / 32], LoadOne load_one, Adv adv,
                                          Store store) {
  using T = Tile<BM, BN, WM, WN>;
  static_assert(NLOAD <= 2 * (BK / 4), "at most two loads per MFMA group");
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm0 = (wave / T::WAVES_N) * WM, wn0 = (wave % T::WAVES_N) * WN;
  if (nk > 0) {
#pragma unroll
    for (int i = 0; i < NLOAD; ++i) load_one(i, kbase);
    store(smem);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    float* cur = smem + (kt & 1) * T::STAGE;
    const bool next = kt + 1 < nk;
    if (next) adv();
    const int k0n = kbase + (kt + 1) * BK;
    mma_stage<BM, BN, WM, WN>(cur, cur + T::A_ELEMS, acc, wm0, wn0, lane, [&](int g) {
      if (next) {
        if (2 * g < NLOAD) load_one(2 * g, k0n);
        if (2 * g + 1 < NLOAD) load_one(2 * g + 1, k0n);
      }
    });
    if (next) store(smem + ((kt + 1) & 1) * T::STAGE);
    __syncthreads();
  }
}

// XCD-aware remap of the M-tile index: consecutive M tiles (neighbouring pixel rows, which share
// halo rows) land on the same XCD / L2 (blocks b and b+8 share an XCD under round-robin dispatch).
__device__ __forceinline__ int remap_mtile(int bx, int nx) {
  if ((nx & 7) != 0) return bx;
  return (bx & 7) * (nx >> 3) + (bx >> 3);
}

// transposing store of a thread's float4 A chunk (4 consecutive k of one row m) into [k][m]
template <int LDA>
__device__ __forceinline__ void store_a_t(float* As, int kr, int ml, const float4& v) {
  As[(kr + 0) * LDA + ml] = v.x;
  As[(kr + 1) * LDA + ml] = v.y;
  As[(kr + 2) * LDA + ml] = v.z;
  As[(kr + 3) * LDA + ml] = v.w;
}

__device__ __forceinline__ void add4(float4& a, const float4& b) {
  a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
}

// ------------------------------------------------------------------------------------------ fprop
template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__((Tile<BM, BN, WM, WN>::NT), 2) void conv_fprop_k(
    const float* __restrict__ x, const float* __restrict__ wp, const float* __restrict__ bias,
    float* __restrict__ y, int H, int W, int C, int Ho, int Wo, int Cop, int S, int st, int pad,
    int reflect, int act, float slope, int M, int Ktot) {
  using T = Tile<BM, BN, WM, WN>;
  constexpr int NT = T::NT;
  constexpr int KSTEP4 = NT / BM;         // k4 stride between a thread's A loads
  constexpr int A_LD = BK / 4 / KSTEP4;   // float4 A loads per thread per stage
  constexpr int BN4 = BN / 4;
  constexpr int KRSTEP = NT / BN4;
  constexpr int B_LD = BK / KRSTEP;
  static_assert(NT % BM == 0 && A_LD >= 1 && B_LD >= 1, "tile shape");
  __shared__ __attribute__((aligned(16))) float smem[2 * T::STAGE];

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int mt = remap_mtile(blockIdx.x, gridDim.x);
  const int m0 = mt * BM, n0 = blockIdx.y * BN;

  const int ml = t % BM, k4b = t / BM;
  const int m = m0 + ml;
  const bool mval = m < M;
  int hb = 0, wb = 0;
  const float* xb = x;
  if (mval) {
    const int hw = Ho * Wo;
    const int n = m / hw, rem = m - n * hw, ho = rem / Wo, wo = rem - ho * Wo;
    hb = ho * st - pad;
    wb = wo * st - pad;
    xb = x + (long)n * H * W * C;
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
  const int bn4 = t % BN4, bkr = t / BN4;
  const int bcol = n0 + 4 * bn4;
  const bool bcval = bcol < Cop;

  float4 ra[A_LD], rb[B_LD];
  auto load_one = [&](int i, int k0) {
    if (i < A_LD) {
      const int j = i;
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
        if (ok) v = *reinterpret_cast<const float4*>(xb + ((long)hi * W + wi) * C + ac[j]);
      }
      ra[j] = v;
    } else {
      const int j = i - A_LD;
      const int kr = k0 + bkr + KRSTEP * j;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (bcval && kr < Ktot) v = *reinterpret_cast<const float4*>(wp + (long)kr * Cop + bcol);
      rb[j] = v;
    }
  };
  auto adv = [&]() {
#pragma unroll
    for (int j = 0; j < A_LD; ++j) {
      ac[j] += BK;
      while (ac[j] >= C) {
        ac[j] -= C;
        if (++as_[j] == S) { as_[j] = 0; ++ar[j]; }
      }
    }
  };
  auto store = [&](float* As) {
    float* Bs = As + T::A_ELEMS;
#pragma unroll
    for (int j = 0; j < A_LD; ++j) store_a_t<T::LDA>(As, 4 * (k4b + KSTEP4 * j), ml, ra[j]);
#pragma unroll
    for (int j = 0; j < B_LD; ++j)
      *reinterpret_cast<float4*>(Bs + (bkr + KRSTEP * j) * T::LDB + 4 * bn4) = rb[j];
  };

  f32x16 acc[T::MI][T::NI];
  zero_acc(acc);
  main_loop<BM, BN, WM, WN, A_LD + B_LD>(smem, (Ktot + BK - 1) / BK, 0, acc, load_one, adv, store);

  const int wm0 = (wave / T::WAVES_N) * WM, wn0 = (wave % T::WAVES_N) * WN;
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
// out[n][h][w][cx] = sum in[n][ho][wo][cy] * wp[r][s][cy][cx] over h = ho*st - pad + r (zero pad)
// or, with reflect (st == 1), over reflect(ho + r - pad) == h.
// blockIdx.z = parity class (a, b): h = a + st*hh; only taps r = r0 + st*i with
// r0 = (a + pad) mod st contribute, at ho = (h + pad - r) / st (exact).
constexpr int NOPOS = -(1 << 20);

template <int BM, int BN, int WM, int WN, int ST>
__global__ __launch_bounds__((Tile<BM, BN, WM, WN>::NT), 2) void conv_tconv_k(
    const float* __restrict__ in, const float* __restrict__ wp, const float* __restrict__ bias,
    const float* __restrict__ addend, float* __restrict__ out, int Hi, int Wi, int Cy, int Ho,
    int Wo, int Cx, int R, int S, int st_rt, int pad, int reflect, int act, float slope, int Nimg) {
  using T = Tile<BM, BN, WM, WN>;
  const int st = ST > 0 ? ST : st_rt;  // compile-time stride for the CycleGAN layers (1, 2)
  constexpr int NT = T::NT;
  constexpr int KSTEP4 = NT / BM;
  constexpr int A_LD = BK / 4 / KSTEP4;
  constexpr int BN4 = BN / 4;
  constexpr int KRSTEP = NT / BN4;
  constexpr int B_LD = BK / KRSTEP;
  __shared__ __attribute__((aligned(16))) float smem[2 * T::STAGE];

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
  // (h + pad) for the direct term and, for reflect, the one mirrored image row/column
  int hp = 0, wq = 0, hm = NOPOS, wmr = NOPOS;
  const float* ib = in;
  if (mval) {
    const int hw = Hc * Wc;
    const int n = m / hw, rem = m - n * hw, hh = rem / Wc, ww = rem - hh * Wc;
    const int h = ca + st * hh, w = cb + st * ww;
    hp = h + pad;
    wq = w + pad;
    if (reflect) {
      if (h >= 1 && h <= pad) hm = pad - h;
      else if (h >= Ho - 1 - pad && h <= Ho - 2) hm = 2 * Ho - 2 - h + pad;
      if (w >= 1 && w <= pad) wmr = pad - w;
      else if (w >= Wo - 1 - pad && w <= Wo - 2) wmr = 2 * Wo - 2 - w + pad;
    }
    ib = in + (long)n * Hi * Wi * Cy;
  }
  int ac[A_LD], ais[A_LD], air[A_LD];
#pragma unroll
  for (int j = 0; j < A_LD; ++j) {
    const int k = 4 * (k4b + KSTEP4 * j);
    ac[j] = k % Cy;
    const int tp = k / Cy;
    air[j] = ns > 0 ? tp / ns : 0;
    ais[j] = tp - air[j] * ns;
  }
  const int bn4 = t % BN4, bkr = t / BN4;
  const int bcol = n0 + 4 * bn4;
  const bool bcval = bcol < Cx;
  int bc[B_LD], bis[B_LD], bir[B_LD];
#pragma unroll
  for (int j = 0; j < B_LD; ++j) {
    const int k = bkr + KRSTEP * j;
    bc[j] = k % Cy;
    const int tp = k / Cy;
    bir[j] = ns > 0 ? tp / ns : 0;
    bis[j] = tp - bir[j] * ns;
  }

  float4 ra[A_LD], rb[B_LD];
  auto gather1 = [&](int hpos, int wpos, int r, int s, int c, float4& v) {
    const int dh = hpos - r, dw = wpos - s;
    if (dh >= 0 && dw >= 0) {
      const int ho = dh / st, wo = dw / st;
      if (ho < Hi && wo < Wi)
        add4(v, *reinterpret_cast<const float4*>(ib + ((long)ho * Wi + wo) * Cy + c));
    }
  };
  auto load_one = [&](int i, int k0) {
    if (i < A_LD) {
      const int j = i;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      const int kk = k0 + 4 * (k4b + KSTEP4 * j);
      if (mval && kk < Ktot) {
        const int r = r0 + st * air[j], s = s0 + st * ais[j];
        gather1(hp, wq, r, s, ac[j], v);
        if (hm != NOPOS) gather1(hm, wq, r, s, ac[j], v);
        if (wmr != NOPOS) {
          gather1(hp, wmr, r, s, ac[j], v);
          if (hm != NOPOS) gather1(hm, wmr, r, s, ac[j], v);
        }
      }
      ra[j] = v;
    } else {
      const int j = i - A_LD;
      const int kk = k0 + bkr + KRSTEP * j;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (bcval && kk < Ktot) {
        const int row = ((r0 + st * bir[j]) * S + (s0 + st * bis[j])) * Cy + bc[j];
        v = *reinterpret_cast<const float4*>(wp + (long)row * Cx + bcol);
      }
      rb[j] = v;
    }
  };
  auto adv = [&]() {
#pragma unroll
    for (int j = 0; j < A_LD; ++j) {
      ac[j] += BK;
      while (ac[j] >= Cy) {
        ac[j] -= Cy;
        if (++ais[j] == ns) { ais[j] = 0; ++air[j]; }
      }
    }
#pragma unroll
    for (int j = 0; j < B_LD; ++j) {
      bc[j] += BK;
      while (bc[j] >= Cy) {
        bc[j] -= Cy;
        if (++bis[j] == ns) { bis[j] = 0; ++bir[j]; }
      }
    }
  };
  auto store = [&](float* As) {
    float* Bs = As + T::A_ELEMS;
#pragma unroll
    for (int j = 0; j < A_LD; ++j) store_a_t<T::LDA>(As, 4 * (k4b + KSTEP4 * j), ml, ra[j]);
#pragma unroll
    for (int j = 0; j < B_LD; ++j)
      *reinterpret_cast<float4*>(Bs + (bkr + KRSTEP * j) * T::LDB + 4 * bn4) = rb[j];
  };

  f32x16 acc[T::MI][T::NI];
  zero_acc(acc);
  main_loop<BM, BN, WM, WN, A_LD + B_LD>(smem, (Ktot + BK - 1) / BK, 0, acc, load_one, adv, store);

  const int wm0 = (wave / T::WAVES_N) * WM, wn0 = (wave % T::WAVES_N) * WN;
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
        float v = apply_act(acc[i][j][r] + bv, act, slope);
        if (addend) v += addend[o];
        out[o] = v;
      }
    }
}

// ------------------------------------------------------------------------------------------ wgrad
// slab[z][m][n] = sum_{pixels p in split z} A[p][m] * dy[p][n],  A[p][m=(r,s,ci)] = x gathered.
template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__((Tile<BM, BN, WM, WN>::NT), 2) void conv_wgrad_k(
    const float* __restrict__ x, const float* __restrict__ dy, float* __restrict__ slab, int H,
    int W, int Cx, int Ho, int Wo, int Cyp, int S, int st, int pad, int reflect, int Mw, int P,
    int chunk) {
  using T = Tile<BM, BN, WM, WN>;
  constexpr int NT = T::NT;
  constexpr int BM4 = BM / 4;
  constexpr int AKSTEP = NT / BM4;
  constexpr int A_LD = BK / AKSTEP;
  constexpr int BN4 = BN / 4;
  constexpr int KRSTEP = NT / BN4;
  constexpr int B_LD = BK / KRSTEP;
  static_assert(A_LD >= 1 && B_LD >= 1, "tile shape");
  __shared__ __attribute__((aligned(16))) float smem[2 * T::STAGE];

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  // 1-D XCD-aware grid (as conv_rk.hip's wgrad): the tiles of one pixel chunk share an XCD's L2
  const int Mt = (Mw + BM - 1) / BM, Nt = (Cyp + BN - 1) / BN, Zt = (P + chunk - 1) / chunk;
  int zz, mx, ny;
  {
    const int tt = xcd_tile(blockIdx.x, Mt * Nt * Zt);
    zz = tt / (Mt * Nt);
    const int rem = tt - zz * Mt * Nt;
    ny = rem / Mt;
    mx = rem - ny * Mt;
  }
  const int m0 = mx * BM, n0 = ny * BN;
  const int pbeg = zz * chunk;
  const int pend = min(P, pbeg + chunk);

  const int am4 = t % BM4, akb = t / BM4;
  const int am = m0 + 4 * am4;
  const bool amval = am < Mw;
  int ar = 0, as_ = 0, aci = 0;
  if (amval) {
    aci = am % Cx;
    const int rs = am / Cx;
    ar = rs / S;
    as_ = rs - ar * S;
  }
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
  auto load_one = [&](int i, int p0) {
    if (i < A_LD) {
      const int j = i;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      const int p = p0 + akb + AKSTEP * j;
      if (amval && p < pend) {
        int hi = pho[j] * st - pad + ar, wi = pwo[j] * st - pad + as_;
        bool ok = true;
        if (reflect) {
          hi = reflect_idx(hi, H);
          wi = reflect_idx(wi, W);
        } else {
          ok = (unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W;
        }
        if (ok) v = *reinterpret_cast<const float4*>(x + (((long)pn[j] * H + hi) * W + wi) * Cx + aci);
      }
      ra[j] = v;
    } else {
      const int j = i - A_LD;
      const int p = p0 + bkr + KRSTEP * j;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (bcval && p < pend) v = *reinterpret_cast<const float4*>(dy + (long)p * Cyp + bcol);
      rb[j] = v;
    }
  };
  auto adv = [&]() {
#pragma unroll
    for (int j = 0; j < A_LD; ++j) {
      pwo[j] += BK;
      while (pwo[j] >= Wo) {
        pwo[j] -= Wo;
        if (++pho[j] == Ho) { pho[j] = 0; ++pn[j]; }
      }
    }
  };
  auto store = [&](float* As) {
    float* Bs = As + T::A_ELEMS;
#pragma unroll
    for (int j = 0; j < A_LD; ++j)
      *reinterpret_cast<float4*>(As + (akb + AKSTEP * j) * T::LDA + 4 * am4) = ra[j];
#pragma unroll
    for (int j = 0; j < B_LD; ++j)
      *reinterpret_cast<float4*>(Bs + (bkr + KRSTEP * j) * T::LDB + 4 * bn4) = rb[j];
  };

  f32x16 acc[T::MI][T::NI];
  zero_acc(acc);
  const int nk = pend > pbeg ? (pend - pbeg + BK - 1) / BK : 0;
  main_loop<BM, BN, WM, WN, A_LD + B_LD>(smem, nk, pbeg, acc, load_one, adv, store);

  const int wm0 = (wave / T::WAVES_N) * WM, wn0 = (wave % T::WAVES_N) * WN;
  float* sl = slab + (long)zz * Mw * Cyp;
#pragma unroll
  for (int i = 0; i < T::MI; ++i)
#pragma unroll
    for (int j = 0; j < T::NI; ++j) {
      const int n = n0 + wn0 + 32 * j + (lane & 31);
      if (n >= Cyp) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int mm = m0 + wm0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (mm < Mw) sl[(long)mm * Cyp + n] = acc[i][j][r];
      }
    }
}

// slab[0][m][n] = sum_z slab[z][m][n] (fixed order), float4 over n: coalesced and fully parallel.
// The split-K reduction and the store in one pass: a 64 (ci, rs) x 64 co tile per block, each thread
// summing 4 float4 column quads over the nsplit slabs (all slab loads of a quad issued back to back,
// z = 0, 1, 2, ...: a fixed order, so deterministic), then an LDS transpose and the [Co][Ci][R][S]
// store (+= across the step's passes).  One launch instead of a slab-sized sum pass + a store pass.
// Split-K slabs S[z][(rs, ci)][Cyp] summed in slab order and stored transposed into dw[co][ci][rs]
// (strides so / si).  A block owns 32 (rs, ci) rows x 64 channels: 2 rows per thread with 8 slabs'
// loads per round trip (16 float4 in flight per thread, ~1100 waves for a ResnetBlock weight), then a
// 32 x 64 LDS transpose for the [co]-major store.  grid (ceil(Ci*RS / 32), ceil(Cyp / 64)).
// NR: rows per thread (block = 16 NR rows x 64 columns)
template <int NR>
__global__ __launch_bounds__(256) void wgrad_reduce_store_k(const float* __restrict__ S, float* __restrict__ dw,
                                                            int Cx, int Cyp, int RS, int Co, int Ci, long so,
                                                            long si, int accumulate, int nsplit, long zs) {
  constexpr int RB = 16 * NR, UZ = 8;
  __shared__ float tile[RB][65];
  const int m0 = blockIdx.x * RB, c0 = blockIdx.y * 64;
  const int t = threadIdx.x, c4 = (t & 15) * 4, r0 = t >> 4;
  const int Md = Ci * RS;
  float4 acc[NR];
  const float* src[NR];
  bool ok[NR];
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int md = m0 + r0 + 16 * i;
    ok[i] = md < Md && c0 + c4 < Cyp;
    const int mm = ok[i] ? md : 0;
    const int ci = mm / RS, rs = mm - ci * RS;
    src[i] = S + (long)(rs * Cx + ci) * Cyp + (ok[i] ? c0 + c4 : 0);
    acc[i] = ok[i] ? *reinterpret_cast<const float4*>(src[i]) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  int z = 1;
  for (; z + UZ - 1 < nsplit; z += UZ) {
    float4 v[UZ][NR];
#pragma unroll
    for (int u = 0; u < UZ; ++u)
#pragma unroll
      for (int i = 0; i < NR; ++i)
        v[u][i] = *reinterpret_cast<const float4*>(src[i] + (ok[i] ? (long)(z + u) * zs : 0));
#pragma unroll
    for (int u = 0; u < UZ; ++u)
#pragma unroll
      for (int i = 0; i < NR; ++i) add4(acc[i], v[u][i]);
  }
  if (z < nsplit) {  // the last < UZ slabs: their loads issued together too (one at a time: a round trip each), then
                    // summed in slab order as above
    float4 v[UZ - 1][NR];
#pragma unroll
    for (int u = 0; u < UZ - 1; ++u)
#pragma unroll
      for (int i = 0; i < NR; ++i)
        v[u][i] = z + u < nsplit ? *reinterpret_cast<const float4*>(src[i] + (ok[i] ? (long)(z + u) * zs : 0))
                                 : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int u = 0; u < UZ - 1; ++u) {
      if (z + u >= nsplit) break;
#pragma unroll
      for (int i = 0; i < NR; ++i) add4(acc[i], v[u][i]);
    }
  }
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int r = r0 + 16 * i;
    tile[r][c4] = acc[i].x;
    tile[r][c4 + 1] = acc[i].y;
    tile[r][c4 + 2] = acc[i].z;
    tile[r][c4 + 3] = acc[i].w;
  }
  __syncthreads();
  const int tx = t % RB, ty = t / RB;
  for (int r = ty; r < 64; r += 256 / RB) {
    const int c = c0 + r, md = m0 + tx;
    if (c >= Co || md >= Md) continue;
    const int ci = md / RS, rs = md - ci * RS;
    float* d = dw + c * so + ci * si + rs;
    const float v = tile[tx][r];
    *d = accumulate ? *d + v : v;
  }
}

// First level of the split-K reduction for small outputs with many slabs (image-size layers: a
// handful of 64x64 output tiles over 100+ pixel chunks): slab group q = slabs [qG, qG+G) summed in
// order into out[q] (4 slabs' loads in flight per round trip), in parallel over (element, group).
__global__ __launch_bounds__(256) void slab_group_sum_k(const float* __restrict__ slab, float* __restrict__ out,
                                                        long n4, int nsplit, int G) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const int q = blockIdx.y, z0 = q * G, z1 = min(nsplit, z0 + G);
  const float4* s4 = reinterpret_cast<const float4*>(slab) + i;
  float4 a = s4[(long)z0 * n4];
  int z = z0 + 1;
  for (; z + 3 < z1; z += 4) {
    const float4 v0 = s4[(long)z * n4], v1 = s4[(long)(z + 1) * n4], v2 = s4[(long)(z + 2) * n4],
                 v3 = s4[(long)(z + 3) * n4];
    add4(a, v0);
    add4(a, v1);
    add4(a, v2);
    add4(a, v3);
  }
  for (; z < z1; ++z) add4(a, s4[(long)z * n4]);
  reinterpret_cast<float4*>(out)[(long)q * n4 + i] = a;
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
    for (int b = 0; b < nw; ++b) add4(acc, src[(((long)n * Hp + hs[a]) * Wp + ws[b]) * C4 + c4]);
  reinterpret_cast<float4*>(dx)[idx] = acc;
}

// ---------------------------------------------------------------------------------- dispatch
// Tile kinds: 0 = 128x128 (8 waves, 64x32 each), 1 = 64x128 (4 waves), 2 = 128x64 (4 waves),
// 3 = 64x64 (4 waves), 4 = 256x32 (skinny N), 5 = 128x128 (4 waves, 64x64 each).
enum TileKind { T128x128w8 = 0, T64x128 = 1, T128x64 = 2, T64x64 = 3, T256x32 = 4, T128x128w4 = 5, TAUTO = -1 };
// Debug tile override (vst_debug_set_tiles): per calling host thread, so concurrent callers on
// other threads / streams are never affected (the library keeps no other mutable state).
static thread_local int g_tile_override[3] = {TAUTO, TAUTO, TAUTO};

static int tile_bm(TileKind k) { return k == T64x128 || k == T64x64 ? 64 : (k == T256x32 ? 256 : 128); }
static int tile_bn(TileKind k) {
  return k == T128x64 || k == T64x64 ? 64 : (k == T256x32 ? 32 : 128);
}

static TileKind pick_tile(long M, int Nc, int which) {
  if (g_tile_override[which] != TAUTO) return (TileKind)g_tile_override[which];
  if (Nc <= 32) return T256x32;
  if (Nc <= 64) return M / 128 >= 256 ? T128x64 : T64x64;
  const long n128 = (Nc + 127) / 128;
  if ((M / 128) * n128 >= 200) return T128x128w8;
  if ((M / 64) * n128 >= 200) return T64x128;
  return T64x64;
}

#define VST_DISPATCH_TILE(kind, LAUNCH)                       \
  switch (kind) {                                              \
    case T128x128w8: LAUNCH(128, 128, 64, 32); break;          \
    case T64x128: LAUNCH(64, 128, 32, 64); break;              \
    case T128x64: LAUNCH(128, 64, 64, 32); break;              \
    case T256x32: LAUNCH(256, 32, 64, 32); break;              \
    case T128x128w4: LAUNCH(128, 128, 64, 64); break;          \
    default: LAUNCH(64, 64, 32, 32); break;                    \
  }

struct WgradPlan {
  int Mw, nsplit, chunk;
  TileKind tile;
  bool trans;        // channel-major operand copies + conv_wgrad_rk_k (stride 1, Wo % 4 == 0)
  bool bfk;          // trans, on the split-bf16 kernel (conv_wgrad_bf_k; x6, Wo % 8 == 0): dy as
                     // pre-split bf16 planes, `tile` is then a conv_bf tile kind
  int pad;           // trans: the border the padded x copy carries (derived from H -> Ho)
  int wpad;          // bfk, stride 1, Wo % 8 != 0: output columns padded to a multiple of 8 (zero dy)
  long xt_floats;    // workspace floats after the slabs: xt [Cx][N*Hp*Wp] then dyt [Cyp][P]
  long dyt_floats;
};

// Split count whose grid fills its last "round" (slots co-resident blocks) best, among grids of
// at least ~3/4 of a round (a 288-block grid on 256 CUs runs two rounds for 1.125 rounds of work).
#ifndef WGRAD_CHUNK_MAX
#define WGRAD_CHUNK_MAX 4096  // pixels per split-K chunk: keeps a block's operand rows L2-resident (A/B: none 53.2, 2560 55.0, 4096 55.7 frames/s)
#endif

static int pick_splits(int tiles, int slots, int max_ns, int min_ns = 1) {
  if (max_ns < 1) max_ns = 1;
  if (min_ns > max_ns) min_ns = max_ns;
  if (min_ns < 1) min_ns = 1;
  int ns = min_ns;
  double best = -1.0;
  for (int c = min_ns; c <= max_ns; ++c) {
    const long blocks = (long)tiles * c;
    const double fill = (double)blocks / (double)(((blocks + slots - 1) / slots) * slots);
    const double score = blocks < (3 * slots) / 4 ? fill * blocks / slots : fill;
    if (score > best + 1e-9) { best = score; ns = c; }
    if (blocks >= 2 * slots) break;
  }
  return ns;
}

#ifndef VST_WG_BIG
#define VST_WG_BIG 5  // rk tile kind of the wide (Cyp > 64, Mw >= 1024) weight gradients
#endif
#ifndef VST_WG_PADW
#define VST_WG_PADW 1  // stride-1 x6 wgrads with Wo % 8 != 0 on the split-bf16 kernel via Wo-padded rows
#endif
#ifndef VST_WG_BIGM
#define VST_WG_BIGM 512  // x6 wgrads with Cyp > 64 and Mw >= this run on 256x128 tiles (A/B: 1024 -> 512, -0.15 ms/step)
#endif
#ifndef VST_WG_BF
#define VST_WG_BF 1   // x6 weight gradients on the split-bf16 kernel (conv_wgrad_bf_k)
#endif

static constexpr int g_wg_kind_s2 = -1;

static WgradPlan plan_wgrad(int N, int H, int W, int Ho, int Wo, int Cx, int Cyp, int R, int S,
                            int stride, int math) {
  WgradPlan p;
  p.Mw = R * S * Cx;
  p.trans = false;
  p.bfk = false;
  p.pad = 0;
  p.wpad = 0;
  p.xt_floats = p.dyt_floats = 0;
  const int P = N * Ho * Wo;
  const int ov = g_tile_override[2];
  const int pd2 = Ho - H + R - 1;  // stride 1: 2 * pad
  const bool s1 = stride == 1 && pd2 >= 0 && pd2 % 2 == 0 && Wo - W + S - 1 == pd2;
  // stride 2: the pad is not recoverable from the shapes; the padded copy is sized for pad <= R - 1
  // (checked at the call) and its rows are column-phase split, which needs W + 2 pad even
  const bool s2 = stride == 2 && W % 2 == 0;
  // stride 1 with Wo % 8 != 0 (PatchGAN's 31-wide layer): the output rows padded to a multiple of
  // 8 columns with zero dy (and zero x columns past the border), so 8-pixel chunks stay in one row
  const int wpad = (s1 && Wo % 8 && Wo >= 8 && VST_WG_PADW) ? (8 - Wo % 8) : 0;
  if (Cyp > 4 && (s1 || s2) && (Wo + wpad) % 8 == 0 && ov < 0 && math == VST_MATH_BF16X6 && VST_WG_BF) {
    // x6: the split-bf16 weight-gradient kernel (conv_bf.hip), 256x128 tiles for the wide layers
    p.trans = p.bfk = true;
    p.pad = s1 ? pd2 / 2 : -1;
    p.wpad = wpad;
    int kind = Cyp > 64 ? (p.Mw >= VST_WG_BIGM ? 7 : 3) : (p.Mw >= 1024 ? 1 : 8);
    // M rows (tap, ci) that 256-row tiles pad more than 128-row ones (the generator's stride-2 3x3 layers:
    // 576 rows = 2.25 x 256, 1152 = 4.5 x 256) run on 128x128 tiles of 8 waves (64x32); round-5 sweep
    // (profiles/r05e_convT_wgrad_tiles.jsonl): 178 -> 172 / 149 -> 136 us at N = 8
    if (kind == 7 && ceil_div(p.Mw, 256) * 256 > ceil_div(p.Mw, 128) * 128) kind = 0;
    if (g_wg_kind_s2 >= 0 && stride == 2) kind = g_wg_kind_s2;  // developer A/B (g_wg_kind_s2)
    p.tile = (TileKind)kind;
    int bm, bn, bk, slots;
    bf_wgrad_geom(kind, math, &bm, &bn, &bk, &slots);
    const int tiles = ceil_div(p.Mw, bm) * ceil_div(Cyp, bn);
    const int Pw = N * Ho * (Wo + wpad);
    const int ns = pick_splits(tiles, slots, ceil_div(Pw, 8 * bk) < 256 ? ceil_div(Pw, 8 * bk) : 256,
                               ceil_div(Pw, WGRAD_CHUNK_MAX));
    p.chunk = ceil_div(ceil_div(Pw, ns), bk) * bk;
    p.nsplit = ceil_div(Pw, p.chunk);
    const int pmax = s1 ? p.pad : (R > S ? R : S) - 1;
    p.xt_floats = rk_cp_ld((long)N * (H + 2 * pmax) * (W + 2 * pmax + wpad)) * Cx;  // padded fp32 image
    p.dyt_floats = (rk_cp_ld(Pw) * Cyp * 3 + 1) / 2;                                // 3 bf16 planes
    return p;
  }
  if (Cyp > 4 && (s1 || s2) && Wo % 4 == 0 && ov < 8) {
    p.trans = true;
    p.pad = s1 ? pd2 / 2 : -1;
    // wide layers: 4 waves of 64x64 (two blocks per CU) under x3; under x6 the 128x128 image fits
    // one block per CU, so the 8-wave kind keeps two waves per SIMD
    const int wide = math == VST_MATH_BF16X6 ? 0 : VST_WG_BIG;
    int kind = (ov >= 0 && ov <= 6) ? ov : (Cyp <= 64 ? (p.Mw >= 1024 ? 2 : 3) : (p.Mw >= 1024 ? wide : 1));
    p.tile = (TileKind)kind;
    int bm, bn, bk, slots;
    rk_tile_geom(kind, math, &bm, &bn, &bk, &slots);
    const int tiles = ceil_div(p.Mw, bm) * ceil_div(Cyp, bn);
    const int ns = pick_splits(tiles, slots, ceil_div(P, 8 * bk) < 256 ? ceil_div(P, 8 * bk) : 256,
                               ceil_div(P, WGRAD_CHUNK_MAX));
    p.chunk = ceil_div(ceil_div(P, ns), bk) * bk;
    p.nsplit = ceil_div(P, p.chunk);
    const int pmax = s1 ? p.pad : (R > S ? R : S) - 1;
    p.xt_floats = rk_cp_ld((long)N * (H + 2 * pmax) * (W + 2 * pmax)) * Cx;  // padded image
    p.dyt_floats = rk_cp_ld(P) * Cyp;
    return p;
  }
  if (Cyp == 4) {  // VALU skinny path: one thread per (tap, 4 input channels) per split
    p.tile = T256x32;
    int ns = ceil_div(262144, p.Mw / 4);  // ~4 waves per SIMD
    if (ns > 256) ns = 256;
    const int max_ns = ceil_div(P, 64);
    if (ns > max_ns) ns = max_ns;
    if (ns < 1) ns = 1;
    p.chunk = ceil_div(P, ns);
    p.nsplit = ceil_div(P, p.chunk);
    return p;
  }
  if (Cyp <= 32) p.tile = T256x32;
  else if (Cyp <= 64) p.tile = p.Mw >= 1024 ? T128x64 : T64x64;
  else p.tile = p.Mw >= 1024 ? T128x128w8 : T64x128;
  if (ov >= 0) p.tile = (TileKind)(ov >= 8 ? ov - 8 : ov);
  const int tiles = ceil_div(p.Mw, tile_bm(p.tile)) * ceil_div(Cyp, tile_bn(p.tile));
  // one 8-wave or two 4-wave blocks per CU form a round of 256 / 512 blocks
  const int max_ns = ceil_div(P, 8 * BK);  // at least 8 K-steps per split
  const int ns = pick_splits(tiles, p.tile == T128x128w8 ? 256 : 512, max_ns < 64 ? max_ns : 64);
  p.chunk = ceil_div(ceil_div(P, ns), BK) * BK;
  p.nsplit = ceil_div(P, p.chunk);
  return p;
}

}  // namespace vst

using namespace vst;

// 4-channel inputs (images) on the split-bf16 kernels (conv_fprop_bf_k<.., false, 3>) rather than
// the fp32 [row][k] kernels; g_bf_c4 = false restores the latter (route selectors like this are compile-time constants).
// wgrad_reduce_store_k on 16-row blocks (g_wg_red16 = false: 32-row): twice the blocks for the same slabs,
// -0.16 ms/step in the same-box A/B (profiles/r03d_wgred_step_ab.jsonl)
static constexpr bool g_wg_red16 = true;

static constexpr bool g_bf_c4 = true;

extern "C" void vst_debug_set_tiles(int fprop, int tconv, int wgrad) {
  g_tile_override[0] = fprop;
  g_tile_override[1] = tconv;
  g_tile_override[2] = wgrad;
}

extern "C" int vst_conv_plan_fwd(int N, int H, int W, int Cx, int Cop, int R, int S, int stride, int padh,
                                 int padw, int math, int* kind, int* m_split, int* tail_kind) {
  VST_REQUIRE(kind && m_split && tail_kind && N > 0 && H > 0 && W > 0 && R > 0 && S > 0 && stride > 0,
              "conv_plan_fwd: bad args");
  const int Ho = (H + 2 * padh - R) / stride + 1, Wo = (W + 2 * padw - S) / stride + 1;
  VST_REQUIRE(Ho > 0 && Wo > 0, "conv_plan_fwd: empty output");
  *m_split = 0;
  *tail_kind = -1;
  if (Cop == 4) {
    *kind = VST_PLAN_SKINNY;
  } else if (Cx == 4 && g_bf_c4 && g_tile_override[0] < 0 && padh == padw &&
             c4_direct_ok(Cx, Cop, R, S, stride, Ho, Wo, math)) {
    *kind = VST_PLAN_C4_DIRECT;
  } else if (math != VST_MATH_F32 && (Cx % 8 == 0 || (Cx == 4 && g_bf_c4))) {
    bf_plan((long)N * Ho * Wo, Cop, math, g_tile_override[0], kind, m_split, tail_kind);
  } else {
    *kind = VST_PLAN_RK;
  }
  return VST_OK;
}

static int conv_fwd_impl(const float* x, const float* wp, const void* wsplit, const float* bias, float* y,
                         int N, int H, int W, int Cx, int Cop, int R, int S, int stride, int padh, int padw,
                         int pad_mode, int act, float slope, int math, hipStream_t s, double* part = nullptr,
                         int* nsplit = nullptr, float* tws = nullptr, size_t tws_bytes = 0, int co_real = 4) {
  if (nsplit) *nsplit = 0;
  VST_REQUIRE(x && wp && y, "conv2d_fwd: null pointer");
  VST_REQUIRE(math >= VST_MATH_F32 && math <= VST_MATH_BF16X6, "conv2d_fwd: bad math %d", math);
  VST_REQUIRE(N > 0 && H > 0 && W > 0 && R > 0 && S > 0 && stride > 0 && padh >= 0 && padw >= 0,
              "conv2d_fwd: bad shape");
  VST_REQUIRE(Cx % 4 == 0 && Cop % 4 == 0, "conv2d_fwd: channel strides must be multiples of 4");
  VST_REQUIRE(pad_mode == VST_PAD_ZERO || (padh < H && padw < W), "conv2d_fwd: reflect pad >= size");
  const int Ho = (H + 2 * padh - R) / stride + 1, Wo = (W + 2 * padw - S) / stride + 1;
  VST_REQUIRE(Ho > 0 && Wo > 0, "conv2d_fwd: empty output");
  const int refl = pad_mode == VST_PAD_REFLECT;
  if (Cop == 4) {  // image-channel outputs / PatchGAN head: VALU path (skinny.hip)
    VST_REQUIRE(padh == padw, "conv2d_fwd: the 4-channel-output path needs equal row/column padding");
    return skinny_out_launch(0, x, wp, bias, nullptr, y, N, H, W, Cx, Ho, Wo, R, S, stride, padh, refl,
                             act, slope, s, co_real);
  }
  if (math != VST_MATH_F32 && wsplit && (Cx % 8 == 0 || (Cx == 4 && g_bf_c4))) {
    // InstanceNorm partials from the epilogue: 32-pixel groups, so the image size must divide
    const bool stats = part && nsplit && (Ho * Wo) % 32 == 0;
    const int rc = bf_fprop_launch(x, wsplit, (long)Cop * R * S * Cx, bias, y, N, H, W, Cx, Ho, Wo, Cop, R, S,
                                   stride, padh, padw, refl, act, slope, math, g_tile_override[0], s,
                                   stats ? part : nullptr, tws, tws_bytes / sizeof(float));
    if (stats && rc == 0) *nsplit = Ho * Wo / 32;
    return rc;
  }
  rk_fprop_launch(x, wp, bias, y, N, H, W, Cx, Ho, Wo, Cop, R, S, stride, padh, padw, refl, act, slope,
                  g_tile_override[0], math, s);
  return check_launch("conv2d_fwd");
}

extern "C" int vst_conv2d_fwd(const float* x, const float* wp, const void* wsplit, const float* bias,
                              float* y, int N,
                              int H, int W, int Cx, int Cop, int R, int S, int stride, int pad,
                              int pad_mode, int act, float slope, int math, void* stream) {
  return conv_fwd_impl(x, wp, wsplit, bias, y, N, H, W, Cx, Cop, R, S, stride, pad, pad, pad_mode, act, slope,
                       math, (hipStream_t)stream);
}

extern "C" int vst_conv2d_fwd_co(const float* x, const float* wp, const void* wsplit, const float* bias, float* y,
                                 int N, int H, int W, int Cx, int Cop, int R, int S, int stride, int pad, int pad_mode,
                                 int act, float slope, int math, int co_real, void* stream) {
  VST_REQUIRE(co_real >= 1 && co_real <= Cop, "conv2d_fwd_co: bad real channel count %d", co_real);
  return conv_fwd_impl(x, wp, wsplit, bias, y, N, H, W, Cx, Cop, R, S, stride, pad, pad, pad_mode, act, slope,
                       math, (hipStream_t)stream, nullptr, nullptr, nullptr, 0, co_real);
}

extern "C" size_t vst_conv2d_fwd_co_ws_bytes(int N, int H, int W, int Cx, int Cop, int R, int S, int stride, int pad,
                                             int pad_mode, int co_real) {
  if (N <= 0 || H <= 0 || W <= 0 || co_real != 1 || Cop != 4 || !g_head) return 0;
  const int Ho = (H + 2 * pad - R) / stride + 1, Wo = (W + 2 * pad - S) / stride + 1;
  if (Ho <= 0 || Wo <= 0 || !head_ok(Cx, R, S, stride, pad_mode == VST_PAD_REFLECT, Wo) || !head_tap_ok(Cx)) return 0;
  return head_tap_ws_floats(N, H, W) * sizeof(float);
}

extern "C" int vst_conv2d_fwd_co_ws(const float* x, const float* wp, const void* wsplit, const float* bias, float* y,
                                    int N, int H, int W, int Cx, int Cop, int R, int S, int stride, int pad,
                                    int pad_mode, int act, float slope, int math, int co_real, float* ws,
                                    size_t ws_bytes, void* stream) {
  const size_t need = vst_conv2d_fwd_co_ws_bytes(N, H, W, Cx, Cop, R, S, stride, pad, pad_mode, co_real);
  if (need && ws && ws_bytes >= need && x && wp && y) {
    const int Ho = (H + 2 * pad - R) / stride + 1, Wo = (W + 2 * pad - S) / stride + 1;
    return head_tap_fwd_launch(x, wp, bias, y, ws, N, H, W, Cx, Ho, Wo, R, S, pad, act, slope, (hipStream_t)stream);
  }
  return vst_conv2d_fwd_co(x, wp, wsplit, bias, y, N, H, W, Cx, Cop, R, S, stride, pad, pad_mode, act, slope, math,
                           co_real, stream);
}

extern "C" int vst_conv2d_fwd_in(const float* x, const float* wp, const void* wsplit, const float* bias,
                                 float* y, int N, int H, int W, int Cx, int Cop, int R, int S, int stride,
                                 int pad, int pad_mode, int act, float slope, int math, double* part,
                                 int* nsplit, void* stream) {
  VST_REQUIRE(part && nsplit, "conv2d_fwd_in: null partials");
  return conv_fwd_impl(x, wp, wsplit, bias, y, N, H, W, Cx, Cop, R, S, stride, pad, pad, pad_mode, act, slope,
                       math, (hipStream_t)stream, part, nsplit);
}

extern "C" size_t vst_conv2d_fwd_ws_bytes(int N, int H, int W, int Cx, int Cop, int R, int S, int stride, int pad,
                                          int math) {
  if (N <= 0 || H <= 0 || W <= 0 || R <= 0 || S <= 0 || stride <= 0 || Cx % 8 || Cop == 4) return 0;
  const int Ho = (H + 2 * pad - R) / stride + 1, Wo = (W + 2 * pad - S) / stride + 1;
  if (Ho <= 0 || Wo <= 0 || g_tile_override[0] >= 0) return 0;
  return bf_fprop_ws_floats((long)N * Ho * Wo, Cop, Cx, R, S, math) * sizeof(float);
}

extern "C" int vst_conv2d_fwd_ws(const float* x, const float* wp, const void* wsplit, const float* bias, float* y,
                                 int N, int H, int W, int Cx, int Cop, int R, int S, int stride, int pad, int pad_mode,
                                 int act, float slope, int math, double* part, int* nsplit, float* ws,
                                 size_t ws_bytes, void* stream) {
  return conv_fwd_impl(x, wp, wsplit, bias, y, N, H, W, Cx, Cop, R, S, stride, pad, pad, pad_mode, act, slope,
                       math, (hipStream_t)stream, part, nsplit, ws, ws_bytes);
}

extern "C" int vst_conv_plan_fwd_tail(int N, int H, int W, int Cx, int Cop, int R, int S, int stride, int pad,
                                      int math, int* ksplit) {
  VST_REQUIRE(ksplit, "conv_plan_fwd_tail: null");
  *ksplit = 0;
  const size_t b = vst_conv2d_fwd_ws_bytes(N, H, W, Cx, Cop, R, S, stride, pad, math);
  if (b) {
    const int Ho = (H + 2 * pad - R) / stride + 1, Wo = (W + 2 * pad - S) / stride + 1;
    int mf;
    bf_split_plan((long)N * Ho * Wo, Cop, Cx, R, S, math, -1, &mf, ksplit);
  }
  return VST_OK;
}

// vst_conv2d_fwd_hw with a padding mode (vst_tapconv_h_fwd's R x 1 reflect conv)
extern "C" int vst_conv2d_fwd_hwp(const float* x, const float* wp, const void* wsplit, const float* bias, float* y,
                                  int N, int H, int W, int Cx, int Cop, int R, int S, int stride, int pad_h, int pad_w,
                                  int pad_mode, int act, float slope, int math, void* stream) {
  return conv_fwd_impl(x, wp, wsplit, bias, y, N, H, W, Cx, Cop, R, S, stride, pad_h, pad_w, pad_mode, act, slope,
                       math, (hipStream_t)stream);
}

extern "C" int vst_conv2d_fwd_hw(const float* x, const float* wp, const void* wsplit, const float* bias,
                                 float* y, int N, int H, int W, int Cx, int Cop, int R, int S, int stride,
                                 int pad_h, int pad_w, int act, float slope, int math, void* stream) {
  return conv_fwd_impl(x, wp, wsplit, bias, y, N, H, W, Cx, Cop, R, S, stride, pad_h, pad_w, VST_PAD_ZERO, act,
                       slope, math, (hipStream_t)stream);
}

// vst_conv2d_fwd_hw with a workspace: the split-K plans of vst_conv2d_fwd_ws for grids that cannot fill the CUs
// (RAFT's SepConvGRU (1,5) / (5,1) convs at 1/8 resolution: M = 7040 rows at Sintel size)
extern "C" size_t vst_conv2d_fwd_hw_ws_bytes(int N, int H, int W, int Cx, int Cop, int R, int S, int stride, int pad_h,
                                             int pad_w, int math) {
  if (N <= 0 || H <= 0 || W <= 0 || R <= 0 || S <= 0 || stride <= 0 || Cx % 8 || Cop == 4) return 0;
  const int Ho = (H + 2 * pad_h - R) / stride + 1, Wo = (W + 2 * pad_w - S) / stride + 1;
  if (Ho <= 0 || Wo <= 0 || g_tile_override[0] >= 0) return 0;
  return bf_fprop_ws_floats((long)N * Ho * Wo, Cop, Cx, R, S, math) * sizeof(float);
}

extern "C" int vst_conv2d_fwd_hw_ws(const float* x, const float* wp, const void* wsplit, const float* bias, float* y,
                                    int N, int H, int W, int Cx, int Cop, int R, int S, int stride, int pad_h,
                                    int pad_w, int act, float slope, int math, float* ws, size_t ws_bytes,
                                    void* stream) {
  return conv_fwd_impl(x, wp, wsplit, bias, y, N, H, W, Cx, Cop, R, S, stride, pad_h, pad_w, VST_PAD_ZERO, act,
                       slope, math, (hipStream_t)stream, nullptr, nullptr, ws, ws_bytes);
}

// One phase (a, b) of a stride-2 ConvTranspose2d(k3, p1, op1) stored straight into the interleaved
// 2H x 2W output y (the phase conv of conv2d_fwd_hw(x, wp, R = 1 + a, S = 1 + b, pad a / b), whose pixel
// (ph, pw) is y's (2(ph-a)+a, 2(pw-b)+b)): the four phases replace four phase images + the
// vst_interleave_phases pass.  Split-bf16 arithmetic only (VST_EUNSUPPORTED otherwise: use the
// phase images + interleave).
extern "C" int vst_conv2d_fwd_phase(const float* x, const void* wsplit, const float* bias, float* y, int N, int H,
                                    int W, int Cx, int Cop, int a, int b, int act, float slope, int math,
                                    void* stream) {
  VST_REQUIRE(x && wsplit && y && (a == 0 || a == 1) && (b == 0 || b == 1), "conv2d_fwd_phase: bad args");
  VST_REQUIRE(N > 0 && H > 0 && W > 0 && Cx % 8 == 0 && Cop % 4 == 0 && Cop != 4, "conv2d_fwd_phase: bad shape");
  if (math == VST_MATH_F32) {
    ::vst::set_error("conv2d_fwd_phase: split-bf16 arithmetic only");
    return VST_EUNSUPPORTED;
  }
  const int R = 1 + a, S = 1 + b;
  return bf_fprop_launch(x, wsplit, (long)Cop * R * S * Cx, bias, y, N, H, W, Cx, H + a, W + b, Cop, R, S, 1, a, b, 0,
                         act, slope, math, g_tile_override[0], (hipStream_t)stream, nullptr, nullptr, 0, nullptr,
                         1 + 2 * a + b);
}

extern "C" int vst_conv2d_convT_s2(const float* x, const void* ws00, const void* ws01, const void* ws10,
                                   const void* ws11, const float* bias, float* y, int N, int H, int W, int Cx, int Cop,
                                   int act, float slope, int math, void* stream) {
  VST_REQUIRE(x && ws00 && ws01 && ws10 && ws11 && y && N > 0 && H > 0 && W > 0, "conv2d_convT_s2: bad args");
  if (!bf_convT_phases_ok(Cx, Cop, math)) {
    ::vst::set_error("conv2d_convT_s2: needs split-bf16 math, Cx %% 32 == 0, Cop %% 4 == 0");
    return VST_EUNSUPPORTED;
  }
  const void* ws[4] = {ws00, ws01, ws10, ws11};
  return bf_convT_phases_launch(x, ws, bias, y, N, H, W, Cx, Cop, act, slope, math, (hipStream_t)stream);
}

extern "C" int vst_conv4s2_dgrad(const float* dy, const void* ws00, const void* ws01, const void* ws10,
                                 const void* ws11, float* dx, int N, int Hd, int Wd, int Cy, int Cop, int math,
                                 void* stream) {
  VST_REQUIRE(dy && ws00 && ws01 && ws10 && ws11 && dx && N > 0 && Hd > 0 && Wd > 0, "conv4s2_dgrad: bad args");
  if (!bf_convT_phases_ok(Cy, Cop, math)) {
    ::vst::set_error("conv4s2_dgrad: needs split-bf16 math, Cy %% 32 == 0, Cop %% 4 == 0");
    return VST_EUNSUPPORTED;
  }
  const void* ws[4] = {ws00, ws01, ws10, ws11};
  return bf_convT_phases_launch(dy, ws, nullptr, dx, N, Hd, Wd, Cy, Cop, VST_ACT_NONE, 0.f, math, (hipStream_t)stream,
                                1);
}

extern "C" int vst_conv2d_tfwd(const float* in, const float* wp, const float* bias,
                               const float* addend, float* out, int N, int Hi, int Wi, int Cy,
                               int Ho, int Wo, int Cx, int R, int S, int stride, int pad,
                               int pad_mode, int act, float slope, int math, void* stream) {
  VST_REQUIRE(in && wp && out, "conv2d_tfwd: null pointer");
  VST_REQUIRE(math >= VST_MATH_F32 && math <= VST_MATH_BF16X6, "conv2d_tfwd: bad math %d", math);
  VST_REQUIRE(N > 0 && Hi > 0 && Wi > 0 && Ho > 0 && Wo > 0 && R > 0 && S > 0 && stride > 0 && pad >= 0,
              "conv2d_tfwd: bad shape");
  VST_REQUIRE(Cy % 4 == 0 && Cx % 4 == 0, "conv2d_tfwd: channel strides must be multiples of 4");
  const int refl = pad_mode == VST_PAD_REFLECT;
  VST_REQUIRE(!refl || (stride == 1 && Ho > 2 * pad + 1 && Wo > 2 * pad + 1),
              "conv2d_tfwd: reflect needs stride 1 and H, W > 2*pad+1");
  hipStream_t s = (hipStream_t)stream;
  const int Hc = (Ho + stride - 1) / stride, Wc = (Wo + stride - 1) / stride;
  const int Mmax = N * Hc * Wc;
  if (Cx == 4)  // image-channel data gradients: VALU path (skinny.hip)
    return skinny_out_launch(1, in, wp, bias, addend, out, N, Hi, Wi, Cy, Ho, Wo, R, S, stride, pad,
                             refl, act, slope, s);
#define VST_TCONV_ST(BM_, BN_, WM_, WN_, ST_)                                                      \
  hipLaunchKernelGGL((conv_tconv_k<BM_, BN_, WM_, WN_, ST_>),                                       \
                     dim3(ceil_div(Mmax, BM_), ceil_div(Cx, BN_), stride * stride),                  \
                     dim3(Tile<BM_, BN_, WM_, WN_>::NT), 0, s, in, wp, bias, addend, out, Hi, Wi, Cy, \
                     Ho, Wo, Cx, R, S, stride, pad, refl, act, slope, N)
#define VST_TCONV(BM_, BN_, WM_, WN_)                     \
  if (stride == 1) VST_TCONV_ST(BM_, BN_, WM_, WN_, 1);     \
  else if (stride == 2) VST_TCONV_ST(BM_, BN_, WM_, WN_, 2); \
  else VST_TCONV_ST(BM_, BN_, WM_, WN_, 0);
  (void)Mmax;
  rk_tconv_launch(in, wp, bias, addend, out, N, Hi, Wi, Cy, Ho, Wo, Cx, R, S, stride, pad, refl, act,
                  slope, g_tile_override[1], math, s);
#undef VST_TCONV
#undef VST_TCONV_ST
  return check_launch("conv2d_tfwd");
}

extern "C" int vst_conv2d_tfwd_co(const float* in, const float* wp, const float* bias, const float* addend, float* out,
                                  int N, int Hi, int Wi, int Cy, int Ho, int Wo, int Cx, int R, int S, int stride,
                                  int pad, int pad_mode, int act, float slope, int math, int co_real, void* stream) {
  VST_REQUIRE(co_real >= 1 && co_real <= Cy, "conv2d_tfwd_co: bad real channel count %d", co_real);
  const int refl = pad_mode == VST_PAD_REFLECT;
  if (in && wp && out && co_real == 1 && Cy == 4 && !bias && act == VST_ACT_NONE && g_head && N > 0 && Hi > 0 &&
      Wi > 0 && pad >= 0 && head_ok(Cx, R, S, stride, refl, Wi) && Ho == Hi + R - 1 - 2 * pad &&
      Wo == Wi + S - 1 - 2 * pad)
    return head_dgrad_launch(in, wp, addend, out, N, Hi, Wi, Cx, Ho, Wo, R, S, pad, (hipStream_t)stream);
  return vst_conv2d_tfwd(in, wp, bias, addend, out, N, Hi, Wi, Cy, Ho, Wo, Cx, R, S, stride, pad, pad_mode, act, slope,
                         math, stream);
}

// Two-level split-K reduction (slab_group_sum_k first) when the fused reduce + store kernel would
// run on few blocks with a long serial slab chain per element.
static constexpr int WG_GROUP = 16;
// Image-input layers (x NHWC4 holding 3 logical channels) on the split-bf16 kernel: the GEMM takes only
// the rows (tap, ci < 3) of the 4-plane x image — M = 3RS instead of 4RS (the generator's first 7x7
// conv: 147 rows = 3 tiles of 64 instead of 4).  g_wg_c3 = false: all four planes.
static constexpr bool g_wg_c3 = true;

// The GEMM's plan for (Cx, logical Ci): p planned with Cx = 3 when the rule above applies; its
// operand-copy sizes stay those of the Cx-channel images.
static WgradPlan plan_wgrad_gemm(const WgradPlan& p, int N, int H, int W, int Ho, int Wo, int Cx, int Ci, int Cyp,
                                 int R, int S, int stride, int math, int* Cxg) {
  *Cxg = Cx;
  if (!(g_wg_c3 && p.bfk && Cx == 4 && Ci == 3)) return p;
  WgradPlan q = plan_wgrad(N, H, W, Ho, Wo, 3, Cyp, R, S, stride, math);
  if (!q.bfk || q.wpad != p.wpad || q.pad != p.pad) return p;
  q.xt_floats = p.xt_floats;
  q.dyt_floats = p.dyt_floats;
  *Cxg = 3;
  return q;
}

static bool wgrad_two_level(const WgradPlan& p, int Cyp, int Ci, int RS, int Co) {
  return p.nsplit > 2 * WG_GROUP && (long)ceil_div(Ci * RS, 64) * ceil_div(Co, 64) < 128;
}

static size_t wgrad_ws_floats(const WgradPlan& p, int Cyp) {
  // after the GEMM the operand copies are dead: the two-level reduction's group sums reuse them
  const size_t l2 = (size_t)ceil_div(p.nsplit, WG_GROUP) * p.Mw * Cyp;
  const size_t ops = p.xt_floats + p.dyt_floats;
  return (size_t)p.nsplit * p.Mw * Cyp + (ops > l2 ? ops : l2);
}

extern "C" int vst_conv_plan_wgrad(int N, int H, int W, int Cx, int Ho, int Wo, int Cyp, int R, int S,
                                   int stride, int math, int* path, int* kind, int* nsplit) {
  VST_REQUIRE(path && kind && nsplit && N > 0 && H > 0 && W > 0 && Ho > 0 && Wo > 0 && R > 0 && S > 0,
              "conv_plan_wgrad: bad args");
  const WgradPlan p = plan_wgrad(N, H, W, Ho, Wo, Cx, Cyp, R, S, stride, math);
  *path = p.bfk ? (p.wpad ? VST_WPLAN_BF_PADW : VST_WPLAN_BF) : p.trans ? VST_WPLAN_RK
                                                                     : Cyp == 4 ? VST_WPLAN_SKINNY : VST_WPLAN_GENERIC;
  *kind = (int)p.tile;
  *nsplit = p.nsplit;
  return VST_OK;
}

extern "C" size_t vst_conv2d_wgrad_ws_bytes(int N, int H, int W, int Cx, int Ho, int Wo, int Cyp,
                                            int R, int S, int stride) {
  // the plan (split count, tile) depends on the arithmetic: size for the largest
  size_t mx = 0;
  for (int math = VST_MATH_F32; math <= VST_MATH_BF16X6; ++math) {
    const WgradPlan p = plan_wgrad(N, H, W, Ho, Wo, Cx, Cyp, R, S, stride, math);
    int cxg;
    const WgradPlan pg = plan_wgrad_gemm(p, N, H, W, Ho, Wo, Cx, 3, Cyp, R, S, stride, math, &cxg);
    const size_t b = wgrad_ws_floats(p, Cyp) * sizeof(float), bg = wgrad_ws_floats(pg, Cyp) * sizeof(float);
    mx = b > mx ? b : mx;
    mx = bg > mx ? bg : mx;
  }
  if (Cyp == 4 && stride == 1) {  // a one-channel head may take patch.hip's row kernel
    const size_t hb = head_wgrad_ws_floats(N, H, Cx, R, S) * sizeof(float);
    mx = hb > mx ? hb : mx;
  }
  if (Cx == 4) {  // an image-input layer may take patch.hip's fp32-MFMA kernel
    const size_t ib = img_wgrad_ws_floats(N, Ho, Wo) * sizeof(float);
    mx = ib > mx ? ib : mx;
  }
  return mx;
}

extern "C" long vst_cp_ld(long P) { return rk_cp_ld(P); }

extern "C" int vst_conv2d_wgrad_pre(const float* x, const float* x_t, const float* dy, const void* dy_planes,
                                    float* dw, float* ws, size_t ws_bytes, int N, int H, int W, int Cx, int Ho, int Wo,
                                    int Cyp, int R, int S, int stride, int pad, int pad_mode, int Co, int Ci, long so,
                                    long si, int accumulate, int math, void* stream);

extern "C" int vst_conv2d_wgrad(const float* x, const float* dy, float* dw, float* ws,
                                size_t ws_bytes, int N, int H, int W, int Cx, int Ho, int Wo,
                                int Cyp, int R, int S, int stride, int pad, int pad_mode, int Co,
                                int Ci, long so, long si, int accumulate, int math, void* stream) {
  return vst_conv2d_wgrad_pre(x, nullptr, dy, nullptr, dw, ws, ws_bytes, N, H, W, Cx, Ho, Wo, Cyp, R, S, stride, pad,
                              pad_mode, Co, Ci, so, si, accumulate, math, stream);
}

extern "C" int vst_conv2d_wgrad_pre(const float* x, const float* x_t, const float* dy, const void* dy_planes,
                                    float* dw, float* ws, size_t ws_bytes, int N, int H, int W, int Cx, int Ho, int Wo,
                                    int Cyp, int R, int S, int stride, int pad, int pad_mode, int Co, int Ci, long so,
                                    long si, int accumulate, int math, void* stream) {
  VST_REQUIRE(x && dy && dw && ws, "conv2d_wgrad: null pointer");
  VST_REQUIRE(math >= VST_MATH_F32 && math <= VST_MATH_BF16X6, "conv2d_wgrad: bad math %d", math);
  const WgradPlan p0 = plan_wgrad(N, H, W, Ho, Wo, Cx, Cyp, R, S, stride, math);
  // any Cx when the split-bf16 kernel reads a caller-made channel-major x image (no NHWC vector loads of x)
  VST_REQUIRE((Cx % 4 == 0 || (x_t && p0.bfk && !p0.wpad)) && Cyp % 4 == 0,
              "conv2d_wgrad: channel strides must be multiples of 4");
  VST_REQUIRE(Co <= Cyp && Ci <= Cx, "conv2d_wgrad: logical channels exceed strides");
  VST_REQUIRE(pad_mode == VST_PAD_ZERO || (pad < H && pad < W), "conv2d_wgrad: reflect pad >= size");
  if (!x_t && !dy_planes && g_img_wgrad && img_wgrad_ok(Cx, Cyp, R, S, stride, pad_mode == VST_PAD_REFLECT, Ci, Wo) &&
      Co <= Cyp && ws_bytes >= img_wgrad_ws_floats(N, Ho, Wo) * sizeof(float))
    return img_wgrad_launch(x, dy, dw, nullptr, ws, N, H, W, Ho, Wo, Cyp, R, S, stride, pad, Co, Ci, so, si, accumulate,
                            (hipStream_t)stream);
  int Cxg;  // the GEMM's channel count (3 for image-input layers, g_wg_c3)
  const WgradPlan p = plan_wgrad_gemm(p0, N, H, W, Ho, Wo, Cx, Ci, Cyp, R, S, stride, math, &Cxg);
  VST_REQUIRE(ws_bytes >= wgrad_ws_floats(p, Cyp) * sizeof(float),
              "conv2d_wgrad: workspace too small (%zu bytes)", ws_bytes);
  hipStream_t s = (hipStream_t)stream;
  const int P = N * Ho * Wo;
  const int refl = pad_mode == VST_PAD_REFLECT;
#define VST_WG(BM_, BN_, WM_, WN_)                                                                 \
  hipLaunchKernelGGL((conv_wgrad_k<BM_, BN_, WM_, WN_>),                                            \
                     dim3(ceil_div(p.Mw, BM_) * ceil_div(Cyp, BN_) * p.nsplit),                      \
                     dim3(Tile<BM_, BN_, WM_, WN_>::NT), 0, s, x, dy, ws, H, W, Cx, Ho, Wo, Cyp, S,  \
                     stride, pad, refl, p.Mw, P, p.chunk)
  if (p.trans) {
    VST_REQUIRE(stride == 2 ? (pad <= R - 1 && pad <= S - 1 && Ho == (H + 2 * pad - R) / 2 + 1 &&
                               Wo == (W + 2 * pad - S) / 2 + 1)
                            : pad == p.pad,
                "conv2d_wgrad: pad %d inconsistent with H %d -> Ho %d (stride %d)", pad, H, Ho, stride);
    float* xt = ws + (size_t)p.nsplit * p.Mw * Cyp;
    float* dyt = xt + p.xt_floats;
    if (p.bfk) {
      if (p.wpad) {  // Wo-padded rows: the producer-made images do not have this layout
        x_t = nullptr;
        dy_planes = nullptr;
      }
      const int Wo8 = Wo + p.wpad;
      if (!x_t) rk_nhwc_to_cp_pad(x, xt, N, H, W, Cx, pad, refl, stride == 2, 0, s, p.wpad);  // else: vst_instnorm_act_fwd_cp
      if (!dy_planes)  // else: made by vst_instnorm_act_bwd_planes
        bf_nhwc_to_planes(dy, dyt, (long)N * Ho * Wo8, Cyp, 3, s, p.wpad ? Wo : 0, p.wpad ? Wo8 : 0);
      bf_wgrad_launch(x_t ? x_t : xt, dy_planes ? dy_planes : dyt, ws, N, H, W + p.wpad, Cxg, Ho, Wo8, Cyp, S, pad,
                      stride, p.Mw, p.chunk, p.nsplit, (int)p.tile, math, s);
    } else {
      const int pack = math == VST_MATH_BF16X3;  // the x3 kernel stages pre-split (hi, lo) words
      rk_nhwc_to_cp_pad(x, xt, N, H, W, Cx, pad, refl, stride == 2, pack, s);
      rk_nhwc_to_cp(dy, dyt, P, Cyp, pack, s);
      rk_wgrad_launch(xt, dyt, ws, N, H, W, Cx, Ho, Wo, Cyp, S, pad, stride, p.Mw, p.chunk, p.nsplit,
                      (int)p.tile, math, s);
    }
  } else if (Cyp == 4 && Co == 1 && g_head && head_ok(Cx, R, S, stride, refl, Wo) &&
             ws_bytes >= head_wgrad_ws_floats(N, H, Cx, R, S) * sizeof(float)) {
    // the PatchGAN head: the activation read once, partials reduced in a fixed order straight into dw
    return head_wgrad_launch(x, dy, dw, ws, N, H, W, Cx, Ci, Ho, Wo, R, S, pad, si, accumulate, s);
  } else if (Cyp == 4) {
    int rc0 = skinny_wgrad_launch(x, dy, ws, H, W, Cx, Ho, Wo, S, stride, pad, refl, p.Mw, P, p.chunk,
                                  p.nsplit, s);
    if (rc0) return rc0;
  } else {
    VST_DISPATCH_TILE(p.tile, VST_WG)
  }
#undef VST_WG
  int rc = check_launch("conv2d_wgrad");
  if (rc) return rc;
  // split-K slabs: summed in slab order and stored transposed in one pass (small outputs over many
  // slabs: groups of WG_GROUP slabs summed in parallel first, into the dead operand-copy region)
  const long slab = (long)p.Mw * Cyp;
  const float* red = ws;
  int nred = p.nsplit;
  if (wgrad_two_level(p, Cyp, Ci, R * S, Co)) {
    float* l2 = ws + (long)p.nsplit * slab;
    nred = ceil_div(p.nsplit, WG_GROUP);
    hipLaunchKernelGGL(slab_group_sum_k, dim3(ceil_div(slab / 4, 256), nred), dim3(256), 0, s, ws, l2, slab / 4,
                       p.nsplit, WG_GROUP);
    red = l2;
  }
  // 16-row blocks: twice the blocks (the 2304 x 256 ResnetBlock gradient: 288 -> 576); with at most 2 slabs the pass is
  // a transpose whose stores / accumulate reads are 16 floats per channel row with 16-row blocks: 32-row blocks keep
  // them whole 128-B lines (the StarGAN discriminator's 1024 -> 2048 layer, one slab, accumulated: 134 MB)
  if (g_wg_red16 && nred > 2)
    hipLaunchKernelGGL(wgrad_reduce_store_k<1>, dim3(ceil_div(Ci * R * S, 16), ceil_div(Co, 64)), dim3(256), 0, s,
                       red, dw, Cxg, Cyp, R * S, Co, Ci, so, si, accumulate, nred, slab);
  else
    hipLaunchKernelGGL(wgrad_reduce_store_k<2>, dim3(ceil_div(Ci * R * S, 32), ceil_div(Co, 64)), dim3(256), 0, s,
                       red, dw, Cxg, Cyp, R * S, Co, Ci, so, si, accumulate, nred, slab);
  return check_launch("conv2d_wgrad_reduce");
}

// The weight gradient over the NHWC operands the convs themselves use (round 6): x fp32 NHWC and dy as its NHWC
// bf16 planes dy_apl [3][N*Ho*Wo*Cyp] (the pre-split A operand the data gradient of the same layer reads), on the
// x6 256x128 plans of the split-bf16 kernel (conv_wgrad_nhwc_k: k-major stage images read by ds_read_b64_tr_b16).
// Same split plan, slabs and reduction as vst_conv2d_wgrad_pre (bit-identical results), but no padded
// channel-major x image and no channel-major dy planes: their producers (the IN apply / IN backward passes) need
// not write them.
static bool wgrad_nhwc_plan(int N, int H, int W, int Cx, int Ho, int Wo, int Cyp, int R, int S, int stride, int pad,
                            int math, WgradPlan* out) {
  if (math != VST_MATH_BF16X6 || R != S || Cx < 8) return false;
  const WgradPlan p = plan_wgrad(N, H, W, Ho, Wo, Cx, Cyp, R, S, stride, math);
  if (!p.bfk || p.wpad || !bf_wgrad_nhwc_ok((int)p.tile, Wo, Cx, Cyp)) return false;
  if (stride == 1 && p.pad != pad) return false;
  if (Ho != (H + 2 * pad - R) / stride + 1 || Wo != (W + 2 * pad - S) / stride + 1) return false;
  // the kernel addresses x and the planes through buffer descriptors with 32-bit byte offsets
  if ((long)N * H * W * Cx * 4 >= 0x7fff0000L || 3L * N * Ho * Wo * Cyp * 2 >= 0x7fff0000L) return false;
  *out = p;
  return true;
}

extern "C" int vst_conv2d_wgrad_nhwc_ok(int N, int H, int W, int Cx, int Ho, int Wo, int Cyp, int R, int S, int stride,
                                        int pad, int math) {
  WgradPlan p;
  return wgrad_nhwc_plan(N, H, W, Cx, Ho, Wo, Cyp, R, S, stride, pad, math, &p) ? 1 : 0;
}

extern "C" size_t vst_conv2d_wgrad_nhwc_ws_bytes(int N, int H, int W, int Cx, int Ho, int Wo, int Cyp, int R, int S,
                                                 int stride, int pad, int math) {
  WgradPlan p;
  if (!wgrad_nhwc_plan(N, H, W, Cx, Ho, Wo, Cyp, R, S, stride, pad, math, &p)) return 0;
  // the slabs, then (two-level reductions: many slabs of a small weight) the group sums
  return ((size_t)p.nsplit + ceil_div(p.nsplit, WG_GROUP)) * p.Mw * Cyp * sizeof(float);
}

static int wgrad_nhwc_impl(const float* x, const void* dy, bool bf32, float* dw, float* ws, size_t ws_bytes, int N,
                           int H, int W, int Cx, int Ho, int Wo, int Cyp, int R, int S, int stride, int pad,
                           int pad_mode, int Co, int Ci, long so, long si, int accumulate, int math, void* stream) {
  VST_REQUIRE(x && dy && dw && ws, "conv2d_wgrad_nhwc: null pointer");
  VST_REQUIRE(Co <= Cyp && Ci <= Cx && pad >= 0 && (pad_mode == VST_PAD_ZERO || (pad < H && pad < W)),
              "conv2d_wgrad_nhwc: bad args");
  WgradPlan p;
  if (!wgrad_nhwc_plan(N, H, W, Cx, Ho, Wo, Cyp, R, S, stride, pad, math, &p)) {
    ::vst::set_error("conv2d_wgrad_nhwc: unsupported shape / arithmetic (vst_conv2d_wgrad_nhwc_ok)");
    return VST_EUNSUPPORTED;
  }
  VST_REQUIRE(ws_bytes >= ((size_t)p.nsplit + ceil_div(p.nsplit, WG_GROUP)) * p.Mw * Cyp * sizeof(float),
              "conv2d_wgrad_nhwc: workspace too small (%zu bytes)", ws_bytes);
  hipStream_t s = (hipStream_t)stream;
  bf_wgrad_nhwc_launch(x, dy, (long)N * Ho * Wo * Cyp, bf32, ws, N, H, W, Cx, Ho, Wo, Cyp, S, pad, stride,
                       pad_mode == VST_PAD_REFLECT, p.Mw, p.chunk, p.nsplit, (int)p.tile, s);
  int rc = check_launch("conv2d_wgrad_nhwc");
  if (rc) return rc;
  // the split-K slabs reduced exactly as vst_conv2d_wgrad_pre's (same grouping and order: bit-identical)
  const long slab = (long)p.Mw * Cyp;
  const float* red = ws;
  int nred = p.nsplit;
  if (wgrad_two_level(p, Cyp, Ci, R * S, Co)) {
    float* l2 = ws + (long)p.nsplit * slab;
    nred = ceil_div(p.nsplit, WG_GROUP);
    hipLaunchKernelGGL(slab_group_sum_k, dim3(ceil_div(slab / 4, 256), nred), dim3(256), 0, s, ws, l2, slab / 4,
                       p.nsplit, WG_GROUP);
    red = l2;
  }
  if (nred > 2)
    hipLaunchKernelGGL(wgrad_reduce_store_k<1>, dim3(ceil_div(Ci * R * S, 16), ceil_div(Co, 64)), dim3(256), 0, s,
                       red, dw, Cx, Cyp, R * S, Co, Ci, so, si, accumulate, nred, slab);
  else
    hipLaunchKernelGGL(wgrad_reduce_store_k<2>, dim3(ceil_div(Ci * R * S, 32), ceil_div(Co, 64)), dim3(256), 0, s,
                       red, dw, Cx, Cyp, R * S, Co, Ci, so, si, accumulate, nred, slab);
  return check_launch("conv2d_wgrad_nhwc_reduce");
}

extern "C" int vst_conv2d_wgrad_nhwc(const float* x, const void* dy_apl, float* dw, float* ws, size_t ws_bytes, int N,
                                     int H, int W, int Cx, int Ho, int Wo, int Cyp, int R, int S, int stride, int pad,
                                     int pad_mode, int Co, int Ci, long so, long si, int accumulate, int math,
                                     void* stream) {
  return wgrad_nhwc_impl(x, dy_apl, false, dw, ws, ws_bytes, N, H, W, Cx, Ho, Wo, Cyp, R, S, stride, pad, pad_mode, Co,
                         Ci, so, si, accumulate, math, stream);
}

// ---- The im2col form of the fp32-dy NHWC weight gradient (round 6): output rows too short for the kernel's 32-pixel
// K steps (Wo % 32 != 0: the StarGAN discriminator's 16x16 / 8x8 / 4x4 layers) over few pixels in all.  x's patches
// are gathered once into xc [P][Cx R S] (a few MB), and conv_wgrad_nhwc_k runs as a 1x1 conv over the P pixels
// (x = xc, Cx = Mw).  With one split (the wide layers: a CU round of tiles or more) the kernel writes the weight
// gradient itself (xc's columns in the weight's (ci, r, s) order; no slab, no transposing reduction — the widest
// layer's 134 MB slab and its pass); with several splits the columns are in the slab order
// (r, s, ci) of the other routes and the usual reduction follows.
static constexpr long WG_IM2COL_MAX_BYTES = 64L << 20;

static bool wgrad_gemm_plan(int N, int H, int W, int Cx, int Ho, int Wo, int Cyp, int R, int S, int stride, int pad,
                            int math, WgradPlan* out) {
  if (math != VST_MATH_BF16X6 || Cx % 8 || Cyp % 8 || Wo % 32 == 0) return false;
  if (Ho != (H + 2 * pad - R) / stride + 1 || Wo != (W + 2 * pad - S) / stride + 1) return false;
  const long P = (long)N * Ho * Wo, Mw = (long)Cx * R * S;
  if (P % 32 || P * Mw * 4 > WG_IM2COL_MAX_BYTES || P * Cyp * 4 >= 0x7fff0000L || Mw >= (1L << 30)) return false;
  const WgradPlan p = plan_wgrad(1, 1, (int)P, 1, (int)P, (int)Mw, Cyp, 1, 1, 1, math);
  if (!p.bfk || p.wpad || !bf_wgrad_nhwc_ok((int)p.tile, (int)P, (int)Mw, Cyp)) return false;
  *out = p;
  return true;
}

static size_t wgrad_gemm_xc_bytes(const WgradPlan& p, long P) {
  return ((size_t)P * p.Mw * sizeof(float) + 255) / 256 * 256;
}

// xc, then the slabs (unused when the one split goes straight into the weight, which the caller's weight layout
// decides — a reservation, not traffic)
static size_t wgrad_gemm_ws_bytes(const WgradPlan& p, long P, int Cyp) {
  const size_t slabs = p.nsplit == 1 ? 1 : (size_t)p.nsplit + ceil_div(p.nsplit, WG_GROUP);
  return wgrad_gemm_xc_bytes(p, P) + slabs * p.Mw * Cyp * sizeof(float);
}

// xc[p][m] for output pixel p = (n, ho, wo) and column m = (ci, r, s) (cmajor) or (r, s, ci): x at the tap's input
// pixel (zero / reflect padding).  One thread per output float: the writes coalesce, the reads gather from an
// activation of a few MB.
__global__ __launch_bounds__(256) void wgrad_im2col_k(const float* __restrict__ x, float* __restrict__ xc, long total,
                                                      int Mw, int H, int W, int Cx, int Ho, int Wo, int R, int S,
                                                      int st, int pad, int reflect, int cmajor) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const long p = i / Mw;
  const int m = (int)(i - p * Mw), RS = R * S;
  int ci, rs;
  if (cmajor) {
    ci = m / RS;
    rs = m - ci * RS;
  } else {
    rs = m / Cx;
    ci = m - rs * Cx;
  }
  const int r = rs / S, sx = rs - r * S, hw = Ho * Wo;
  const int n = (int)(p / hw), rem = (int)(p - (long)n * hw), ho = rem / Wo, wo = rem - ho * Wo;
  int hi = ho * st + r - pad, wi = wo * st + sx - pad;
  if (reflect) {
    hi = reflect_idx(hi, H);
    wi = reflect_idx(wi, W);
  }
  xc[i] = ((unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W) ? x[(((long)n * H + hi) * W + wi) * Cx + ci] : 0.f;
}

static int wgrad_gemm_impl(const WgradPlan& p, const float* x, const float* dy, float* dw, float* ws, size_t ws_bytes,
                           int N, int H, int W, int Cx, int Ho, int Wo, int Cyp, int R, int S, int stride, int pad,
                           int pad_mode, int Co, int Ci, long so, long si, int accumulate, hipStream_t s) {
  const long P = (long)N * Ho * Wo;
  VST_REQUIRE(ws_bytes >= wgrad_gemm_ws_bytes(p, P, Cyp), "conv2d_wgrad_nhwc_f32: workspace too small (%zu bytes)",
              ws_bytes);
  // one split into the weight itself needs its layout to be xc's columns: dw [Co][Cx][R][S] contiguous
  const bool direct = p.nsplit == 1 && Ci == Cx && si == (long)R * S && so == (long)p.Mw;
  float* xc = ws;
  const long total = P * p.Mw;
  hipLaunchKernelGGL(wgrad_im2col_k, dim3((unsigned)ceil_div(total, 256)), dim3(256), 0, s, x, xc, total, p.Mw, H, W,
                     Cx, Ho, Wo, R, S, stride, pad, pad_mode == VST_PAD_REFLECT ? 1 : 0, direct ? 1 : 0);
  int rc = check_launch("conv2d_wgrad_im2col");
  if (rc) return rc;
  float* sl = ws + wgrad_gemm_xc_bytes(p, P) / sizeof(float);
  bf_wgrad_nhwc_launch(xc, dy, P * Cyp, true, direct ? nullptr : sl, 1, 1, (int)P, p.Mw, 1, (int)P, Cyp, 1, 0, 1, 0,
                       p.Mw, p.chunk, p.nsplit, (int)p.tile, s, direct ? dw : nullptr, Co, accumulate);
  rc = check_launch("conv2d_wgrad_nhwc_gemm");
  if (rc || direct) return rc;
  const long slab = (long)p.Mw * Cyp;
  const float* red = sl;
  int nred = p.nsplit;
  if (wgrad_two_level(p, Cyp, Ci, R * S, Co)) {
    float* l2 = sl + (long)p.nsplit * slab;
    nred = ceil_div(p.nsplit, WG_GROUP);
    hipLaunchKernelGGL(slab_group_sum_k, dim3(ceil_div(slab / 4, 256), nred), dim3(256), 0, s, sl, l2, slab / 4,
                       p.nsplit, WG_GROUP);
    red = l2;
  }
  if (nred > 2)
    hipLaunchKernelGGL(wgrad_reduce_store_k<1>, dim3(ceil_div(Ci * R * S, 16), ceil_div(Co, 64)), dim3(256), 0, s,
                       red, dw, Cx, Cyp, R * S, Co, Ci, so, si, accumulate, nred, slab);
  else
    hipLaunchKernelGGL(wgrad_reduce_store_k<2>, dim3(ceil_div(Ci * R * S, 32), ceil_div(Co, 64)), dim3(256), 0, s,
                       red, dw, Cx, Cyp, R * S, Co, Ci, so, si, accumulate, nred, slab);
  return check_launch("conv2d_wgrad_nhwc_gemm_reduce");
}

extern "C" int vst_conv2d_wgrad_nhwc_f32_ok(int N, int H, int W, int Cx, int Ho, int Wo, int Cyp, int R, int S,
                                            int stride, int pad, int math) {
  WgradPlan p;
  return (wgrad_nhwc_plan(N, H, W, Cx, Ho, Wo, Cyp, R, S, stride, pad, math, &p) ||
          wgrad_gemm_plan(N, H, W, Cx, Ho, Wo, Cyp, R, S, stride, pad, math, &p)) ? 1 : 0;
}

extern "C" size_t vst_conv2d_wgrad_nhwc_f32_ws_bytes(int N, int H, int W, int Cx, int Ho, int Wo, int Cyp, int R,
                                                     int S, int stride, int pad, int math) {
  WgradPlan p;
  if (wgrad_nhwc_plan(N, H, W, Cx, Ho, Wo, Cyp, R, S, stride, pad, math, &p))
    return vst_conv2d_wgrad_nhwc_ws_bytes(N, H, W, Cx, Ho, Wo, Cyp, R, S, stride, pad, math);
  if (wgrad_gemm_plan(N, H, W, Cx, Ho, Wo, Cyp, R, S, stride, pad, math, &p))
    return wgrad_gemm_ws_bytes(p, (long)N * Ho * Wo, Cyp);
  return 0;
}

// ... with dy fp32 NHWC [N][Ho][Wo][Cyp] itself (split in the kernel's registers like x): no operand image at all
// (shapes with Wo % 32 != 0 and few pixels: the im2col form above)
extern "C" int vst_conv2d_wgrad_nhwc_f32(const float* x, const float* dy, float* dw, float* ws, size_t ws_bytes, int N,
                                         int H, int W, int Cx, int Ho, int Wo, int Cyp, int R, int S, int stride,
                                         int pad, int pad_mode, int Co, int Ci, long so, long si, int accumulate,
                                         int math, void* stream) {
  WgradPlan p;
  if (!wgrad_nhwc_plan(N, H, W, Cx, Ho, Wo, Cyp, R, S, stride, pad, math, &p) &&
      wgrad_gemm_plan(N, H, W, Cx, Ho, Wo, Cyp, R, S, stride, pad, math, &p)) {
    VST_REQUIRE(x && dy && dw && ws, "conv2d_wgrad_nhwc_f32: null pointer");
    VST_REQUIRE(Co <= Cyp && Ci <= Cx && pad >= 0 && (pad_mode == VST_PAD_ZERO || (pad < H && pad < W)),
                "conv2d_wgrad_nhwc_f32: bad args");
    return wgrad_gemm_impl(p, x, dy, dw, ws, ws_bytes, N, H, W, Cx, Ho, Wo, Cyp, R, S, stride, pad, pad_mode, Co, Ci,
                           so, si, accumulate, (hipStream_t)stream);
  }
  return wgrad_nhwc_impl(x, dy, true, dw, ws, ws_bytes, N, H, W, Cx, Ho, Wo, Cyp, R, S, stride, pad, pad_mode, Co, Ci,
                         so, si, accumulate, math, stream);
}

extern "C" int vst_conv2d_wgrad_bias(const float* x, const float* dy, float* dw, float* db, float* ws, size_t ws_bytes,
                                     int N, int H, int W, int Cx, int Ho, int Wo, int Cyp, int R, int S, int stride,
                                     int pad, int pad_mode, int Co, int Ci, long so, long si, int accumulate, int math,
                                     void* stream) {
  (void)math;
  VST_REQUIRE(x && dy && dw && db && ws && N > 0 && H > 0 && W > 0 && Ho > 0 && Wo > 0 && R > 0 && S > 0 &&
                  stride > 0 && pad >= 0 && Co >= 1 && Co <= Cyp && Ci >= 1 && Ci <= Cx,
              "conv2d_wgrad_bias: bad args");
  const int refl = pad_mode == VST_PAD_REFLECT;
  hipStream_t s = (hipStream_t)stream;
  if (g_img_wgrad && img_wgrad_ok(Cx, Cyp, R, S, stride, refl, Ci, Wo) &&
      ws_bytes >= img_wgrad_ws_floats(N, Ho, Wo) * sizeof(float))
    return img_wgrad_launch(x, dy, dw, db, ws, N, H, W, Ho, Wo, Cyp, R, S, stride, pad, Co, Ci, so, si, accumulate, s);
  if (Cyp == 4 && Co == 1 && g_head && head_ok(Cx, R, S, stride, refl, Wo) &&
      ws_bytes >= head_wgrad_ws_floats(N, H, Cx, R, S) * sizeof(float))
    return head_wgrad_launch(x, dy, dw, ws, N, H, W, Cx, Ci, Ho, Wo, R, S, pad, si, accumulate, s, db);
  ::vst::set_error("conv2d_wgrad_bias: no fused route for this shape (use vst_conv2d_wgrad + vst_channel_sum)");
  return VST_EUNSUPPORTED;
}

extern "C" int vst_reflect_fold(const float* dxp, const float* addend, float* dx, int N, int H,
                                int W, int C, int p, void* stream) {
  VST_REQUIRE(dxp && dx && C % 4 == 0 && p >= 0 && p < H && p < W, "reflect_fold: bad args");
  const long total = (long)N * H * W * (C / 4);
  hipLaunchKernelGGL(reflect_fold_k, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream,
                     dxp, addend, dx, N, H, W, C / 4, p);
  return check_launch("reflect_fold");
}
