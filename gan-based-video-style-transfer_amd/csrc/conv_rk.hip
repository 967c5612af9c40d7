// Forward and transposed (data-gradient) implicit-GEMM convolutions on gfx950 fp32 MFMA with a
// row-major [row][k] LDS image — the production path behind vst_conv2d_fwd / vst_conv2d_tfwd.
//
// Why this layout: v_mfma_f32_32x32x2_f32 takes ONE f32 per lane per operand (lane l supplies
// A[l&31][k = l>>5]).  The reduction order inside a K group is free, so within each 8-deep group
// lane-half kh feeds k = 4*kh + t to MFMA t (t = 0..3).  A lane's four operands for four MFMAs are
// then 4 consecutive floats of its row: one ds_read_b128 replaces four ds_read_b32, and both
// operand tiles are written with ds_write_b128 straight from coalesced 128-byte global rows
// (8 lanes x float4 per pixel row / weight row) — no transposing scalar LDS writes.  Row stride is
// BK + 4 floats (144 B at BK = 32): the 16-lane groups of ds_read_b128 hit 16 distinct 16-byte bank slots.
//
//   conv_fprop_rk_k : y = act(conv(x, w) + bias)   m = output pixel, n = out channel,
//                     k = (r, s, ci); B operand = VST_PACK_OK pack [Co][R][S][Ci]
//   conv_tconv_rk_k : transposed conv / data gradient, gathered per output-parity class
//                     (blockIdx.z), stride-specialised (ST), reflect-pad gradient folded into the
//                     gather (mirrored rows/columns), residual addend fused in the epilogue;
//                     B operand = VST_PACK_IK pack [Ci][R][S][Co]
// Both keep the next K-step's global loads interleaved into the current MFMA stream and the
// double-buffered LDS stage with one barrier per 32-deep K-step.
#include "common.h"

#ifndef WGRAD_XCD
#define WGRAD_XCD 1
#endif

namespace vst {
namespace rk {

constexpr int NOPOS = -(1 << 20);
#ifndef VST_RK_PROBE
#define VST_RK_PROBE 0  // developer probes: 1 = fprop without global loads, 2 = without MFMAs
#endif
#ifndef VST_RK_LG
#define VST_RK_LG 4   // the next stage's global loads are spread over the first LG MFMA groups
#endif

template <int BM, int BN, int WM, int WN, int BK_, int MATH_ = VST_MATH_F32>
struct Tile {
  static constexpr int MATH = MATH_;
  static constexpr bool X3 = MATH != VST_MATH_F32;    // bf16 split-operand image (x3 or x6)
  static constexpr int NP = MATH == VST_MATH_BF16X6 ? 3 : 2;  // bf16 planes per operand
  static constexpr int BM_ = BM, BN_ = BN, WM_ = WM, WN_ = WN;
  static constexpr int BK = BK_;
  static constexpr int LDK = BK + 4;             // fp32 image: row stride in floats
  static constexpr int LDH = BK + 8;             // bf16x3 image: row stride in bf16 elements
  static constexpr int KQ = BK / 4;              // lanes (float4s) per staged row
  static constexpr int NW = (BM / WM) * (BN / WN);
  static constexpr int NT = 64 * NW;
  static constexpr int WAVES_N = BN / WN;
  static constexpr int MI = WM / 32;
  static constexpr int NI = WN / 32;
  // stage sizes in floats; a bf16 split image holds NP planes [rows][LDH] (hi, (mid,) lo)
  static constexpr int A_ELEMS = X3 ? BM * LDH * NP / 2 : BM * LDK;
  static constexpr int B_ELEMS = X3 ? BN * LDH * NP / 2 : BN * LDK;
  static constexpr int STAGE = A_ELEMS + B_ELEMS;
  static constexpr int ROWS_PER_PASS = NT / KQ;  // KQ lanes x float4 cover one BK-deep row
  static constexpr int A_LD = BM / ROWS_PER_PASS;
  static constexpr int B_LD = BN / ROWS_PER_PASS;
  // Staging row of thread t.  bf16 images (row stride LDH = 40 bf16 = 20 banks) with 8 lanes per
  // row: a 32-lane half-wave writes 4 rows, and rows r, r+4, r+8, r+12 start on banks 0/16/32/48
  // (+ const) — the 4 x 16-bank row segments tile the 64 banks without overlap, where 4
  // consecutive rows (banks 0/20/40/60) collide.  Bijective on [0, RP); loads follow the rows.
  static __device__ __forceinline__ int row_of(int t) {
    const int q = t / KQ;
    if constexpr (X3 && KQ == 8) {
      const int h = q >> 2, e = q & 3;
      return ((h >> 2) << 4) + (h & 3) + 4 * e;
    } else {
      return q;
    }
  }
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  static_assert(!X3 || BK % 16 == 0, "bf16 k groups are 16 deep");
  static_assert(BM % ROWS_PER_PASS == 0 && BN % ROWS_PER_PASS == 0, "row coverage");
};

__device__ __forceinline__ float comp(const float4& v, int t) {
  return t == 0 ? v.x : (t == 1 ? v.y : (t == 2 ? v.z : v.w));
}

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

// Two fp32 -> two bf16 (RNE, v_cvt_pk_bf16_f32), packed low = a, high = b.
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  const f32x2_t v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

// bf16 operand split of four fp32 values into NP planes.  NP = 2: hi = bf16(v), lo = bf16(v - hi);
// v - hi is exact in fp32, so hi + lo carries 16 significant bits (|v - hi - lo| <= 2^-17 |v|).
// NP = 3 splits the remainder once more (mid, lo): hi + mid + lo carries all 24 bits of v.
__device__ __forceinline__ float bf16_lo_f(uint32_t p) { return __uint_as_float(p << 16); }
__device__ __forceinline__ float bf16_hi_f(uint32_t p) { return __uint_as_float(p & 0xffff0000u); }

template <int NP>
__device__ __forceinline__ void split4(const float4& v, uint2 (&o)[NP]) {
  float r0 = v.x, r1 = v.y, r2 = v.z, r3 = v.w;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    o[p].x = pack_bf16x2(r0, r1);
    o[p].y = pack_bf16x2(r2, r3);
    if (p + 1 < NP) {
      r0 -= bf16_lo_f(o[p].x);
      r1 -= bf16_hi_f(o[p].x);
      r2 -= bf16_lo_f(o[p].y);
      r3 -= bf16_hi_f(o[p].y);
    }
  }
}

// fp32 image: v_mfma_f32_32x32x2_f32, 4 MFMAs per 8-deep k group and fragment pair.
template <class T, class Hook>
__device__ __forceinline__ void mma_stage_f32(const float* __restrict__ As, const float* __restrict__ Bs,
                                              f32x16 (&acc)[T::MI][T::NI], int wm0, int wn0, int lane,
                                              Hook hook) {
  constexpr int LDK = T::LDK, BK = T::BK;
  const int kh = lane >> 5, li = lane & 31;
  const float* pa = As + (wm0 + li) * LDK + 4 * kh;
  const float* pb = Bs + (wn0 + li) * LDK + 4 * kh;
  float4 fa[2][T::MI], fb[2][T::NI];
#pragma unroll
  for (int i = 0; i < T::MI; ++i) fa[0][i] = *reinterpret_cast<const float4*>(pa + 32 * i * LDK);
#pragma unroll
  for (int j = 0; j < T::NI; ++j) fb[0][j] = *reinterpret_cast<const float4*>(pb + 32 * j * LDK);
#pragma unroll
  for (int g = 0; g < BK / 8; ++g) {
    const int cur = g & 1, nxt = cur ^ 1;
    hook(g);
    if (g + 1 < BK / 8) {
#pragma unroll
      for (int i = 0; i < T::MI; ++i)
        fa[nxt][i] = *reinterpret_cast<const float4*>(pa + 32 * i * LDK + 8 * (g + 1));
#pragma unroll
      for (int j = 0; j < T::NI; ++j)
        fb[nxt][j] = *reinterpret_cast<const float4*>(pb + 32 * j * LDK + 8 * (g + 1));
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < T::MI; ++i)
#pragma unroll
        for (int j = 0; j < T::NI; ++j)
#if VST_RK_PROBE == 2  // developer probe: LDS + global traffic without the MFMAs
          acc[i][j][t] += comp(fa[cur][i], t) * comp(fb[cur][j], t);
#else
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(comp(fa[cur][i], t), comp(fb[cur][j], t),
                                                           acc[i][j], 0, 0, 0);
#endif
  }
}

// bf16 split image: per 16-deep k group, lane (li, kh) reads 8 consecutive k of its row
// (k = 16g + 8kh + 0..7, the v_mfma_f32_32x32x16_bf16 A/B operand map) from every plane with one
// ds_read_b128 each, then accumulates the split products in fp32, smallest terms first:
//   x3 (NP = 2): lo*hi + hi*lo + hi*hi                (dropped lo*lo <= 2^-16 |a*b|)
//   x6 (NP = 3): lo*hi + hi*lo + mid*mid + mid*hi + hi*mid + hi*hi   (dropped terms <= 2^-24 |a*b|)
// Row stride BK + 8 bf16 = 16-B slots that put the 16 lanes of every ds_read_b128 group on 16
// distinct slots.
template <class T, class Hook>
__device__ __forceinline__ void mma_stage_bf16(const float* __restrict__ As, const float* __restrict__ Bs,
                                               f32x16 (&acc)[T::MI][T::NI], int wm0, int wn0, int lane,
                                               Hook hook) {
  constexpr int LDH = T::LDH, BK = T::BK, NP = T::NP;
  constexpr int PA = T::BM_ * LDH, PB = T::BN_ * LDH;  // plane sizes (bf16)
  const int kh = lane >> 5, li = lane & 31;
  const __bf16* pa = reinterpret_cast<const __bf16*>(As) + (wm0 + li) * LDH + 8 * kh;
  const __bf16* pb = reinterpret_cast<const __bf16*>(Bs) + (wn0 + li) * LDH + 8 * kh;
  bf16x8_t fa[2][NP][T::MI], fb[2][NP][T::NI];
  auto rd = [&](int buf, int o) {
#pragma unroll
    for (int p = 0; p < NP; ++p) {
#pragma unroll
      for (int i = 0; i < T::MI; ++i)
        fa[buf][p][i] = *reinterpret_cast<const bf16x8_t*>(pa + p * PA + 32 * i * LDH + o);
#pragma unroll
      for (int j = 0; j < T::NI; ++j)
        fb[buf][p][j] = *reinterpret_cast<const bf16x8_t*>(pb + p * PB + 32 * j * LDH + o);
    }
  };
  rd(0, 0);
#pragma unroll
  for (int g = 0; g < BK / 16; ++g) {
    const int cur = g & 1;
    hook(g);
    if (g + 1 < BK / 16) rd(cur ^ 1, 16 * (g + 1));
#pragma unroll
    for (int i = 0; i < T::MI; ++i)
#pragma unroll
      for (int j = 0; j < T::NI; ++j) {
#define VST_MF(pA, pB) \
  acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[cur][pA][i], fb[cur][pB][j], acc[i][j], 0, 0, 0)
        if constexpr (NP == 3) {
          VST_MF(2, 0); VST_MF(0, 2); VST_MF(1, 1); VST_MF(1, 0); VST_MF(0, 1); VST_MF(0, 0);
        } else {
          VST_MF(1, 0); VST_MF(0, 1); VST_MF(0, 0);
        }
#undef VST_MF
      }
  }
}

// Write one thread's staged float4s (A rows rb + RP*j, B rows likewise, k = 4*kq..4*kq+3) into a
// stage image: float4 rows for fp32, split hi/lo bf16 quads (ds_write_b64 each) for bf16x3.
template <class T, int A_LD, int B_LD>
__device__ __forceinline__ void store_stage(float* As, const float4 (&ra)[A_LD], const float4 (&rbv)[B_LD],
                                            int rb, int kq) {
  constexpr int RP = T::ROWS_PER_PASS;
  float* Bs = As + T::A_ELEMS;
  if constexpr (T::X3) {
    constexpr int LDH = T::LDH, NP = T::NP;
    __bf16* ah = reinterpret_cast<__bf16*>(As);
    __bf16* bh = reinterpret_cast<__bf16*>(Bs);
#pragma unroll
    for (int j = 0; j < A_LD; ++j) {
      uint2 s[NP];
      split4<NP>(ra[j], s);
      const int o = (rb + RP * j) * LDH + 4 * kq;
#pragma unroll
      for (int p = 0; p < NP; ++p) *reinterpret_cast<uint2*>(ah + p * T::BM_ * LDH + o) = s[p];
    }
#pragma unroll
    for (int j = 0; j < B_LD; ++j) {
      uint2 s[NP];
      split4<NP>(rbv[j], s);
      const int o = (rb + RP * j) * LDH + 4 * kq;
#pragma unroll
      for (int p = 0; p < NP; ++p) *reinterpret_cast<uint2*>(bh + p * T::BN_ * LDH + o) = s[p];
    }
  } else {
    constexpr int LDK = T::LDK;
#pragma unroll
    for (int j = 0; j < A_LD; ++j) *reinterpret_cast<float4*>(As + (rb + RP * j) * LDK + 4 * kq) = ra[j];
#pragma unroll
    for (int j = 0; j < B_LD; ++j) *reinterpret_cast<float4*>(Bs + (rb + RP * j) * LDK + 4 * kq) = rbv[j];
  }
}

template <class T, int NLOAD, class LoadOne, class Adv, class Store>
__device__ __forceinline__ void main_loop(float* smem, int nk, f32x16 (&acc)[T::MI][T::NI],
                                          LoadOne load_one, Adv adv, Store store) {
  constexpr int BK = T::BK;
  constexpr int NG = T::X3 ? BK / 16 : BK / 8;  // k groups per stage (hook slots)
  constexpr int LG = VST_RK_LG < NG ? VST_RK_LG : NG;
  constexpr int PER = (NLOAD + LG - 1) / LG;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm0 = (wave / T::WAVES_N) * T::WM_, wn0 = (wave % T::WAVES_N) * T::WN_;
  if (nk > 0) {
#pragma unroll
    for (int i = 0; i < NLOAD; ++i) load_one(i, 0);
    store(smem);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    float* cur = smem + (kt & 1) * T::STAGE;
    const bool next = kt + 1 < nk;
    if (next) adv();
    const int k0n = (kt + 1) * BK;
    auto hook = [&](int g) {
      if (next) {
#pragma unroll
        for (int u = 0; u < PER; ++u)
          if (PER * g + u < NLOAD) load_one(PER * g + u, k0n);
      }
    };
    if constexpr (T::X3) mma_stage_bf16<T>(cur, cur + T::A_ELEMS, acc, wm0, wn0, lane, hook);
    else mma_stage_f32<T>(cur, cur + T::A_ELEMS, acc, wm0, wn0, lane, hook);
    if (next) store(smem + ((kt + 1) & 1) * T::STAGE);
    __syncthreads();
  }
}

__device__ __forceinline__ int remap_mtile(int bx, int nx) {
  if ((nx & 7) != 0) return bx;
  return (bx & 7) * (nx >> 3) + (bx >> 3);
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

// ------------------------------------------------------------------------------------------ fprop
template <int BM, int BN, int WM, int WN, int BK, int MATH>
__global__ __launch_bounds__((Tile<BM, BN, WM, WN, BK, MATH>::NT), 2) void conv_fprop_rk_k(
    const float* __restrict__ x, const float* __restrict__ wp, const float* __restrict__ bias,
    float* __restrict__ y, int H, int W, int C, int Ho, int Wo, int Cop, int S, int st, int padh,
    int padw, int reflect, int act, float slope, int M, int Ktot) {
  using T = Tile<BM, BN, WM, WN, BK, MATH>;
  constexpr int NT = T::NT, A_LD = T::A_LD, B_LD = T::B_LD, RP = T::ROWS_PER_PASS;
  __shared__ __attribute__((aligned(16))) float smem[2 * T::STAGE];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int mt = remap_mtile(blockIdx.x, gridDim.x);
  const int m0 = mt * BM, n0 = blockIdx.y * BN;
  const int kq = t % T::KQ, rb = T::row_of(t);

  // k state (one per thread: every row this thread stages uses the same k position)
  int kc = (4 * kq) % C, ks, kr;
  {
    const int rs = (4 * kq) / C;
    kr = rs / S;
    ks = rs - kr * S;
  }
  // A rows: output pixels m0 + rb + RP*j
  int hb[A_LD], wb[A_LD];
  const float* xb[A_LD];
  bool mv[A_LD];
#pragma unroll
  for (int j = 0; j < A_LD; ++j) {
    const int m = m0 + rb + RP * j;
    mv[j] = m < M;
    const int mm = mv[j] ? m : 0;
    const int hw = Ho * Wo;
    const int n = mm / hw, rem = mm - n * hw, ho = rem / Wo, wo = rem - ho * Wo;
    hb[j] = ho * st - padh;
    wb[j] = wo * st - padw;
    xb[j] = x + (long)n * H * W * C;
  }
  const float* wrow[B_LD];
  bool nv[B_LD];
#pragma unroll
  for (int j = 0; j < B_LD; ++j) {
    const int n = n0 + rb + RP * j;
    nv[j] = n < Cop;
    wrow[j] = wp + (long)(nv[j] ? n : 0) * Ktot;
  }

  float4 ra[A_LD], rbv[B_LD];
  int kcur = 4 * kq;  // absolute k of this thread's float4 in the stage being loaded
  auto load_one = [&](int i, int) {
#if VST_RK_PROBE == 1
    if (i < A_LD) ra[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    else rbv[i - A_LD] = make_float4(0.f, 0.f, 0.f, 0.f);
    return;
#endif
    if (i < A_LD) {
      const int j = i;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (mv[j] && kcur < Ktot) {
        int hi = hb[j] + kr, wi = wb[j] + ks;
        bool ok = true;
        if (reflect) {
          hi = reflect_idx(hi, H);
          wi = reflect_idx(wi, W);
        } else {
          ok = (unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W;
        }
        if (ok) v = *reinterpret_cast<const float4*>(xb[j] + ((long)hi * W + wi) * C + kc);
      }
      ra[j] = v;
    } else {
      const int j = i - A_LD;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (nv[j] && kcur < Ktot) v = *reinterpret_cast<const float4*>(wrow[j] + kcur);
      rbv[j] = v;
    }
  };
  auto adv = [&]() {
    kcur += BK;
    kc += BK;
    while (kc >= C) {
      kc -= C;
      if (++ks == S) { ks = 0; ++kr; }
    }
  };
  auto store = [&](float* As) { store_stage<T, A_LD, B_LD>(As, ra, rbv, rb, kq); };

  f32x16 acc[T::MI][T::NI];
  zero_acc(acc);
  main_loop<T, A_LD + B_LD>(smem, (Ktot + BK - 1) / BK, acc, load_one, adv, store);
  (void)NT;

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
template <int BM, int BN, int WM, int WN, int BK, int ST, int MATH>
__global__ __launch_bounds__((Tile<BM, BN, WM, WN, BK, MATH>::NT), 2) void conv_tconv_rk_k(
    const float* __restrict__ in, const float* __restrict__ wp, const float* __restrict__ bias,
    const float* __restrict__ addend, float* __restrict__ out, int Hi, int Wi, int Cy, int Ho,
    int Wo, int Cx, int R, int S, int st_rt, int pad, int reflect, int act, float slope, int Nimg) {
  using T = Tile<BM, BN, WM, WN, BK, MATH>;
  constexpr int A_LD = T::A_LD, B_LD = T::B_LD, RP = T::ROWS_PER_PASS;
  __shared__ __attribute__((aligned(16))) float smem[2 * T::STAGE];
  const int st = ST > 0 ? ST : st_rt;
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
  const int kq = t % T::KQ, rb = T::row_of(t);
  int kc = ns > 0 ? (4 * kq) % Cy : 0, kis, kir;
  {
    const int tp = Cy > 0 ? (4 * kq) / Cy : 0;
    kir = ns > 0 ? tp / ns : 0;
    kis = tp - kir * ns;
  }
  int hp[A_LD], wq[A_LD], hm[A_LD], wm[A_LD];
  const float* ib[A_LD];
  bool mv[A_LD];
#pragma unroll
  for (int j = 0; j < A_LD; ++j) {
    const int m = m0 + rb + RP * j;
    mv[j] = m < M;
    const int mm = mv[j] ? m : 0;
    const int hw = Hc * Wc;
    const int n = mm / hw, rem = mm - n * hw, hh = rem / Wc, ww = rem - hh * Wc;
    const int h = ca + st * hh, w = cb + st * ww;
    hp[j] = h + pad;
    wq[j] = w + pad;
    hm[j] = NOPOS;
    wm[j] = NOPOS;
    if (reflect) {
      if (h >= 1 && h <= pad) hm[j] = pad - h;
      else if (h >= Ho - 1 - pad && h <= Ho - 2) hm[j] = 2 * Ho - 2 - h + pad;
      if (w >= 1 && w <= pad) wm[j] = pad - w;
      else if (w >= Wo - 1 - pad && w <= Wo - 2) wm[j] = 2 * Wo - 2 - w + pad;
    }
    ib[j] = in + (long)n * Hi * Wi * Cy;
  }
  const long wstride = (long)R * S * Cy;
  const float* wrow[B_LD];
  bool nv[B_LD];
#pragma unroll
  for (int j = 0; j < B_LD; ++j) {
    const int n = n0 + rb + RP * j;
    nv[j] = n < Cx;
    wrow[j] = wp + (long)(nv[j] ? n : 0) * wstride;
  }

  float4 ra[A_LD], rbv[B_LD];
  int kcur = 4 * kq;
  auto gather1 = [&](const float* base, int hpos, int wpos, int r, int s, float4& v) {
    const int dh = hpos - r, dw = wpos - s;
    if (dh >= 0 && dw >= 0) {
      const int ho = dh / st, wo = dw / st;
      if (ho < Hi && wo < Wi) add_f4(v, *reinterpret_cast<const float4*>(base + ((long)ho * Wi + wo) * Cy + kc));
    }
  };
  auto load_one = [&](int i, int) {
    const int r = r0 + st * kir, s = s0 + st * kis;
    if (i < A_LD) {
      const int j = i;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (mv[j] && kcur < Ktot) {
        gather1(ib[j], hp[j], wq[j], r, s, v);
        if (hm[j] != NOPOS) gather1(ib[j], hm[j], wq[j], r, s, v);
        if (wm[j] != NOPOS) {
          gather1(ib[j], hp[j], wm[j], r, s, v);
          if (hm[j] != NOPOS) gather1(ib[j], hm[j], wm[j], r, s, v);
        }
      }
      ra[j] = v;
    } else {
      const int j = i - A_LD;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (nv[j] && kcur < Ktot)
        v = *reinterpret_cast<const float4*>(wrow[j] + (long)(r * S + s) * Cy + kc);
      rbv[j] = v;
    }
  };
  auto adv = [&]() {
    kcur += BK;
    kc += BK;
    while (kc >= Cy) {
      kc -= Cy;
      if (++kis == ns) { kis = 0; ++kir; }
    }
  };
  auto store = [&](float* As) { store_stage<T, A_LD, B_LD>(As, ra, rbv, rb, kq); };

  f32x16 acc[T::MI][T::NI];
  zero_acc(acc);
  main_loop<T, A_LD + B_LD>(smem, (Ktot + BK - 1) / BK, acc, load_one, adv, store);

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

// ------------------------------------------------------------------ weight gradient, stride 1
// dW[m = (r, s, ci)][co] = sum_p X[shift_rs(p)][ci] * dY[p][co] with both operands read from
// channel-major copies (xt = [Cx][N][Hp][Wp], the input with its reflect / zero border already
// applied, made by nhwc_to_cp_pad_k; dyt = [Cyp][N*Ho*Wo], made by nhwc_to_cp_k), so every GEMM
// row is contiguous along the reduction (pixel) axis and stages into the row-major [row][k] LDS
// image with ds_write_b128 exactly like the forward kernel.  For stride 1 the 4 pixels of a
// float4 are 4 consecutive padded columns: one (unaligned) 16-byte load, no border branches.
// Stride 2 reads the same way from a copy whose padded rows are split into even / odd columns.
// The split-K chunk index comes from the XCD-aware 1-D grid; partial tiles land in
// slab[z][m][Cyp] (summed and transposed into dw by conv.hip).
template <int BM, int BN, int WM, int WN, int BK, int MATH>
__global__ __launch_bounds__((Tile<BM, BN, WM, WN, BK, MATH>::NT), 2) void conv_wgrad_rk_k(
    const float* __restrict__ xt, const float* __restrict__ dyt, float* __restrict__ slab, int H,
    int W, int Cx, int Ho, int Wo, int Cyp, int S, int pad, int st, int Mw, int P, int chunk,
    long ldx, long ldy) {
  using T = Tile<BM, BN, WM, WN, BK, MATH>;
  constexpr int A_LD = T::A_LD, B_LD = T::B_LD, RP = T::ROWS_PER_PASS;
  constexpr bool PACKED = MATH == VST_MATH_BF16X3;  // xt / dyt hold (hi << 16 | lo) bf16 words
  typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
  __shared__ __attribute__((aligned(16))) float smem[2 * T::STAGE];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
#if WGRAD_XCD
  // 1-D grid, XCD-aware: consecutive workgroup ids go to consecutive XCDs, so XCD x takes the
  // contiguous range [x*T/8, (x+1)*T/8) of (split-major, then n, then m) tiles — every tile of a
  // split-K chunk runs on one XCD and its x / dy chunk rows stay in that XCD's L2 (the 3-D grid
  // spread each chunk over all eight L2s: ~11x the algorithmic HBM reads).
  const int Mt = (Mw + BM - 1) / BM, Nt = (Cyp + BN - 1) / BN, Zt = (P + chunk - 1) / chunk;
  int mx, ny, zz;
  {
    const int tt = xcd_tile(blockIdx.x, Mt * Nt * Zt);
    zz = tt / (Mt * Nt);
    const int rem = tt - zz * Mt * Nt;
    ny = rem / Mt;
    mx = rem - ny * Mt;
  }
  const int m0 = mx * BM, n0 = ny * BN;
  const int pbeg = zz * chunk;
#else
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int pbeg = blockIdx.z * chunk;
#endif
  const int pend = min(P, pbeg + chunk);
  const int kq = t % T::KQ, rb = T::row_of(t);

  // A rows: tap (r, s) of input channel ci over the PADDED channel-major image xt =
  // [Cx][N][Hp][Wp] (nhwc_to_cp_pad_k applied the reflect / zero border), so the 4 pixels of a
  // float4 are 4 consecutive words of one padded row — always in bounds, one 16-byte load.
  const int Hp = H + 2 * pad, Wp = W + 2 * pad;
  const float* xrow[A_LD];
  bool mv[A_LD];
#pragma unroll
  for (int j = 0; j < A_LD; ++j) {
    const int m = m0 + rb + RP * j;
    mv[j] = m < Mw;
    const int mm = mv[j] ? m : 0;
    const int tap = mm / Cx, ci = mm - tap * Cx;
    const int r = tap / S, s_ = tap - r * S;
    // stride 2: padded rows are stored column-phase split ([even cols][odd cols], Wp / 2 each),
    // so tap s of 4 consecutive output columns is 4 consecutive words of phase s & 1
    xrow[j] = xt + (long)ci * ldx + r * Wp + (st == 1 ? s_ : (s_ & 1) * (Wp >> 1) + (s_ >> 1));
  }
  const float* dyrow[B_LD];
  bool nv[B_LD];
#pragma unroll
  for (int j = 0; j < B_LD; ++j) {
    const int n = n0 + rb + RP * j;
    nv[j] = n < Cyp;
    dyrow[j] = dyt + (long)(nv[j] ? n : 0) * ldy;
  }
  // pixel state of this thread's float4 (shared by all its rows): output pixel kp = (pn, pho, pwo)
  // and its padded-image offset poff = (pn * Hp + pho) * Wp + pwo
  int kp = pbeg + 4 * kq, pho, pwo;
  long poff;
  {
    const int hw = Ho * Wo;
    const int pn = kp / hw;
    const int rem = kp - pn * hw;
    pho = rem / Wo;
    pwo = rem - pho * Wo;
    poff = ((long)pn * Hp + st * pho) * Wp + pwo;
  }
  float4 ra[A_LD], rbv[B_LD];
  auto load_one = [&](int i, int) {
    const bool live = kp < pend;
    if (i < A_LD) {
      const int j = i;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (mv[j] && live) {
        const f4u u = *reinterpret_cast<const f4u*>(xrow[j] + poff);
        v = make_float4(u.x, u.y, u.z, u.w);
      }
      ra[j] = v;
    } else {
      const int j = i - A_LD;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (nv[j] && live) v = *reinterpret_cast<const float4*>(dyrow[j] + kp);
      rbv[j] = v;
    }
  };
  auto adv = [&]() {
    kp += BK;
    pwo += BK;
    poff += BK;
    while (pwo >= Wo) {
      pwo -= Wo;
      poff += st * Wp - Wo;
      if (++pho == Ho) { pho = 0; poff += (long)(Hp - st * Ho) * Wp; }
    }
  };
  // bf16x3: the channel-major copies already hold each value as a (hi, lo) bf16 word pair
  // (nhwc_to_cp_k<true>), so a staged float4 is four packed words and the stage image takes
  // one byte permute per plane pair instead of the convert / subtract / convert split.
  auto store = [&](float* As) {
    if constexpr (PACKED) {
      constexpr int LDH = T::LDH;
      __bf16* ah = reinterpret_cast<__bf16*>(As);
      __bf16* bh = reinterpret_cast<__bf16*>(As + T::A_ELEMS);
      auto put = [&](__bf16* base, int plane, const float4& v, int o) {
        const uint32_t x0 = __float_as_uint(v.x), x1 = __float_as_uint(v.y);
        const uint32_t x2 = __float_as_uint(v.z), x3 = __float_as_uint(v.w);
        uint2 h, l;
        h.x = __builtin_amdgcn_perm(x1, x0, 0x07060302u);
        h.y = __builtin_amdgcn_perm(x3, x2, 0x07060302u);
        l.x = __builtin_amdgcn_perm(x1, x0, 0x05040100u);
        l.y = __builtin_amdgcn_perm(x3, x2, 0x05040100u);
        *reinterpret_cast<uint2*>(base + o) = h;
        *reinterpret_cast<uint2*>(base + plane + o) = l;
      };
#pragma unroll
      for (int j = 0; j < A_LD; ++j) put(ah, BM * LDH, ra[j], (rb + RP * j) * LDH + 4 * kq);
#pragma unroll
      for (int j = 0; j < B_LD; ++j) put(bh, BN * LDH, rbv[j], (rb + RP * j) * LDH + 4 * kq);
    } else {
      store_stage<T, A_LD, B_LD>(As, ra, rbv, rb, kq);
    }
  };

  f32x16 acc[T::MI][T::NI];
  zero_acc(acc);
  const int nk = pend > pbeg ? (pend - pbeg + BK - 1) / BK : 0;
  main_loop<T, A_LD + B_LD>(smem, nk, acc, load_one, adv, store);

  const int wm0 = (wave / T::WAVES_N) * WM, wn0 = (wave % T::WAVES_N) * WN;
#if WGRAD_XCD
  float* sl = slab + (long)zz * Mw * Cyp;
#else
  float* sl = slab + (long)blockIdx.z * Mw * Cyp;
#endif
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

// One fp32 value as its bf16x3 operand pair in one word: hi = bf16(v) in the high half,
// lo = bf16(v - hi) in the low half (the same RNE conversions as split4<2>).
__device__ __forceinline__ float split_word(float v) {
  const uint32_t h = pack_bf16x2(v, 0.f) & 0xffffu;
  const uint32_t l = pack_bf16x2(v - __uint_as_float(h << 16), 0.f) & 0xffffu;
  return __uint_as_float((h << 16) | l);
}

// NHWC [P][Cs] -> channel-major [Cs][ld] through a 64x64 LDS tile (float4 reads and writes);
// PACK stores every value as its split_word (the bf16x3 weight gradient's operand image).
template <bool PACK>
__global__ __launch_bounds__(256) void nhwc_to_cp_k(const float* __restrict__ x, float* __restrict__ y,
                                                    long P, int Cs, long ld) {
  __shared__ float tile[64][65];
  const long p0 = (long)blockIdx.x * 64;
  const int c0 = blockIdx.y * 64;
  const int t = threadIdx.x;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int idx = t + 256 * it, pr = idx >> 4, c4 = (idx & 15) * 4;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (p0 + pr < P && c0 + c4 < Cs) v = *reinterpret_cast<const float4*>(x + (p0 + pr) * Cs + c0 + c4);
    if (PACK) v = make_float4(split_word(v.x), split_word(v.y), split_word(v.z), split_word(v.w));
    tile[pr][c4] = v.x;
    tile[pr][c4 + 1] = v.y;
    tile[pr][c4 + 2] = v.z;
    tile[pr][c4 + 3] = v.w;
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int idx = t + 256 * it, cr = idx >> 4, p4 = (idx & 15) * 4;
    if (c0 + cr >= Cs || p0 + p4 >= P) continue;
    float* dst = y + (long)(c0 + cr) * ld + p0 + p4;
    if (p0 + p4 + 3 < P && (ld & 3) == 0) {
      *reinterpret_cast<float4*>(dst) =
          make_float4(tile[p4][cr], tile[p4 + 1][cr], tile[p4 + 2][cr], tile[p4 + 3][cr]);
    } else {  // ragged plane length (P % 4 != 0): element stores, never past the plane
      for (int e = 0; e < 4 && p0 + p4 + e < P; ++e) dst[e] = tile[p4 + e][cr];
    }
  }
}

// NHWC [N][H][W][Cs] -> padded channel-major [Cs][N][H+2p][W+2p] (reflect or zero border), the
// weight gradient's A-operand image; same 64x64 LDS tile walk as nhwc_to_cp_k over padded pixels.
// phase (stride 2, W + 2p even): each padded row stored as its even columns then its odd columns.
template <bool PACK>
__global__ __launch_bounds__(256) void nhwc_to_cp_pad_k(const float* __restrict__ x, float* __restrict__ y,
                                                        int N, int H, int W, int Cs, int pad, int reflect,
                                                        int phase, long ld, int extra) {
  __shared__ float tile[64][65];
  const int Hp = H + 2 * pad, Wp = W + 2 * pad + extra;  // extra: zero columns right of the border
  const long P = (long)N * Hp * Wp;
  const long p0 = (long)blockIdx.x * 64;
  const int c0 = blockIdx.y * 64;
  const int t = threadIdx.x;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int idx = t + 256 * it, pr = idx >> 4, c4 = (idx & 15) * 4;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    const long q = p0 + pr;
    if (q < P && c0 + c4 < Cs) {
      const int n = (int)(q / ((long)Hp * Wp));
      const int rem = (int)(q - (long)n * Hp * Wp);
      int h = rem / Wp - pad, w = rem % Wp;
      if (phase) {  // destination word e of a row holds padded column 2e (e < Wp/2) or 2(e - Wp/2) + 1
        const int wh = Wp >> 1;
        w = w < wh ? 2 * w : 2 * (w - wh) + 1;
      }
      w -= pad;
      bool ok = w < W + pad;  // the extra columns stay zero
      if (reflect) {
        h = reflect_idx(h, H);
        w = reflect_idx(w, W);
      } else {
        ok = (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
      }
      if (ok) v = *reinterpret_cast<const float4*>(x + (((long)n * H + h) * W + w) * Cs + c0 + c4);
    }
    if (PACK) v = make_float4(split_word(v.x), split_word(v.y), split_word(v.z), split_word(v.w));
    tile[pr][c4] = v.x;
    tile[pr][c4 + 1] = v.y;
    tile[pr][c4 + 2] = v.z;
    tile[pr][c4 + 3] = v.w;
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int idx = t + 256 * it, cr = idx >> 4, p4 = (idx & 15) * 4;
    if (c0 + cr >= Cs || p0 + p4 >= P) continue;
    float* dst = y + (long)(c0 + cr) * ld + p0 + p4;
    if (p0 + p4 + 3 < P && (ld & 3) == 0) {
      *reinterpret_cast<float4*>(dst) =
          make_float4(tile[p4][cr], tile[p4 + 1][cr], tile[p4 + 2][cr], tile[p4 + 3][cr]);
    } else {
      for (int e = 0; e < 4 && p0 + p4 + e < P; ++e) dst[e] = tile[p4 + e][cr];
    }
  }
}

}  // namespace rk

// Plane stride of a channel-major copy: a multiple of 4 floats that is NOT a multiple of a large
// power of two (P = 65536 would put all 128 rows of a tile on one L2 channel).
long rk_cp_ld(long P) { return (P + 63) / 64 * 64 + 64; }

void rk_nhwc_to_cp_pad(const float* x, float* y, int N, int H, int W, int Cs, int pad, int reflect,
                       int phase, int pack, hipStream_t s, int extra) {
  const long P = (long)N * (H + 2 * pad) * (W + 2 * pad + extra);
  const dim3 g((unsigned)((P + 63) / 64), ceil_div(Cs, 64));
  if (pack)
    hipLaunchKernelGGL(rk::nhwc_to_cp_pad_k<true>, g, dim3(256), 0, s, x, y, N, H, W, Cs, pad, reflect,
                       phase, rk_cp_ld(P), extra);
  else
    hipLaunchKernelGGL(rk::nhwc_to_cp_pad_k<false>, g, dim3(256), 0, s, x, y, N, H, W, Cs, pad, reflect,
                       phase, rk_cp_ld(P), extra);
}

void rk_nhwc_to_cp(const float* x, float* y, long P, int Cs, int pack, hipStream_t s) {
  const dim3 g((unsigned)((P + 63) / 64), ceil_div(Cs, 64));
  if (pack) hipLaunchKernelGGL(rk::nhwc_to_cp_k<true>, g, dim3(256), 0, s, x, y, P, Cs, rk_cp_ld(P));
  else hipLaunchKernelGGL(rk::nhwc_to_cp_k<false>, g, dim3(256), 0, s, x, y, P, Cs, rk_cp_ld(P));
}

// Tile kinds: 0 = 128x128 (8 waves, 64x32 each), 1 = 64x128, 2 = 128x64, 3 = 64x64 (4 waves),
// all 32-deep K-steps; 4 = 128x128 with 64-deep K-steps (139 KB LDS, one block per CU);
// 5 / 6 = 128x128 with 4 waves of 64x64 (4 accumulators per wave), 32- / 64-deep K-steps
int rk_pick(long M, int Nc, int override_kind) {
  if (override_kind >= 0 && override_kind <= 6) return override_kind;
  if (Nc <= 64) return M / 128 >= 256 ? 2 : 3;
  const long n128 = (Nc + 127) / 128;
  if ((M / 128) * n128 >= 200) return 0;
  if ((M / 64) * n128 >= 200) return 1;
  return 3;
}

// Geometry of a tile kind under `math` (the x6 image maps kinds 4 / 6 to their 32-deep twins) and
// its co-resident blocks per round: LDS-limited (double-buffered stage image: fp32 [rows][BK+4] or
// NP bf16 planes [rows][BK+8]) and at most two blocks per CU (__launch_bounds__(NT, 2)), one for
// the 8-wave kinds.  The x6 128x128 image (122 KB) fits one block per CU.
void rk_tile_geom(int kind, int math, int* bm, int* bn, int* bk, int* slots) {
  if (math == VST_MATH_BF16X6) kind = kind == 4 ? 0 : (kind == 6 ? 5 : kind);
  *bm = (kind == 1 || kind == 3) ? 64 : 128;
  *bn = (kind == 2 || kind == 3) ? 64 : 128;
  *bk = (kind == 4 || kind == 6) ? 64 : 32;
  const int np = math == VST_MATH_BF16X6 ? 3 : 2;
  const long stage = math == VST_MATH_F32 ? (long)(*bm + *bn) * (*bk + 4) * 4
                                          : (long)(*bm + *bn) * (*bk + 8) * 2 * np;
  long per_cu = (160L * 1024) / (2 * stage);
  const long cap = (kind == 0 || kind == 4) ? 1 : 2;
  if (per_cu > cap) per_cu = cap;
  if (per_cu < 1) per_cu = 1;
  *slots = (int)per_cu * VST_NUM_CUS;
}

#define VST_RK_DISPATCH_M(kind, LAUNCH, M_)                             \
  switch (kind) {                                                        \
    case 0: LAUNCH(128, 128, 64, 32, 32, M_) break;                      \
    case 1: LAUNCH(64, 128, 32, 64, 32, M_) break;                       \
    case 2: LAUNCH(128, 64, 64, 32, 32, M_) break;                       \
    case 4: LAUNCH(128, 128, 64, 32, (M_ == VST_MATH_BF16X6 ? 32 : 64), M_) break; \
    case 5: LAUNCH(128, 128, 64, 64, 32, M_) break;                      \
    case 6: LAUNCH(128, 128, 64, 64, (M_ == VST_MATH_BF16X6 ? 32 : 64), M_) break; \
    default: LAUNCH(64, 64, 32, 32, 32, M_) break;                       \
  }

// Conv GEMM arithmetic (per call): VST_MATH_F32 = v_mfma_f32_32x32x2_f32 (exact fp32 products);
// VST_MATH_BF16X3 / VST_MATH_BF16X6 = split-operand v_mfma_f32_32x32x16_bf16 (3 / 6 products per
// operand pair, fp32 accumulate).  The 3-plane x6 image only fits the 32-deep K-step tiles.
static int math_kind(int math, int kind) {
  if (math == VST_MATH_BF16X6) return kind == 4 ? 0 : (kind == 6 ? 5 : kind);
  return kind;
}

#define VST_MATH_SWITCH(math, LAUNCH_M)                                        \
  switch (math) {                                                               \
    case VST_MATH_BF16X3: { LAUNCH_M(VST_MATH_BF16X3) } break;                  \
    case VST_MATH_BF16X6: { LAUNCH_M(VST_MATH_BF16X6) } break;                  \
    default: { LAUNCH_M(VST_MATH_F32) } break;                                  \
  }

void rk_fprop_launch(const float* x, const float* wp, const float* bias, float* y, int N, int H, int W,
                     int C, int Ho, int Wo, int Cop, int R, int S, int st, int padh, int padw, int reflect,
                     int act, float slope, int kind, int math, hipStream_t s) {
  const int M = N * Ho * Wo, K = R * S * C;
  const int kd = math_kind(math, rk_pick(M, Cop, kind));
#define VST_LX(BM_, BN_, WM_, WN_, BK_, M_)                                                        \
  hipLaunchKernelGGL((rk::conv_fprop_rk_k<BM_, BN_, WM_, WN_, BK_, M_>),                             \
                     dim3(ceil_div(M, BM_), ceil_div(Cop, BN_)),                                     \
                     dim3(rk::Tile<BM_, BN_, WM_, WN_, BK_>::NT),                                    \
                     0, s, x, wp, bias, y, H, W, C, Ho, Wo, Cop, S, st, padh, padw, reflect, act, slope, \
                     M, K);
#define VST_LM(M_) VST_RK_DISPATCH_M(kd, VST_LX, M_)
  VST_MATH_SWITCH(math, VST_LM)
#undef VST_LM
#undef VST_LX
}

void rk_tconv_launch(const float* in, const float* wp, const float* bias, const float* addend,
                     float* out, int N, int Hi, int Wi, int Cy, int Ho, int Wo, int Cx, int R, int S,
                     int st, int pad, int reflect, int act, float slope, int kind, int math, hipStream_t s) {
  const int Hc = (Ho + st - 1) / st, Wc = (Wo + st - 1) / st;
  const int Mmax = N * Hc * Wc;
  const int kd = math_kind(math, rk_pick((long)Mmax * st * st, Cx, kind));
#define VST_LST(BM_, BN_, WM_, WN_, BK_, ST_, M_)                                                  \
  hipLaunchKernelGGL((rk::conv_tconv_rk_k<BM_, BN_, WM_, WN_, BK_, ST_, M_>),                        \
                     dim3(ceil_div(Mmax, BM_), ceil_div(Cx, BN_), st * st),                          \
                     dim3(rk::Tile<BM_, BN_, WM_, WN_, BK_>::NT), 0, s, in, wp, bias, addend, out, Hi, Wi, \
                     Cy, Ho, Wo, Cx, R, S, st, pad, reflect, act, slope, N)
#define VST_LX(BM_, BN_, WM_, WN_, BK_, M_)                 \
  if (st == 1) VST_LST(BM_, BN_, WM_, WN_, BK_, 1, M_);       \
  else if (st == 2) VST_LST(BM_, BN_, WM_, WN_, BK_, 2, M_);  \
  else VST_LST(BM_, BN_, WM_, WN_, BK_, 0, M_);
#define VST_LM(M_) VST_RK_DISPATCH_M(kd, VST_LX, M_)
  VST_MATH_SWITCH(math, VST_LM)
#undef VST_LM
#undef VST_LX
#undef VST_LST
}

#if WGRAD_XCD
#define WGRAD_GRID(mt, nt, z) dim3((mt) * (nt) * (z))
#else
#define WGRAD_GRID(mt, nt, z) dim3((mt), (nt), (z))
#endif

void rk_wgrad_launch(const float* xt, const float* dyt, float* slab, int N, int H, int W, int Cx,
                     int Ho, int Wo, int Cyp, int S, int pad, int st, int Mw, int chunk,
                     int nsplit, int kind, int math, hipStream_t s) {
  const int P = N * Ho * Wo;
  const int kd = math_kind(math, kind);
#define VST_LX(BM_, BN_, WM_, WN_, BK_, M_)                                                        \
  hipLaunchKernelGGL((rk::conv_wgrad_rk_k<BM_, BN_, WM_, WN_, BK_, M_>),                             \
                     WGRAD_GRID(ceil_div(Mw, BM_), ceil_div(Cyp, BN_), nsplit),                       \
                     dim3(rk::Tile<BM_, BN_, WM_, WN_, BK_>::NT), 0, s, xt, dyt, slab, H, W, Cx, Ho, \
                     Wo, Cyp, S, pad, st, Mw, P, chunk,                                         \
                     rk_cp_ld((long)N * (H + 2 * pad) * (W + 2 * pad)), rk_cp_ld(P));
#define VST_LM(M_) VST_RK_DISPATCH_M(kd, VST_LX, M_)
  VST_MATH_SWITCH(math, VST_LM)
#undef VST_LM
#undef VST_LX
}

}  // namespace vst
