// Split-operand bf16 implicit-GEMM convolutions for gfx950 — the VST_MATH_BF16X3 / _BF16X6 path of
// vst_conv2d_fwd / vst_conv2d_tfwd / vst_conv2d_wgrad when the channel counts allow 8-deep chunks.
//
// Arithmetic: every fp32 operand value v is carried as NP bf16 planes, hi = bf16(v), mid =
// bf16(v - hi), lo = bf16(v - hi - mid) (each difference exact in fp32), and the GEMM accumulates
// the split products on v_mfma_f32_32x32x16_bf16 into fp32:
//   NP = 2 (x3): lo*hi + hi*lo + hi*hi                       product error <= ~2^-16 relative
//   NP = 3 (x6): lo*hi + hi*lo + mid*mid + mid*hi + hi*mid + hi*hi    error <= ~2^-24 (fp32-equal)
// (here "lo" of the 2-plane form is the "mid" plane of the 3-plane pack, so one 3-plane weight
// pack serves both).
//
// Operands and staging:
//   A (activations, gathered with padding/stride/reflection) is loaded as fp32 — 8 consecutive k
//     (two float4) per thread and row — split in registers and written with one ds_write_b128
//     per plane.  Row addresses are recomputed only when the thread's filter tap changes.
//   B (conv weights) arrives pre-split (vst_weight_split planes of the packed [rows][K] matrix)
//     and is copied 16 B per plane straight into the LDS image.
// LDS image: per plane, [rows][BK] bf16 without padding; the 16-byte chunk c of row r sits at slot
// c ^ ((r >> SWS) & (KC - 1)), which makes every ds_read_b128 lane group (16 rows, one chunk
// column) and every ds_write_b128 group (8 lanes = two 64-B rows or one 128-B row) conflict-free.
#include <type_traits>

#include "common.h"

#ifndef VST_BF_X6K3
#define VST_BF_X6K3 0
#endif
#ifndef VST_BF_MINB
#define VST_BF_MINB 1
#endif
#ifndef VST_BF_X6_256
#define VST_BF_X6_256 1
#endif
#ifndef VST_BF_KSLICE
#define VST_BF_KSLICE 1
#endif
#ifndef VST_BF_TAIL_KIND
#define VST_BF_TAIL_KIND 8
#endif
#ifndef VST_BF_TAIL
#define VST_BF_TAIL 1
#endif

namespace vst {
namespace bf {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

template <int BM_, int BN_, int WM_, int WN_, int BK_, int NP_>
struct Tile {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, BK = BK_, NP = NP_;
  static constexpr int NW = (BM / WM) * (BN / WN);
  static constexpr int NT = 64 * NW;
  static constexpr int WAVES_N = BN / WN;
  static constexpr int MI = WM / 32, NI = WN / 32;
  static constexpr int KC = BK / 8;                      // 16-byte chunks per row
  static constexpr int SWS = KC == 2 ? 3 : (KC == 4 ? 2 : 1);
  static constexpr int ROWB = BK * 2;                    // bytes per row per plane
  static constexpr int A_PLANE = BM * ROWB, B_PLANE = BN * ROWB;  // bytes
  static constexpr int A_BYTES = NP * A_PLANE, STAGE = NP * (A_PLANE + B_PLANE);
  static constexpr int RPP = NT / KC;                    // rows staged per pass
  static constexpr int A_LD = BM / RPP, B_LD = BN / RPP;
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  static_assert(KC == 2 || KC == 4 || KC == 8, "BK in {16, 32, 64}");
  static_assert(BM % RPP == 0 && BN % RPP == 0, "row coverage");
  static_assert(2 * STAGE <= 160 * 1024, "LDS");
  // co-resident blocks per CU the register budget is compiled for: two when two double-buffered
  // stage pairs fit the 160 KB LDS, else one (then each wave may use the whole 2-wave budget)
#if VST_BF_MINB
  static constexpr int MINB = 4 * STAGE <= 160 * 1024 ? 2 : 1;
#else
  static constexpr int MINB = 2;
#endif
};

__device__ __forceinline__ int swz_off(int row, int c, int rowb, int sws, int kcm) {
  return row * rowb + 16 * (c ^ ((row >> sws) & kcm));
}

__device__ __forceinline__ uint32_t pack2(float a, float b) {
  const f32x2_t v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

// Split 8 fp32 values into NP bf16 planes (uint4 = 8 bf16 each).
template <int NP>
__device__ __forceinline__ void split8(const float4& a, const float4& b, uint4 (&o)[NP]) {
  float r[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    uint32_t q[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) q[e] = pack2(r[2 * e], r[2 * e + 1]);
    o[p] = make_uint4(q[0], q[1], q[2], q[3]);
    if (p + 1 < NP) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        r[2 * e] -= __uint_as_float(q[e] << 16);
        r[2 * e + 1] -= __uint_as_float(q[e] & 0xffff0000u);
      }
    }
  }
}

// MMA over one staged K-step.  hook(g) runs before k group g (used to issue the next stage's loads).
template <class T, class Hook>
__device__ __forceinline__ void mma_stage(const char* __restrict__ As, const char* __restrict__ Bs,
                                          f32x16 (&acc)[T::MI][T::NI], int wm0, int wn0, int lane,
                                          Hook hook) {
  constexpr int NP = T::NP;
  const int kh = lane >> 5, li = lane & 31;
  bf16x8_t fa[2][NP][T::MI], fb[2][NP][T::NI];
  auto rd = [&](int buf, int g) {
    const int c = 2 * g + kh;
#pragma unroll
    for (int i = 0; i < T::MI; ++i) {
      const int off = swz_off(wm0 + 32 * i + li, c, T::ROWB, T::SWS, T::KC - 1);
#pragma unroll
      for (int p = 0; p < NP; ++p) fa[buf][p][i] = *reinterpret_cast<const bf16x8_t*>(As + p * T::A_PLANE + off);
    }
#pragma unroll
    for (int j = 0; j < T::NI; ++j) {
      const int off = swz_off(wn0 + 32 * j + li, c, T::ROWB, T::SWS, T::KC - 1);
#pragma unroll
      for (int p = 0; p < NP; ++p) fb[buf][p][j] = *reinterpret_cast<const bf16x8_t*>(Bs + p * T::B_PLANE + off);
    }
  };
  rd(0, 0);
#pragma unroll
  for (int g = 0; g < T::BK / 16; ++g) {
    const int cur = g & 1;
    hook(g);
    if (g + 1 < T::BK / 16) rd(cur ^ 1, g + 1);
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

// Stage writer: A rows as fp32 pairs (split here), B rows as pre-split planes.  The row masks are
// applied here, not at load time, so that no wait for the loads is forced before the MFMAs.
template <class T>
__device__ __forceinline__ void store_stage(char* st, const float4 (&ra)[T::A_LD][2],
                                            const uint4 (&rbv)[T::B_LD][T::NP], uint32_t msk, int rb,
                                            int kq) {
  char* Bs = st + T::A_BYTES;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int j = 0; j < T::A_LD; ++j) {
    uint4 s[T::NP];
    const bool ok = (msk >> j) & 1;
    split8<T::NP>(ok ? ra[j][0] : z, ok ? ra[j][1] : z, s);
    const int off = swz_off(rb + T::RPP * j, kq, T::ROWB, T::SWS, T::KC - 1);
#pragma unroll
    for (int p = 0; p < T::NP; ++p) *reinterpret_cast<uint4*>(st + p * T::A_PLANE + off) = s[p];
  }
#pragma unroll
  for (int j = 0; j < T::B_LD; ++j) {
    const bool ok = (msk >> (16 + j)) & 1;
    const int off = swz_off(rb + T::RPP * j, kq, T::ROWB, T::SWS, T::KC - 1);
#pragma unroll
    for (int p = 0; p < T::NP; ++p)
      *reinterpret_cast<uint4*>(Bs + p * T::B_PLANE + off) = ok ? rbv[j][p] : make_uint4(0, 0, 0, 0);
  }
}

// K loop with a two-deep load pipeline: the global loads of stage k + 2 are issued at the start of
// stage k's MFMAs into the register set stage k vacated, and stage k + 1's registers (loaded one
// whole stage earlier) are split and written to the other LDS buffer after stage k's MFMAs; one
// barrier per stage.  load_all(set) loads the cursor's stage into register set `set`; adv() moves
// the cursor one stage on.
template <class T, class LoadAll, class Adv>
__device__ __forceinline__ void main_loop(char* smem, int nk, f32x16 (&acc)[T::MI][T::NI],
                                          float4 (&ra)[2][T::A_LD][2], uint4 (&rbv)[2][T::B_LD][T::NP],
                                          uint32_t (&msk)[2], int rb, int kq, LoadAll load_all, Adv adv) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm0 = (wave / T::WAVES_N) * T::WM, wn0 = (wave % T::WAVES_N) * T::WN;
  if (nk <= 0) return;
  load_all(0);
  store_stage<T>(smem, ra[0], rbv[0], msk[0], rb, kq);
  if (nk > 1) {
    adv();
    load_all(1);
  }
  __syncthreads();
  auto step = [&](int kt, auto par) {
    constexpr int P = decltype(par)::value;
    char* cur = smem + P * T::STAGE;
    mma_stage<T>(cur, cur + T::A_BYTES, acc, wm0, wn0, lane, [&](int g) {
      if (g == 0 && kt + 2 < nk) {
        adv();
        load_all(P);
      }
    });
    if (kt + 1 < nk) store_stage<T>(smem + (P ^ 1) * T::STAGE, ra[P ^ 1], rbv[P ^ 1], msk[P ^ 1], rb, kq);
    __syncthreads();
  };
  for (int kt = 0; kt < nk; kt += 2) {
    step(kt, std::integral_constant<int, 0>());
    if (kt + 1 < nk) step(kt + 1, std::integral_constant<int, 1>());
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

__device__ __forceinline__ int remap_mtile(int bx, int nx) {
  if ((nx & 7) != 0) return bx;
  return (bx & 7) * (nx >> 3) + (bx >> 3);
}

// XCD-aware tile order for a 1-D grid of Mt*Nt tiles.  Consecutive workgroup ids land on
// consecutive XCDs, so XCD x (= L % 8) gets the contiguous tile range [x*T/8, (x+1)*T/8) in
// (m-major, n-minor) order: the N-tiles that share an A row block run together on one XCD and the
// XCD's resident working set is (CUs per XCD / Nt) M-tiles of activations, which stays in its L2.
__device__ __forceinline__ void tile_of(int L, int Mt, int Nt, int& mt, int& nt) {
  const int T = Mt * Nt;
  const int t = (T & 7) ? L : (L & 7) * (T >> 3) + (L >> 3);
  mt = t / Nt;
  nt = t - mt * Nt;
}

// ------------------------------------------------------------------------------------------ fprop
// y[m = (n, ho, wo)][co] = act(sum_k x_gather[m][k] * w[co][k] + bias[co]),  k = (r, s, ci);
// requires C % 8 == 0 (a thread's 8-deep chunk stays inside one tap).  ws = pre-split weight planes
// of the VST_PACK_OK matrix [Cop][R*S*C], plane stride wps elements.
template <class T>
__global__ __launch_bounds__(T::NT, T::MINB) void conv_fprop_bf_k(
    const float* __restrict__ x, const __bf16* __restrict__ ws, long wps, const float* __restrict__ bias,
    float* __restrict__ y, int H, int W, int C, int Ho, int Wo, int Cop, int S, int st, int padh,
    int padw, int reflect, int act, float slope, int M, int Ktot, int m_base) {
  __shared__ __attribute__((aligned(16))) char smem[2 * T::STAGE];
  constexpr int A_LD = T::A_LD, B_LD = T::B_LD, RPP = T::RPP, NP = T::NP;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  int mt_, nt_;
  tile_of(blockIdx.x, (M - m_base + T::BM - 1) / T::BM, (Cop + T::BN - 1) / T::BN, mt_, nt_);
  const int m0 = m_base + mt_ * T::BM, n0 = nt_ * T::BN;
  const int kq = t % T::KC, rb = t / T::KC;

  // this thread's chunk: absolute k = kcur, tap (kr, ks), channel kc.
  // Channel-sliced K order (C % BK == 0): K-steps walk the R*S taps of one BK-channel slice, then
  // the next slice, so one slice of the block's activation rows is reused by all taps while it
  // is L2-resident (tap-major order streams the whole C-deep block through L2 once per tap).  The
  // weight planes keep their (r, s, ci) layout: the B offset of a step is (r*S + s)*C + kc.
  // Applied where the tap-major order overflows L2: the 256-row x6 tiles (one round, 4 MB live
  // activation block per XCD: 289 -> 96 MB HBM traffic per N=8 ResnetBlock launch).  Smaller
  // tiles keep the tap-major summation order.
  const bool ksl = VST_BF_KSLICE && T::BM == 256 && NP == 3 && C % T::BK == 0 && Ktot % C == 0;
  const int Rk = ksl ? Ktot / (S * C) : 0;
  int kcur = 8 * kq;
  int kc = kcur % C, ks, kr;
  {
    const int rs = kcur / C;
    kr = rs / S;
    ks = rs - kr * S;
  }
  int hb[A_LD], wb[A_LD], nb[A_LD], aoff[A_LD];
#pragma unroll
  for (int j = 0; j < A_LD; ++j) {
    const int m = m0 + rb + RPP * j;
    const int mm = m < M ? m : 0;
    const int hw = Ho * Wo;
    const int n = mm / hw, rem = mm - n * hw, ho = rem / Wo, wo = rem - ho * Wo;
    hb[j] = ho * st - padh;
    wb[j] = wo * st - padw;
    nb[j] = m < M ? n : -1;
  }
  auto tap_rows = [&]() {
#pragma unroll
    for (int j = 0; j < A_LD; ++j) {
      int hi = hb[j] + kr, wi = wb[j] + ks;
      bool ok = nb[j] >= 0;
      if (reflect) {
        hi = reflect_idx(hi, H);
        wi = reflect_idx(wi, W);
      } else {
        ok = ok && (unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W;
      }
      aoff[j] = ok ? ((nb[j] * H + hi) * W + wi) * C : -1;
    }
  };
  tap_rows();
  const __bf16* wrow[B_LD];
  bool nv[B_LD];
#pragma unroll
  for (int j = 0; j < B_LD; ++j) {
    const int n = n0 + rb + RPP * j;
    nv[j] = n < Cop;
    wrow[j] = ws + (long)(nv[j] ? n : 0) * Ktot;
  }

  float4 ra[2][A_LD][2];
  uint4 rbv[2][B_LD][NP];
  uint32_t msk[2];
  // unconditional loads: invalid rows / the K tail read a safe address; the row mask (bit j = A row
  // j, bit 16 + j = B row j) zeroes them when the stage is written to LDS
  auto load_all = [&](int set) {
    const bool kin = ksl ? kc < C : kcur < Ktot;
    const int kk = kin ? (ksl ? (kr * S + ks) * C + kc : kcur) : 0;
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < A_LD; ++j) {
      const bool ok = kin && aoff[j] >= 0;
      m |= (uint32_t)ok << j;
      const float* p = x + (ok ? aoff[j] + kc : 0);
      ra[set][j][0] = *reinterpret_cast<const float4*>(p);
      ra[set][j][1] = *reinterpret_cast<const float4*>(p + 4);
    }
#pragma unroll
    for (int j = 0; j < B_LD; ++j) {
      m |= (uint32_t)(kin && nv[j]) << (16 + j);
#pragma unroll
      for (int p = 0; p < NP; ++p) rbv[set][j][p] = *reinterpret_cast<const uint4*>(wrow[j] + p * wps + kk);
    }
    msk[set] = m;
  };
  auto adv = [&]() {
    if (ksl) {
      if (++ks == S) {
        ks = 0;
        if (++kr == Rk) { kr = 0; kc += T::BK; }
      }
      tap_rows();
      return;
    }
    kcur += T::BK;
    kc += T::BK;
    if (kc >= C) {
      do {
        kc -= C;
        if (++ks == S) { ks = 0; ++kr; }
      } while (kc >= C);
      tap_rows();
    }
  };

  f32x16 acc[T::MI][T::NI];
  zero_acc(acc);
  main_loop<T>(smem, (Ktot + T::BK - 1) / T::BK, acc, ra, rbv, msk, rb, kq, load_all, adv);

  const int wm0 = (wave / T::WAVES_N) * T::WM, wn0 = (wave % T::WAVES_N) * T::WN;
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

// split an fp32 buffer into three bf16 planes (hi, mid, lo) of n elements each
__global__ void split3_k(const float* __restrict__ w, __bf16* __restrict__ out, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = w[i];
  const __bf16 h = (__bf16)v;
  const float r = v - (float)h;
  const __bf16 m = (__bf16)r;
  out[i] = h;
  out[n + i] = m;
  out[2 * n + i] = (__bf16)(r - (float)m);
}

}  // namespace bf

// Tile table of the split-arithmetic kernels (kind; x6 maps the BK = 64 kinds to their BK = 32
// twins when the three-plane image would not fit):
//   0: 128x128, 8 waves of 64x32, BK 32      1: 128x64, 4 waves of 64x32, BK 32 (2 blocks / CU)
//   2: 128x128, 4 waves of 64x64, BK 32      3: 64x128, 4 waves of 32x64, BK 32
//   4: 128x128, 8 waves of 64x32, BK 64      5: 128x64, 4 waves of 64x32, BK 64
//   6: 64x64, 4 waves of 32x32, BK 32
#define VST_BF_DISPATCH(kind, np, L)                                   \
  switch (kind) {                                                      \
    case 1: L(128, 64, 64, 32, 32, np) break;                          \
    case 2: L(128, 128, 64, 64, 32, np) break;                         \
    case 3: L(64, 128, 32, 64, 32, np) break;                          \
    case 4: L(128, 128, 64, 32, (np == 3 ? 32 : 64), np) break;        \
    case 5: L(128, 64, 64, 32, 64, np) break;                          \
    case 6: L(64, 64, 32, 32, 32, np) break;                           \
    case 7: L(256, 128, 64, 64, 32, np) break;                         \
    case 8: L(64, 64, 32, 32, (np == 3 ? 32 : 64), np) break;          \
    default: L(128, 128, 64, 32, 32, np) break;                        \
  }

int bf_pick(long M, int Nc, int override_kind) {
  if (override_kind >= 0 && override_kind <= 7) return override_kind;
  if (Nc <= 64) return M / 128 >= 256 ? 1 : 6;
  const long n128 = (Nc + 127) / 128;
  if ((M / 128) * n128 >= 200) return 0;
  if ((M / 64) * n128 >= 200) return 3;
  return 6;
}

// Launch plan of the split-arithmetic forward for an M x Cop output: the tile kind of the main
// launch and, when the grid is split for wave quantisation, the first pixel row of the tail launch
// (0 = one launch).  Host-only; also exported through vst_conv_plan_fwd for tests and the bench.
void bf_plan(long M, int Cop, int math, int kind, int* kind_out, int* m_split_out) {
  int kd = bf_pick(M, Cop, kind);
#if VST_BF_X6K3
  // x6: the 128x128 three-plane stage pair (96 KB) fits one block per CU; 64x128 tiles fit two
  if (kind < 0 && kd == 0 && math == VST_MATH_BF16X6) kd = 3;
#endif
#if VST_BF_X6_256
  // x6, one block per CU either way: 256x128 tiles of 8 waves x (64x64) halve the LDS fragment
  // reads per MFMA and the barriers per FLOP — when the grid is whole rounds of 256 blocks
  if (kind < 0 && kd == 0 && math == VST_MATH_BF16X6) {
    const long b256 = (long)((M + 255) / 256) * ((Cop + 127) / 128);
    if (b256 % VST_NUM_CUS == 0 || b256 >= 4 * VST_NUM_CUS) kd = 7;
  }
#endif
  int m_split = 0;
#if VST_BF_TAIL
  // Wave quantisation: 128x128 x3 blocks run two per CU, so a grid a few tiles past a whole
  // number of blocks per CU (the padded-frame dgrad: 546 = 2 x 256 + 34 blocks at N = 8) keeps
  // most CUs idle for one extra block time.  Such a tail (<= 1/4 of the CUs) runs as a second
  // launch of 64x64 tiles over the remaining pixel rows (4x as many, 4x smaller blocks).
  if (kind < 0 && kd == 0 && math != VST_MATH_BF16X6) {
    const long nt = (Cop + 127) / 128, blocks = (long)((M + 127) / 128) * nt;
    const long per = blocks / VST_NUM_CUS, tail = blocks - per * VST_NUM_CUS;
    if (per >= 1 && tail > 0 && 4 * tail <= VST_NUM_CUS && (per * VST_NUM_CUS) % nt == 0)
      m_split = (int)(per * VST_NUM_CUS / nt) * 128;
  }
#endif
  *kind_out = kd;
  *m_split_out = m_split;
}

int bf_fprop_launch(const float* x, const void* wsplit, long wps, const float* bias, float* y, int N,
                    int H, int W, int C, int Ho, int Wo, int Cop, int R, int S, int st, int padh, int padw,
                    int reflect, int act, float slope, int math, int kind, hipStream_t s) {
  const int M = N * Ho * Wo, K = R * S * C;
  const __bf16* ws = reinterpret_cast<const __bf16*>(wsplit);
  int kd, m_split;
  bf_plan(M, Cop, math, kind, &kd, &m_split);
#define VST_BF(BM_, BN_, WM_, WN_, BK_, NP_)                                                     \
  {                                                                                                 \
    using T = bf::Tile<BM_, BN_, WM_, WN_, BK_, NP_>;                                              \
    hipLaunchKernelGGL(bf::conv_fprop_bf_k<T>, dim3(ceil_div(Mend - mb, BM_) * ceil_div(Cop, BN_)),   \
                       dim3(T::NT), 0, s, x, ws, wps, bias, y, H, W, C, Ho, Wo, Cop, S,             \
                       st, padh, padw, reflect, act, slope, Mend, K, mb);                           \
  }
  for (int part = 0; part < (m_split ? 2 : 1); ++part) {
    const int mb = part ? m_split : 0, Mend = (m_split && !part) ? m_split : M;
    const int kp = part ? VST_BF_TAIL_KIND : kd;
    if (math == VST_MATH_BF16X6) {
      VST_BF_DISPATCH(kp, 3, VST_BF)
    } else {
      VST_BF_DISPATCH(kp, 2, VST_BF)
    }
  }
#undef VST_BF
  return check_launch("conv2d_fwd(bf16 split)");
}

}  // namespace vst

using namespace vst;

extern "C" int vst_weight_split(const float* w, void* out, long n, void* stream) {
  VST_REQUIRE(w && out && n > 0, "weight_split: bad args");
  hipLaunchKernelGGL(bf::split3_k, dim3(ceil_div(n, 256)), dim3(256), 0, (hipStream_t)stream, w,
                     reinterpret_cast<__bf16*>(out), n);
  return check_launch("weight_split");
}
