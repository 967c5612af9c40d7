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
#ifndef VST_BF_SCHED
#define VST_BF_SCHED 1
#endif
#ifndef VST_BF_PRIO
#define VST_BF_PRIO 0
#endif
#ifndef VST_BF_MF16
#define VST_BF_MF16 1
#endif
#ifndef VST_M16_STORE
#define VST_M16_STORE 0  // M16 loop: stage store in group B (0) or group A (1)
#endif
#ifndef VST_M16_RDLO
#define VST_M16_RDLO 0  // M16 loop: lo plane read in group B (0) or with hi in group A (1)
#endif
#ifndef VST_M16_SCHED
#define VST_M16_SCHED 0  // M16 loop: sched_group_barrier filler pattern (0: compiler order)
#endif
#ifndef VST_M16_LOADFIRST
#define VST_M16_LOADFIRST 0  // M16 loop: scheduling fence after group A (its global loads issue before group B's stores)
#endif
#ifndef VST_M16_PRIO
#define VST_M16_PRIO 0  // M16 loop: s_setprio 1 for the second-dispatched half of the waves
#endif
#ifndef VST_M16_LOADEARLY
#define VST_M16_LOADEARLY 0  // M16 loop: the next stages' loads first in the step, fenced
#endif
#ifndef VST_BF_SPLITK
#define VST_BF_SPLITK 1  // split-K wave-quantisation tails (when the caller passes a workspace)
#endif
#ifndef VST_BF_FULLSPLIT_MAX
#define VST_BF_FULLSPLIT_MAX 128  // x6 forwards of at most this many 256x128 tiles run whole as split-K
#endif
#ifndef VST_BF_TAIL_FORCE
#define VST_BF_TAIL_FORCE -1
#endif
#ifndef VST_WG_SELECT
#define VST_WG_SELECT 1
#endif
#ifndef VST_BF_STORE_LATE
#define VST_BF_STORE_LATE 0
#endif
#ifndef VST_BF_LDS_EPI
#define VST_BF_LDS_EPI 0  // M16 forward epilogue: tile staged through LDS, stored as whole float4 rows
#endif

namespace vst {
namespace bf {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));  // a 16-B chunk as a first-class value

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
  // M16 (x6, BK 32, 64-deep wave tiles): the products run on v_mfma_f32_16x16x32_bf16 (16x16
  // blocks, one 32-deep k step per stage) instead of 32x32x16 — the same cycles per FLOP, but the
  // chip holds a higher clock on it under load (MI355X_MICROARCH.md, DVFS item 7).
  static constexpr bool M16 = VST_BF_MF16 && NP == 3 && BK == 32 && WM % 32 == 0 && WN % 32 == 0;
  static constexpr int MI16 = WM / 16, NI16 = WN / 16;
  // chunk XOR of a row's 16-B chunks: row group q = (row >> SWS) & (KC - 1).  The 16x16x32 reads
  // (lane: row l & 15, chunk l >> 4) are conflict-free for the ds_read_b128 lane groups
  // {0-3,12-15,20-27}, {4-11,16-19,28-31}, ... with q -> {0, 2, 3, 1}; the 32x32x16 reads with q.
  __device__ static __forceinline__ int swz(int row) {
    const int q = (row >> SWS) & (KC - 1);
    if constexpr (M16) return (0x1320 >> (4 * q)) & 3;  // KC == 4
    return q;
  }
  // co-resident blocks per CU the register budget is compiled for: two when two double-buffered
  // stage pairs fit the 160 KB LDS, else one (then each wave may use the whole 2-wave budget)
#if VST_BF_MINB
  static constexpr int MINB = 4 * STAGE <= 160 * 1024 ? 2 : 1;
#else
  static constexpr int MINB = 2;
#endif
};

template <class T>
__device__ __forceinline__ int swz_off(int row, int c) {
  return row * T::ROWB + 16 * (c ^ T::swz(row));
}

__device__ __forceinline__ uint32_t pack2(float a, float b) {
  const f32x2_t v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

// Split 8 fp32 values into NP bf16 planes (uint4 = 8 bf16 each).
#ifndef VST_BF_FAKE16
#define VST_BF_FAKE16 0
#endif
#ifndef VST_BF_FAKESPLIT
#define VST_BF_FAKESPLIT 0  // developer timing experiment only: hi plane replicated (WRONG results)
#endif
// The two timing modes above compute WRONG results: only a developer variant build (tools/
// build_variant.py, which defines VST_DEV_VARIANT and writes _build/variants/, never the product
// library) may turn them on.
#ifndef VST_BF_FAKE_ZA
#define VST_BF_FAKE_ZA 0  // developer timing experiment only: every A gather reads the zero page (WRONG results)
#endif
#ifndef VST_BF_FAKE_ADMA
#define VST_BF_FAKE_ADMA 0  // developer timing experiment only: A LDS-DMA'd from x's own bytes (WRONG results)
#endif
#ifndef VST_BF_FAKE_ZB
#define VST_BF_FAKE_ZB 0  // developer timing experiment only: every B load reads the zero page (WRONG results)
#endif
#if (VST_BF_FAKESPLIT || VST_BF_FAKE16 || VST_BF_FAKE_ZA || VST_BF_FAKE_ZB || VST_BF_FAKE_ADMA) && !defined(VST_DEV_VARIANT)
#error "VST_BF_FAKESPLIT / VST_BF_FAKE16 are developer-only timing modes (wrong results): build them with tools/build_variant.py"
#endif
template <int NP>
__device__ __forceinline__ void split8(const float4& a, const float4& b, uint4 (&o)[NP]) {
  if (VST_BF_FAKESPLIT) {
    const uint4 h = make_uint4(pack2(a.x, a.y), pack2(a.z, a.w), pack2(b.x, b.y), pack2(b.z, b.w));
#pragma unroll
    for (int p = 0; p < NP; ++p) o[p] = h;
    return;
  }
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

// One k group (16 deep) of a wave's operand fragments: NP planes x (MI A + NI B) bf16x8 per lane.
template <class T>
struct Frag {
  bf16x8_t a[T::NP][T::MI], b[T::NP][T::NI];
};

// LDS -> registers: k group g of the stage image at st (lane l: row l % 32, 8-deep chunk 2g + l / 32).
template <class T>
__device__ __forceinline__ void read_frag(Frag<T>& f, const char* __restrict__ st, int g, int wm0, int wn0,
                                          int lane) {
  const char* As = st;
  const char* Bs = st + T::A_BYTES;
  const int c = 2 * g + (lane >> 5), li = lane & 31;
#pragma unroll
  for (int i = 0; i < T::MI; ++i) {
    const int off = swz_off<T>(wm0 + 32 * i + li, c);
#pragma unroll
    for (int p = 0; p < T::NP; ++p) f.a[p][i] = *reinterpret_cast<const bf16x8_t*>(As + p * T::A_PLANE + off);
  }
#pragma unroll
  for (int j = 0; j < T::NI; ++j) {
    const int off = swz_off<T>(wn0 + 32 * j + li, c);
#pragma unroll
    for (int p = 0; p < T::NP; ++p) f.b[p][j] = *reinterpret_cast<const bf16x8_t*>(Bs + p * T::B_PLANE + off);
  }
}

// The split products of one k group into the wave's accumulators.
template <class T>
__device__ __forceinline__ void mma_frag(const Frag<T>& f, f32x16 (&acc)[T::MI][T::NI]) {
#pragma unroll
  for (int i = 0; i < T::MI; ++i)
#pragma unroll
    for (int j = 0; j < T::NI; ++j) {
#if VST_BF_FAKE16  // developer timing experiment only (WRONG results): each 32x32x16 as two 16x16x32
#define VST_MF(pA, pB)                                                                                   \
  {                                                                                                      \
    f32x4v q0 = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};                                 \
    f32x4v q1 = {acc[i][j][4], acc[i][j][5], acc[i][j][6], acc[i][j][7]};                                 \
    q0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[pA][i], f.b[pB][j], q0, 0, 0, 0);                  \
    q1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.b[pB][j], f.a[pA][i], q1, 0, 0, 0);                  \
    acc[i][j][0] = q0[0]; acc[i][j][1] = q0[1]; acc[i][j][2] = q0[2]; acc[i][j][3] = q0[3];              \
    acc[i][j][4] = q1[0]; acc[i][j][5] = q1[1]; acc[i][j][6] = q1[2]; acc[i][j][7] = q1[3];              \
  }
#else
#define VST_MF(pA, pB) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[pA][i], f.b[pB][j], acc[i][j], 0, 0, 0)
#endif
      if constexpr (T::NP == 3) {
        VST_MF(2, 0); VST_MF(0, 2); VST_MF(1, 1); VST_MF(1, 0); VST_MF(0, 1); VST_MF(0, 0);
      } else {
        VST_MF(1, 0); VST_MF(0, 1); VST_MF(0, 0);
      }
#undef VST_MF
    }
}

// Stage writer: A rows as fp32 pairs (split here), B rows as pre-split planes.  Masked rows were
// loaded from the zero page, so every row is written unconditionally.
#ifndef VST_BF_GLDS_B
#define VST_BF_GLDS_B 1  // x6 M16 KSL forwards: the pre-split B operand LDS-DMA'd (global_load_lds_dwordx4)
                         // instead of register-staged
#endif
template <class T>
__device__ __forceinline__ void store_stage(char* st, const float4 (&ra)[T::A_LD][2],
                                            const u32x4_t (&rbv)[T::B_LD][T::NP], int rb, int kq,
                                            bool with_b = true, bool with_a = true) {
  char* Bs = st + T::A_BYTES;
#pragma unroll
  for (int j = 0; j < T::A_LD; ++j) {
    if (!with_a) break;
    uint4 s[T::NP];
    split8<T::NP>(ra[j][0], ra[j][1], s);
    const int off = swz_off<T>(rb + T::RPP * j, kq);
#pragma unroll
    for (int p = 0; p < T::NP; ++p) *reinterpret_cast<uint4*>(st + p * T::A_PLANE + off) = s[p];
  }
  if (!with_b) return;
#pragma unroll
  for (int j = 0; j < T::B_LD; ++j) {
    const int off = swz_off<T>(rb + T::RPP * j, kq);
#pragma unroll
    for (int p = 0; p < T::NP; ++p) *reinterpret_cast<u32x4_t*>(Bs + p * T::B_PLANE + off) = rbv[j][p];
  }
}

// Issue pattern of one k group's MFMAs (VST_BF_SCHED): each MFMA is followed by a share of the
// group's other work, so the fragment reads, global loads, the split VALU and its ds_writes sit
// in the MFMA gaps instead of in blocks the matrix pipe waits behind.  first: the group that also
// issues the next loads and the stage store; the group after the barrier only reads fragments.
template <class T>
__device__ __forceinline__ void sched_group(bool first, bool after_barrier) {
  constexpr int NM = T::MI * T::NI * (T::NP == 3 ? 6 : 3) * (VST_BF_FAKE16 ? 2 : 1);  // MFMAs per k group
  constexpr int NR = T::NP * (T::MI + T::NI);                   // ds_read_b128 per k group
  constexpr int NV = T::A_LD * 2 + T::B_LD * T::NP;             // global loads per stage
  constexpr int NW = T::A_LD * T::NP + T::B_LD * T::NP;         // ds_write_b128 per stage
  if (first && !after_barrier) {
    if (VST_BF_SCHED < 2) return;
#pragma unroll
    for (int i = 0; i < NM; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);          // MFMA
      if (i < NR) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
      if (i < NV) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read
      __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);          // VALU
      if (i >= NM - NW - 1 && i < NM - 1) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // DS write
    }
  } else {
#pragma unroll
    for (int i = 0; i < NM; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      if (i < NR) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
    }
  }
}

// K loop with a two-deep global-load pipeline and LDS fragments read one k group ahead, across
// the stage boundary.  Stage kt (LDS buffer P = kt & 1):
//   group 0: read group 1's fragments; issue the global loads of stage kt + 2 into register set P;
//            split + write stage kt + 1 (register set P ^ 1, loaded one stage earlier) into buffer
//            P ^ 1; MFMAs of group 0 — the split VALU and ds_writes fill the MFMA gaps;
//   last group: barrier (buffer P ^ 1 complete, every read of buffer P done), read stage kt + 1's
//            group 0 from buffer P ^ 1 into the free fragment set, then this group's MFMAs, which
//            cover that read's latency.
// Every load and store is unconditional (the last two stages re-load the final stage's addresses
// and write an LDS image nobody reads; the cursor stops advancing there): a conditional load
// makes the wait-count pass merge "issued / not issued" paths and drain the whole prefetch
// (vmcnt(0)) before each stage's stores.  load_all(set) loads the cursor's stage into register
// set `set`; adv(go) moves the cursor one stage on when go.  An odd stage count runs its last stage after
// the two-stage loop.
template <class T, class LoadAll, class Adv, class Prep>
__device__ __forceinline__ void main_loop(char* smem, int nk, f32x16 (&acc)[T::MI][T::NI],
                                          float4 (&ra)[2][T::A_LD][2], u32x4_t (&rbv)[2][T::B_LD][T::NP],
                                          int rb, int kq, LoadAll load_all, Adv adv, Prep prep) {
  constexpr int G = T::BK / 16;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm0 = (wave / T::WAVES_N) * T::WM, wn0 = (wave % T::WAVES_N) * T::WN;
  if (nk <= 0) return;
  // second-dispatched half of the waves: static priority 1 (it otherwise loses every issue
  // arbitration to its older partner on the SIMD; MI355X_MICROARCH.md, two waves per SIMD, item 4)
  if (VST_BF_PRIO && wave >= T::NW / 2) __builtin_amdgcn_s_setprio(1);
  load_all(0);
  prep(0);
  store_stage<T>(smem, ra[0], rbv[0], rb, kq);
  adv(nk > 1);
  load_all(1);
  __syncthreads();
  Frag<T> fr[2];
  read_frag<T>(fr[0], smem, 0, wm0, wn0, lane);
  auto step = [&](int kt, auto par) __attribute__((always_inline)) {
    constexpr int P = decltype(par)::value;
    const char* cur = smem + P * T::STAGE;
    char* nxt = smem + (P ^ 1) * T::STAGE;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int fi = (P * G + g) & 1;
      if (g + 1 < G) read_frag<T>(fr[fi ^ 1], cur, g + 1, wm0, wn0, lane);
      if (g == 0) {
        adv(kt + 2 < nk);
        load_all(P);
        if (!VST_BF_STORE_LATE) {
          prep(P ^ 1);
          store_stage<T>(nxt, ra[P ^ 1], rbv[P ^ 1], rb, kq);
        }
      }
      if (g == G - 1) {
        if (VST_BF_STORE_LATE) {
          prep(P ^ 1);
          store_stage<T>(nxt, ra[P ^ 1], rbv[P ^ 1], rb, kq);
        }
        __builtin_amdgcn_sched_barrier(0);  // keep this group's MFMAs after the barrier (they cover the read)
        __syncthreads();
        read_frag<T>(fr[fi ^ 1], nxt, 0, wm0, wn0, lane);
      }
      mma_frag<T>(fr[fi], acc);
      if (VST_BF_SCHED) sched_group<T>(g == 0, g == G - 1);
    }
  };
  int kt = 0;
  for (; kt + 1 < nk; kt += 2) {
    step(kt, std::integral_constant<int, 0>());
    step(kt + 1, std::integral_constant<int, 1>());
  }
  if (kt < nk) step(kt, std::integral_constant<int, 0>());
}

// ---- M16: v_mfma_f32_16x16x32_bf16 (lane l: A row l & 15 / B column l & 15, k = 8 (l >> 4) .. +7;
// C/D: column l & 15, rows 4 (l >> 4) + r).  One plane of a wave's operands for the stage's 32-deep
// k step: MI16 A and NI16 B fragments.
template <class T>
struct Plane16 {
  bf16x8_t a[T::MI16], b[T::NI16];
};

template <class T>
__device__ __forceinline__ void read_plane16(Plane16<T>& f, const char* __restrict__ st, int p, int wm0, int wn0,
                                             int lane) {
  const char* As = st + p * T::A_PLANE;
  const char* Bs = st + T::A_BYTES + p * T::B_PLANE;
  const int c = lane >> 4, li = lane & 15;
#pragma unroll
  for (int i = 0; i < T::MI16; ++i)
    f.a[i] = *reinterpret_cast<const bf16x8_t*>(As + swz_off<T>(wm0 + 16 * i + li, c));
#pragma unroll
  for (int j = 0; j < T::NI16; ++j)
    f.b[j] = *reinterpret_cast<const bf16x8_t*>(Bs + swz_off<T>(wn0 + 16 * j + li, c));
}

template <class T>
__device__ __forceinline__ void mma16(const Plane16<T>& A, const Plane16<T>& B, f32x4v (&acc)[T::MI16][T::NI16]) {
#pragma unroll
  for (int i = 0; i < T::MI16; ++i)
#pragma unroll
    for (int j = 0; j < T::NI16; ++j)
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A.a[i], B.b[j], acc[i][j], 0, 0, 0);
}

// Fillers of an M16 group: every MFMA followed by its share of the group's reads / loads / VALU /
// ds_writes (the same idea as sched_group).
template <int NM, int NR, int NV, int NVALU, int NW>
__device__ __forceinline__ void sched16() {
#pragma unroll
  for (int i = 0; i < NM; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    if (i < NR) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    if (i < NV) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    if (NVALU) __builtin_amdgcn_sched_group_barrier(0x002, NVALU, 0);
    if (i >= NM - NW - 1 && i < NM - 1) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
  }
}

// K loop of the M16 tiles.  The three planes are consumed in three groups per stage so that only
// three plane sets are ever live (as the 32x32x16 loop's two k-group sets):
//   A: (mid, mid)                        read hi of this stage; global loads of stage kt + 2
//   B: (mid, hi), (hi, mid)              read lo of this stage; split + store stage kt + 1
//   C: barrier; (hi, hi), (lo, hi), (hi, lo)   read mid of stage kt + 1 (the freed mid set)
// Every product term of the x6 sum is the 32x32x16 loop's; only the summation order of the six
// terms into the fp32 accumulator differs (mid*mid first).
struct NoDma {
  static constexpr bool active = false, a_active = false;
  __device__ __forceinline__ void operator()(char*) const {}
};
template <class F, bool A = false>
struct DmaB {
  static constexpr bool active = true, a_active = A;  // B (and with A: the A operand too) by LDS-DMA
  F f;
  __device__ __forceinline__ void operator()(char* st) const { f(st); }
};
typedef __attribute__((address_space(3))) void lds_void;

// dmab(stage): VST_BF_GLDS_B's LDS-DMA of the B operand of the stage the K cursor points at into that
// stage's LDS image (a no-op otherwise), issued at the prologue and at the start of every step.
template <class T, class LoadAll, class Adv, class Prep, class DmaB>
__device__ __forceinline__ void main_loop16(char* smem, int nk, f32x4v (&acc)[T::MI16][T::NI16],
                                            float4 (&ra)[2][T::A_LD][2], u32x4_t (&rbv)[2][T::B_LD][T::NP],
                                            int rb, int kq, LoadAll load_all, Adv adv, Prep prep, DmaB dmab) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm0 = (wave / T::WAVES_N) * T::WM, wn0 = (wave % T::WAVES_N) * T::WN;
  if (nk <= 0) return;
  constexpr int NM = T::MI16 * T::NI16, NR = T::MI16 + T::NI16;
  constexpr int NV = T::A_LD * 2 + T::B_LD * T::NP, NW = T::A_LD * T::NP + T::B_LD * T::NP;
  if (VST_M16_PRIO && wave >= T::NW / 2) __builtin_amdgcn_s_setprio(1);
  dmab(smem);
  load_all(0);
  prep(0);
  store_stage<T>(smem, ra[0], rbv[0], rb, kq, !dmab.active, !dmab.a_active);
  adv(nk > 1);
  load_all(1);
  __syncthreads();
  Plane16<T> hi, mid, lo;
  read_plane16<T>(mid, smem, 1, wm0, wn0, lane);
  auto step = [&](int kt, auto par) __attribute__((always_inline)) {
    constexpr int P = decltype(par)::value;
    const char* cur = smem + P * T::STAGE;
    char* nxt = smem + (P ^ 1) * T::STAGE;
    constexpr bool SA = VST_M16_STORE == 1, RA = VST_M16_RDLO == 1;
    dmab(nxt);  // the cursor is on stage kt + 1 here (adv below moves it to kt + 2)
    if (VST_M16_LOADEARLY) {
      adv(kt + 2 < nk);
      load_all(P);
      __builtin_amdgcn_sched_barrier(0);
    }
    read_plane16<T>(hi, cur, 0, wm0, wn0, lane);
    if (RA) read_plane16<T>(lo, cur, 2, wm0, wn0, lane);
    if (!VST_M16_LOADEARLY) {
      adv(kt + 2 < nk);
      load_all(P);
    }
    if (SA) {
      prep(P ^ 1);
      store_stage<T>(nxt, ra[P ^ 1], rbv[P ^ 1], rb, kq, !dmab.active, !dmab.a_active);
    }
    mma16<T>(mid, mid, acc);
    if (VST_M16_SCHED) sched16<NM, RA ? 2 * NR : NR, NV, SA ? 4 : 0, SA ? NW : 0>();
    if (VST_M16_LOADFIRST) __builtin_amdgcn_sched_barrier(0);
    if (!RA) read_plane16<T>(lo, cur, 2, wm0, wn0, lane);
    if (!SA) {
      prep(P ^ 1);
      store_stage<T>(nxt, ra[P ^ 1], rbv[P ^ 1], rb, kq, !dmab.active, !dmab.a_active);
    }
    mma16<T>(mid, hi, acc);
    mma16<T>(hi, mid, acc);
    if (VST_M16_SCHED) sched16<2 * NM, RA ? 0 : NR, 0, SA ? 0 : 2, SA ? 0 : NW>();
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
    read_plane16<T>(mid, nxt, 1, wm0, wn0, lane);
    mma16<T>(hi, hi, acc);
    mma16<T>(lo, hi, acc);
    mma16<T>(hi, lo, acc);
    if (VST_M16_SCHED) sched16<3 * NM, NR, 0, 0, 0>();
  };
  int kt = 0;
  for (; kt + 1 < nk; kt += 2) {
    step(kt, std::integral_constant<int, 0>());
    step(kt + 1, std::integral_constant<int, 1>());
  }
  if (kt < nk) step(kt, std::integral_constant<int, 0>());
}

template <int MI, int NI>
__device__ __forceinline__ void zero_acc4(f32x4v (&acc)[MI][NI]) {
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};
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

// XCD-aware tile order for a 1-D grid of Mt*Nt tiles (xcd_tile, common.h).  Consecutive workgroup
// ids land on consecutive XCDs, so XCD x (= L % 8) gets a contiguous ~T/8 tile range in
// (m-major, n-minor) order: the N-tiles that share an A row block run together on one XCD and the
// XCD's resident working set is (CUs per XCD / Nt) M-tiles of activations, which stays in its L2.
__device__ __forceinline__ void tile_of(int L, int Mt, int Nt, int& mt, int& nt) {
  const int t = xcd_tile(L, Mt * Nt);
  mt = t / Nt;
  nt = t - mt * Nt;
}

// The InstanceNorm(+act) backward partials of the layer below a data gradient, taken by the GEMM's
// epilogue (vst_conv2d_dgrad_refl_in_epi): the stored output g (+ addend) is the IN output's gradient;
// z = the IN input [M][Cop] NHWC, st = its statistics [N][Cop][2] (mean, rstd); per 32-row group of an
// image (slice zg = group index) and channel the fp64 sums {sum g', sum g' xh, sum xh} (xh = (z - mean)
// rstd, g' = g act'(xh)) go to part[n][zg][Cop][3] — in_partial_k<1>'s per-element arithmetic, ns
// slices per image (the groups, then the border-correction slices of dgrad_border5_add_inb_k).
struct InbArgs {
  const float* z;
  const float* st;
  double* part;
  int act;
  float slope;
  int ns;
};

// g' = g act'(xh) of element (g, z) under (mean, rstd): in_partial_k<1>'s expression
__device__ __forceinline__ void inb_term(float g, float z, float mean, float rstd, int act, float slope, float& gd,
                                         float& xh) {
  xh = (z - mean) * rstd;
  float d = 1.f;
  if (act == VST_ACT_RELU) d = xh > 0.f ? 1.f : 0.f;
  else if (act == VST_ACT_LRELU) d = xh > 0.f ? 1.f : slope;
  gd = g * d;
}

// ---------------------------------------------------------- reflect-pad-1 data gradient border
// The data gradient of ReflectionPad2d(1) + 3x3 conv (stride 1) on an H x W map is
//   dx(j) = sum over padded positions q with r(q) = j of dxp(q),   r(-1) = 1, r(H) = H - 2,
// dxp = the full correlation of dy with the rotated taps (a 3x3 conv of dy with zero padding 2).
// The interior term dxp(j), j in H x W, is the zero-pad-1 forward conv over dy (one exact grid: for
// N = 8 at 64 x 64 the 256x128 tiles make one whole CU round).  The 2(H+W)+4 padded border
// positions q add into the rows / columns 1 and H-2 / W-2: this map orders them per image as
//   rows [0, S):   single targets — top (q = (-1, w)), bottom (q = (H, w)) for w not in {1, W-2},
//                  then left (q = (h, -1)), right (q = (h, W)) for h not in {1, H-2};
//   rows [S, S4):  padding to a multiple of 4 (no position);
//   rows S4 + 4g + {0, 1, 2}: the three positions of corner target g (g: (1,1), (1,W-2), (H-2,1),
//                  (H-2,W-2)), + 4g + 3 none — a 4-row group sits in one lane's accumulator rows.
// S = 2 (W - 2) + 2 (H - 2), S4 = S rounded up to a multiple of 4, rows per image S4 + 16.
// (qh, qw) = the padded position (-100 for none: every tap gathers zeros), (th, tw) its target.
__host__ __device__ __forceinline__ int dgrad_border_rows(int H, int W) {
  return ((2 * (W - 2) + 2 * (H - 2) + 3) / 4) * 4 + 16;
}

__host__ __device__ __forceinline__ void dgrad_border_pos(int b, int H, int W, int& qh, int& qw, int& th, int& tw) {
  const int sw = W - 2, sh = H - 2, S = 2 * sw + 2 * sh, S4 = (S + 3) / 4 * 4;
  qh = qw = th = tw = -100;
  if (b < 2 * sw) {  // top / bottom
    const int k = b < sw ? b : b - sw;
    tw = k == 0 ? 0 : (k == sw - 1 ? W - 1 : k + 1);
    qw = tw;
    qh = b < sw ? -1 : H;
    th = b < sw ? 1 : H - 2;
    return;
  }
  if (b < S) {  // left / right
    const int b2 = b - 2 * sw, k = b2 < sh ? b2 : b2 - sh;
    th = k == 0 ? 0 : (k == sh - 1 ? H - 1 : k + 1);
    qh = th;
    qw = b2 < sh ? -1 : W;
    tw = b2 < sh ? 1 : W - 2;
    return;
  }
  if (b < S4) return;
  const int g = (b - S4) >> 2, r = (b - S4) & 3;
  if (r == 3) return;
  const int top = g < 2, left = (g & 1) == 0;
  th = top ? 1 : H - 2;
  tw = left ? 1 : W - 2;
  const int ph = top ? -1 : H, pw = left ? -1 : W;  // the out-of-frame row / column
  if (r == 0) { qh = ph; qw = tw; }
  else if (r == 1) { qh = ph; qw = pw; }
  else { qh = th; qw = pw; }
}

// dx[n][th][tw][c] += the border rows' GEMM result (split slabs summed in order); a corner target's
// three rows are summed in row order by one thread.  grid (ceil(N*NB / 16), ceil(C / 64)): thread
// (one of 16 rows, 4-channel group); every dx element has exactly one writer.  The slab loads of a
// row are issued together (up to 16 splits in flight per thread).
__global__ __launch_bounds__(256) void dgrad_border_add_k(const float* __restrict__ slab, int ks, int Mb, int C,
                                                          float* __restrict__ dx, int H, int W, int NB) {
  const int t = threadIdx.x;
  const int c = blockIdx.y * 64 + (t & 15) * 4;
  const int m = blockIdx.x * 16 + (t >> 4);
  if (m >= Mb || c >= C) return;
  const int n = m / NB, b = m - n * NB;
  int qh, qw, th, tw;
  dgrad_border_pos(b, H, W, qh, qw, th, tw);
  if (th < 0) return;
  const int S4 = NB - 16;
  if (b >= S4 && ((b - S4) & 3) != 0) return;
  const int nr = b >= S4 ? 3 : 1;
  const long zst = (long)Mb * C;
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int r = 0; r < nr; ++r) {
    const float* base = slab + (long)(m + r) * C + c;
    float4 u[16];
#pragma unroll
    for (int z = 0; z < 16; ++z)
      if (z < ks) u[z] = *reinterpret_cast<const float4*>(base + z * zst);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int z = 0; z < 16; ++z)
      if (z < ks) add_f4(acc, u[z]);
    add_f4(v, acc);
  }
  float4* d = reinterpret_cast<float4*>(dx + (((long)n * H + th) * W + tw) * C + c);
  float4 o = *d;
  add_f4(o, v);
  *d = o;
}

// The K-restricted border GEMM (conv_fprop_bf_k REFL 5): the padded positions as four segments of
// rows, each padded to a whole number of M-tiles:
//   top    [0, Lt):            image n, k in [0, W+2): q = (-1, k-1)  (the two corners included)
//   bottom [Lt, 2Lt):          q = (H, k-1)
//   left   [2Lt, 2Lt+Ll):      image n, k in [0, H):   q = (k, -1)
//   right  [2Lt+Ll, 2Lt+2Ll):  q = (k, W)
// A top / bottom row reads only dy row 0 / H-1 (taps (2, s) / (0, s)), a left / right row only dy
// column 0 / W-1 (taps (r, 2) / (r, 0)): K = 3 C instead of 9 C (the other six taps of a border
// position gather zeros).  Lt = N (W+2), Ll = N H, each rounded up to the tile height bm.
__host__ __device__ __forceinline__ int border5_seg_rows(int n_img, int len, int bm) {
  return (n_img * len + bm - 1) / bm * bm;
}

// dx[n][th][tw][c] += the sum of the REFL-5 slab rows whose position mirrors onto (th, tw): the
// targets are rows 1 / H-2 (all columns), then columns 1 / W-2 (rows not 1 / H-2), T = 2W + 2H per
// image; a target sums its (1..3) rows in a fixed order (top / bottom rows by column, then the left
// / right row), each row's splits in order.  grid (ceil(N*T / 16), ceil(C / 64)), thread = (target,
// 4-channel group); every dx element has exactly one writer.
__global__ __launch_bounds__(256) void dgrad_border5_add_k(const float* __restrict__ slab, int ks, int Mb, int C,
                                                           float* __restrict__ dx, int N, int H, int W, int Lt,
                                                           int Ll) {
  const int t = threadIdx.x;
  const int c = blockIdx.y * 64 + (t & 15) * 4;
  const int T = 2 * W + 2 * H;
  const int m = blockIdx.x * 16 + (t >> 4);
  if (m >= N * T || c >= C) return;
  const int n = m / T, b = m - n * T;
  int th, tw;
  if (b < 2 * W) {
    th = b < W ? 1 : H - 2;
    tw = b < W ? b : b - W;
  } else {
    const int b2 = b - 2 * W;
    th = b2 < H ? b2 : b2 - H;
    tw = b2 < H ? 1 : W - 2;
    if (th == 1 || th == H - 2) return;  // a row target
  }
  int rows[3];
  const int nr = dgrad_border_slab_rows(n, th, tw, H, W, Lt, Ll, rows);
  const long zst = (long)Mb * C;
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int r = 0; r < nr; ++r) {
    const float* base = slab + (long)rows[r] * C + c;
    float4 u[16];
#pragma unroll
    for (int z = 0; z < 16; ++z)
      if (z < ks) u[z] = *reinterpret_cast<const float4*>(base + z * zst);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int z = 0; z < 16; ++z)
      if (z < ks) add_f4(acc, u[z]);
    add_f4(v, acc);
  }
  float4* d = reinterpret_cast<float4*>(dx + (((long)n * H + th) * W + tw) * C + c);
  float4 o = *d;
  add_f4(o, v);
  *d = o;
}

// dgrad_border5_add_k with the IN-backward partials' border correction (vst_conv2d_dgrad_refl_in_epi): the
// interior GEMM's epilogue summed g' of the pre-border g over every pixel (InbArgs), so a target whose
// g moves from g0 to g1 = g0 + its slab sum adds (g1' - g0') and (g1' - g0') xh (fp64, from the fp32 g'
// products) to the partials.  grid (ceil(T / 16), N, ceil(C / 64)), T = 2W + 2H targets per image: a block
// takes 16 targets of one image; its 16 target-threads' sums fold through LDS in a fixed order into
// slice first_slice + blockIdx.x of part (sum xh gets 0: the border add leaves z alone).
__device__ __forceinline__ void border5_target(int b, int W, int H, int& th, int& tw, bool& live) {
  live = true;
  if (b < 2 * W) {
    th = b < W ? 1 : H - 2;
    tw = b < W ? b : b - W;
  } else {
    const int b2 = b - 2 * W;
    th = b2 < H ? b2 : b2 - H;
    tw = b2 < H ? 1 : W - 2;
    if (th == 1 || th == H - 2) live = false;  // a row target
  }
}

__global__ __launch_bounds__(256) void dgrad_border5_add_inb_k(const float* __restrict__ slab, int ks, int Mb, int C,
                                                               float* __restrict__ dx, int H, int W, int Lt, int Ll,
                                                               InbArgs inb, int first_slice) {
  __shared__ double red[2][16][65];
  const int t = threadIdx.x, c4 = (t & 15) * 4, sub = t >> 4;
  const int c = blockIdx.z * 64 + c4, n = blockIdx.y;
  const int T = 2 * W + 2 * H;
  const int b = blockIdx.x * 16 + sub;
  double a0[4] = {0, 0, 0, 0}, a1[4] = {0, 0, 0, 0};
  int th = 0, tw = 0;
  bool live = false;
  if (b < T && c < C) border5_target(b, W, H, th, tw, live);
  if (live) {
    int rows[3];
    const int nr = dgrad_border_slab_rows(n, th, tw, H, W, Lt, Ll, rows);
    const long zst = (long)Mb * C;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int r = 0; r < nr; ++r) {
      const float* base = slab + (long)rows[r] * C + c;
      float4 u[16];
#pragma unroll
      for (int z = 0; z < 16; ++z)
        if (z < ks) u[z] = *reinterpret_cast<const float4*>(base + z * zst);
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int z = 0; z < 16; ++z)
        if (z < ks) add_f4(acc, u[z]);
      add_f4(v, acc);
    }
    const long e = (((long)n * H + th) * W + tw) * C + c;
    float4* d = reinterpret_cast<float4*>(dx + e);
    const float4 o0 = *d;
    float4 o = o0;
    add_f4(o, v);
    *d = o;
    const float4 zz = *reinterpret_cast<const float4*>(inb.z + e);
    const float4 s0 = reinterpret_cast<const float4*>(inb.st)[((long)n * C + c) / 2];
    const float4 s1 = reinterpret_cast<const float4*>(inb.st)[((long)n * C + c) / 2 + 1];
    const float mu[4] = {s0.x, s0.z, s1.x, s1.z}, rs[4] = {s0.y, s0.w, s1.y, s1.w};
    const float g0[4] = {o0.x, o0.y, o0.z, o0.w}, g1[4] = {o.x, o.y, o.z, o.w}, zv[4] = {zz.x, zz.y, zz.z, zz.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float d0, d1, xh;
      inb_term(g0[k], zv[k], mu[k], rs[k], inb.act, inb.slope, d0, xh);
      inb_term(g1[k], zv[k], mu[k], rs[k], inb.act, inb.slope, d1, xh);
      a0[k] = (double)d1 - (double)d0;
      a1[k] = (double)d1 * xh - (double)d0 * xh;
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    red[0][sub][c4 + k] = a0[k];
    red[1][sub][c4 + k] = a1[k];
  }
  __syncthreads();
  if (t < 192) {
    const int v = t >> 6, cc = t & 63, nn = blockIdx.z * 64 + cc;
    if (nn >= C) return;
    double acc = 0.0;
    if (v < 2)
      for (int q = 0; q < 16; ++q) acc += red[v][q][cc];
    inb.part[(((long)n * inb.ns + first_slice + blockIdx.x) * C + nn) * 3 + v] = acc;
  }
}

// ------------------------------------------------------------------------ ConvTranspose phases
// Stride-2 ConvTranspose2d(k3, p1, op1) as four phase convs (vst_interleave_phases): phase (a, b) =
// oph - 1 = 2a + b is an (H+a) x (W+b) conv whose pixel (ph, pw) is output pixel (2(ph-a)+a,
// 2(pw-b)+b) of the 2H x 2W result, its first row (a = 1) / column (b = 1) unused.  With oph > 0 the
// forward kernel stores each row there directly: -1 = the unused row / column (not stored).
// oph 5..8 (oph - 5 = 2a + b): the data gradient of Conv2d(k4, s2, p1) (vst_conv4s2_dgrad): every
// phase is an (H+1) x (W+1) conv with the same map, its row H / column W (a = 0, b = 0) or its first
// row / column (a = 1, b = 1) unused.
__device__ __forceinline__ int phase_row(int mm, int oph, int Ho, int Wo) {
  const bool full = oph > 4;
  const int q = full ? oph - 5 : oph - 1, a = q >> 1, b = q & 1;
  const int hw = Ho * Wo, n = mm / hw, rem = mm - n * hw, ph = rem / Wo, pw = rem - ph * Wo;
  const int H = full ? Ho - 1 : Ho - a, W = full ? Wo - 1 : Wo - b;
  const int i = ph - a, j = pw - b;
  if (i < 0 || j < 0 || i >= H || j >= W) return -1;
  return (n * 2 * H + 2 * i + a) * 2 * W + 2 * j + b;
}

// ------------------------------------------------------------------------------------------ fprop
// Target of every masked A gather (zero-padding taps, the K tail): loads from it return zeros, so
// the stage writer needs no per-row select.  Never written.
__device__ __attribute__((aligned(256))) float g_zero_page[64];

// y[m = (n, ho, wo)][co] = act(sum_k x_gather[m][k] * w[co][k] + bias[co]),  k = (r, s, ci);
// requires C % 8 == 0 (a thread's 8-deep chunk stays inside one tap).  ws = pre-split weight planes
// of the VST_PACK_OK matrix [Cop][R*S*C], plane stride wps elements.
//
// KSL (C % BK == 0): K-steps walk the R*S taps of one BK-channel slice, then the next slice, so one
// slice of the block's activation rows is reused by all taps while it is L2-resident (tap-major
// order streams the whole C-deep block through L2 once per tap: 289 -> 96 MB HBM traffic per N=8
// ResnetBlock launch on the 256x128 tiles; the 128x128 dgrad tiles fetched 356 MB per launch tap-
// major).  The K cursor (tap, slice) is block-uniform, so it lives in scalar registers; only the
// per-row pixel offsets are recomputed (one reflect / bounds map per row) when the tap changes.
// The weight planes keep their (r, s, ci) layout: the B offset of a step is (r*S + s)*C + slice.
// Without KSL (C not a multiple of BK: the image-input layers) the K-steps walk k = (r, s, ci) in
// order with a per-thread cursor.
// REFL: 0 = zero padding, 1 = reflect padding (compile-time, branch-free tap map), 2 = runtime
// `reflect` (the rarely used tap-major variants), 3 = as 2 for a 4-channel input (the image layers:
// 3 channels + 1 zero): a thread's 8-deep K chunk then spans two taps, the second one's rows have
// their own offsets (aoff2), and a K that ends half-way through a chunk (R*S odd) reads zeros for the
// missing tap.  K = R*S*4 instead of R*S*8 with the input padded to 8 channels: half the MFMA work.
// SPLIT (KSL only): split-K over the K-steps — block L = z * tiles + tile runs K-steps
// [z * spk, z * spk + spk) and stores its raw partial tile to slab[z][m - m_base][Cop]
// (fprop_splitk_reduce_k sums the splits in order and applies bias / act / IN partials).
// (body of conv_fprop_bf_k and conv_convT_phases_k; bid = the block's index in its tile grid)
template <class T, bool KSL, int REFL, bool SPLIT, bool APRE = false>
__device__ __forceinline__ void conv_fprop_bf_body(
    int bid, const float* __restrict__ x, const __bf16* __restrict__ ws, long wps, const float* __restrict__ bias,
    float* __restrict__ y, int H, int W, int C, int Ho, int Wo, int Cop, int S, int st, int padh,
    int padw, int reflect, int act, float slope, int M, int Ktot, int m_base, double* __restrict__ part,
    int spk, float* __restrict__ slab, const float* __restrict__ addend, int oph,
    InbArgs inb = InbArgs{}, const __bf16* __restrict__ apl = nullptr, long pps = 0) {
  static_assert(!SPLIT || KSL, "split-K needs the channel-slice-major K walk");
  static_assert(REFL < 4 || (SPLIT && KSL), "border rows run as split-K slabs");
  __shared__ __attribute__((aligned(16))) char smem[2 * T::STAGE];
  constexpr int A_LD = T::A_LD, B_LD = T::B_LD, RPP = T::RPP, NP = T::NP;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  int mt_, nt_;
  const int Mt_ = (M - m_base + T::BM - 1) / T::BM, Nt_ = (Cop + T::BN - 1) / T::BN;
  const int zs = SPLIT ? bid / (Mt_ * Nt_) : 0;
  tile_of(SPLIT ? bid - zs * Mt_ * Nt_ : bid, Mt_, Nt_, mt_, nt_);
  const int m0 = m_base + mt_ * T::BM, n0 = nt_ * T::BN;
  const int kq = t % T::KC, rb = t / T::KC;
  const float* zp = g_zero_page;

  // A rows (output pixels m0 + rb + RPP*j): tap-independent geometry.  Rows past M gather row 0's
  // pixels instead: their outputs are never stored, so no mask is needed for them.
  constexpr bool C4 = REFL == 3;
  // REFL 5 (dgrad_border5 rows: segment `seg` of the block; Ho / Wo = the padded top-bottom / left-right
  // segment lengths, st = images): K = the 3 taps that reach the frame, Sx of them per tap row
  const int seg = REFL != 5 ? 0 : (m0 < Ho ? 0 : (m0 < 2 * Ho ? 1 : (m0 < 2 * Ho + Wo ? 2 : 3)));
  const int Sx = REFL != 5 ? S : (seg < 2 ? 3 : 1);
  int hb[A_LD], wb[A_LD], pb[A_LD], aoff[A_LD], aoff2[C4 ? A_LD : 1];
#pragma unroll
  for (int j = 0; j < A_LD; ++j) {
    const int m = m0 + rb + RPP * j;
    const int mm = m < M ? m : 0;
    if constexpr (REFL == 5) {
      const int L = seg < 2 ? W + 2 : H;
      const int r = mm - (seg == 0 ? 0 : (seg == 1 ? Ho : (seg == 2 ? 2 * Ho : 2 * Ho + Wo)));
      const int n = r / L, k = r - n * L;
      const bool live = (unsigned)r < (unsigned)(st * L);  // the segment's padding rows gather zeros
      hb[j] = !live ? -1000000 : (seg == 0 ? 0 : (seg == 1 ? H - 1 : k - 1));
      wb[j] = seg < 2 ? k - 2 : (seg == 2 ? 0 : W - 1);
      pb[j] = live ? n * H * W * C : 0;
      continue;
    }
    if constexpr (REFL == 4) {
      // border rows of a reflect-pad-1 data gradient (dgrad_border_pos): Wo = rows per image
      const int n = mm / Wo;
      int qh, qw, th, tw;
      dgrad_border_pos(mm - n * Wo, H, W, qh, qw, th, tw);
      hb[j] = qh - padh;
      wb[j] = qw - padw;
      pb[j] = n * H * W * C;
      continue;
    }
    const int hw = Ho * Wo;
    const int n = mm / hw, rem = mm - n * hw, ho = rem / Wo, wo = rem - ho * Wo;
    hb[j] = ho * st - padh;
    wb[j] = wo * st - padw;
    pb[j] = n * H * W * C;
  }
  // element offset of row j's pixel under tap (kr, ks), -1 where the tap reads zero padding
  const bool refl = REFL >= 2 ? reflect != 0 : REFL == 1;
  const int WC = W * C;
  auto tap_rows_to = [&](int* dst, int kr, int ks) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < A_LD; ++j) {
      int hi = hb[j] + kr, wi = wb[j] + ks;
      if (refl) {
        hi = reflect_idx(hi, H);
        wi = reflect_idx(wi, W);
        dst[j] = pb[j] + __mul24(hi, WC) + __mul24(wi, C);
      } else {
        const bool ok = (unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W;
        dst[j] = ok ? pb[j] + __mul24(hi, WC) + __mul24(wi, C) : -1;
      }
    }
  };
  // C4: the chunk's second tap is the one after (kr, ks) (past the last tap it is never read)
  auto tap_rows = [&](int kr, int ks) __attribute__((always_inline)) {
    tap_rows_to(aoff, kr, ks);
    if constexpr (C4) {
      const bool wrap = ks + 1 == S;
      tap_rows_to(aoff2, wrap ? kr + 1 : kr, wrap ? 0 : ks + 1);
    }
  };
  // B rows (output channels n0 + rb + RPP*j); channels past Cop read row Cop-1 (never stored)
  const __bf16* wrow[B_LD];
#pragma unroll
  for (int j = 0; j < B_LD; ++j) {
    const int n = n0 + rb + RPP * j;
    wrow[j] = ws + (long)(n < Cop ? n : Cop - 1) * (REFL == 5 ? 3 * Ktot : Ktot);
  }

  // K cursor.  KSL: block-uniform (tap r, tap s, slice base) + this thread's chunk 8*kq.
  // Otherwise: per-thread absolute k (kcur) with its channel kc and tap (kr, ks).
  const int kq8 = 8 * kq;
  int tr = 0, ts = 0, ksb = 0;                 // KSL
  int kcur = kq8, kc = kq8 % C, kr = 0, ks = 0;  // tap-major
  const int Rk = KSL ? Ktot / (Sx * C) : 0;
  const int nk_all = (Ktot + T::BK - 1) / T::BK;
  int k0 = 0, nk = nk_all;
  if (SPLIT) {  // K-steps [k0, k0 + nk): slice k0 / (R S), tap k0 % (R S)
    k0 = zs * spk;
    nk = min(spk, nk_all - k0);
    const int taps = Rk * Sx, tap = k0 % taps;
    tr = tap / Sx;
    ts = tap - tr * Sx;
    ksb = (k0 / taps) * T::BK;
  }
  if (KSL) {
    tap_rows(tr, ts);
  } else {
    const int rs = kq8 / C;
    kr = rs / S;
    ks = rs - kr * S;
    tap_rows(kr, ks);
  }

  float4 ra[2][A_LD][2];
  u32x4_t rbv[2][B_LD][NP];
  constexpr bool GLDS = VST_BF_GLDS_B && T::M16 && KSL && !C4 && REFL != 5;
  // APRE: the A operand arrives pre-split (apl: three bf16 planes of x's NHWC layout, plane stride pps
  // elements) by LDS-DMA like B — no fp32 A image, no split in the staging.  VST_BF_FAKE_ADMA (developer timing
  // only, WRONG results): every GLDS kernel DMAs A from x's own bytes read as planes.
  constexpr bool GLDS_A = (APRE || VST_BF_FAKE_ADMA) && GLDS;
  // APRE without the DMA (the K-restricted border GEMM, REFL 5): A's planes loaded into registers and put back
  // together as fp32 (hi + mid + lo is the value exactly), then staged as usual — the same planes in LDS
  constexpr bool APRE_REG = APRE && !GLDS_A;
  static_assert(!APRE || GLDS_A || REFL == 5, "pre-split A: the x6 M16 channel-slice kernels with LDS-DMA B, or REFL 5");
  const __bf16* apl_ = VST_BF_FAKE_ADMA ? reinterpret_cast<const __bf16*>(x) : apl;
  const long pps_ = VST_BF_FAKE_ADMA ? (long)(M / (Ho * Wo)) * H * W * C / 2 : pps;
  auto load_all = [&](int set) __attribute__((always_inline)) {
    const bool kin = KSL || kcur < Ktot;  // the K tail reads zeros (A) against row 0 (B)
    const int ka = KSL ? ksb + kq8 : kc;
    // REFL 5: tap (2, ts) top, (0, ts) bottom, (tr, 2) left, (tr, 0) right of the 3x3 weight rows
    const int tap5 = seg == 0 ? 6 + ts : (seg == 1 ? ts : 3 * tr + (seg == 2 ? 2 : 0));
    const int kb = KSL ? (REFL == 5 ? tap5 : tr * S + ts) * C + ksb + kq8 : (kin ? kcur : 0);
    if constexpr (C4) {
      // chunk = taps kcur/4 and kcur/4 + 1; the second is missing when kcur + 4 == Ktot.  Weight rows
      // are 4*R*S bf16 long (8-byte aligned for odd R*S): two 8-byte loads per plane.
      const bool kin2 = kcur + 4 < Ktot;
#pragma unroll
      for (int j = 0; j < A_LD; ++j) {
        const float* p0 = (kin && aoff[j] >= 0) ? x + aoff[j] : zp;
        const float* p1 = (kin2 && aoff2[j] >= 0) ? x + aoff2[j] : zp;
        ra[set][j][0] = *reinterpret_cast<const float4*>(p0);
        ra[set][j][1] = *reinterpret_cast<const float4*>(p1);
      }
      const __bf16* zb = reinterpret_cast<const __bf16*>(zp);
#pragma unroll
      for (int j = 0; j < B_LD; ++j) {
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          const __bf16* q = wrow[j] + p * wps + kb;
          const uint2 lo = *reinterpret_cast<const uint2*>(q);
          const uint2 hi = *reinterpret_cast<const uint2*>(kin2 ? q + 4 : zb);
          rbv[set][j][p] = u32x4_t{lo.x, lo.y, hi.x, hi.y};
        }
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < A_LD; ++j) {
      if constexpr (GLDS_A) break;  // A arrives by LDS-DMA (dma_b)
      // FAKE_ZA 1: every A gather from the zero page; 2: all but the first tap of each channel slice
      // (only the L2-miss-prone loads stay real); 3: only the first tap's loads from the zero page
      const bool tap0 = KSL && tr == 0 && ts == 0;
      // 4: every row reads the first pixel's channel slice (real, changing values, one cache line)
      const bool fake = VST_BF_FAKE_ZA == 1 || (VST_BF_FAKE_ZA == 2 && !tap0) || (VST_BF_FAKE_ZA == 3 && tap0);
      if constexpr (APRE_REG) {
        const bool live = kin && aoff[j] >= 0;
        const __bf16* q = live ? apl + aoff[j] + ka : reinterpret_cast<const __bf16*>(zp);
        const long ps = live ? pps : 0;
        const u32x4_t h = *reinterpret_cast<const u32x4_t*>(q), m = *reinterpret_cast<const u32x4_t*>(q + ps),
                      l = *reinterpret_cast<const u32x4_t*>(q + 2 * ps);
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[2 * e] = (__uint_as_float(h[e] << 16) + __uint_as_float(m[e] << 16)) + __uint_as_float(l[e] << 16);
          v[2 * e + 1] = (__uint_as_float(h[e] & 0xffff0000u) + __uint_as_float(m[e] & 0xffff0000u)) +
                         __uint_as_float(l[e] & 0xffff0000u);
        }
        ra[set][j][0] = make_float4(v[0], v[1], v[2], v[3]);
        ra[set][j][1] = make_float4(v[4], v[5], v[6], v[7]);
        continue;
      }
      const float* p = (kin && aoff[j] >= 0 && !fake) ? x + (VST_BF_FAKE_ZA == 4 ? 0 : aoff[j]) + ka : zp;
      ra[set][j][0] = *reinterpret_cast<const float4*>(p);
      ra[set][j][1] = *reinterpret_cast<const float4*>(p + 4);
    }
    if constexpr (GLDS) return;  // B arrives by LDS-DMA (dma_b)
#pragma unroll
    for (int j = 0; j < B_LD; ++j) {
#pragma unroll
      for (int p = 0; p < NP; ++p)
        rbv[set][j][p] = *reinterpret_cast<const u32x4_t*>(
            VST_BF_FAKE_ZB == 1 ? reinterpret_cast<const __bf16*>(zp)
                                : (VST_BF_FAKE_ZB == 2 ? ws : wrow[j]) + p * wps + kb);  // 2: weight row 0 for every row
    }
  };
  // VST_BF_GLDS_B: the B image of the stage the cursor is on, one global_load_lds_dwordx4 per (row
  // block, plane) and wave — a wave fills 16 whole 64-B rows (1 KiB, lane-linear): lane l's 16 B land
  // at row 16 w + l / 4, slot l % 4, so it reads source chunk (l % 4) ^ swz(row) (the LDS image's
  // chunk swizzle applied on the source address)
  auto dma_b = [&](char* st) __attribute__((always_inline)) {
    if constexpr (GLDS_A) {  // the A rows of the stage (row rb + RPP j: this thread's aoff[j]), planes apl_
      const __bf16* zb = reinterpret_cast<const __bf16*>(zp);
#pragma unroll
      for (int j = 0; j < A_LD; ++j) {
        const int row = rb + RPP * j;
        const int csrc = (t % T::KC) ^ T::swz(row);
        const int wrow0 = __builtin_amdgcn_readfirstlane(row - (lane / T::KC));
        const bool live = aoff[j] >= 0;
        const __bf16* src = live ? apl_ + aoff[j] + ksb + 8 * csrc : zb + 8 * csrc;
#pragma unroll
        for (int p = 0; p < NP; ++p) {
#if defined(__HIP_DEVICE_COMPILE__)
          __builtin_amdgcn_global_load_lds(src + (live ? p * pps_ : 0), (lds_void*)(st + p * T::A_PLANE + wrow0 * T::ROWB),
                                           16, 0, 0);
#endif
        }
      }
    }
    const int kbase = (tr * S + ts) * C + ksb;
#pragma unroll
    for (int j = 0; j < B_LD; ++j) {
      const int row = rb + RPP * j;
      const int csrc = (t % T::KC) ^ T::swz(row);
      const int wrow0 = __builtin_amdgcn_readfirstlane(row - (lane / T::KC));  // the wave's first row
#pragma unroll
      for (int p = 0; p < NP; ++p) {
#if defined(__HIP_DEVICE_COMPILE__)  // (a device builtin: the host pass only parses this body)
        __builtin_amdgcn_global_load_lds(wrow[j] + p * wps + kbase + 8 * csrc,
                                         (lds_void*)(st + T::A_BYTES + p * T::B_PLANE + wrow0 * T::ROWB), 16, 0, 0);
#endif
      }
    }
  };
  // go = false (the last two stages): the cursor stays on the final stage.  KSL: branch-free
  // (scalar selects), so the stage body stays one basic block for the scheduler.
  auto adv = [&](bool go) __attribute__((always_inline)) {
    if (KSL) {
      const int ts1 = ts + 1;
      const bool w1 = ts1 == Sx;
      const int tr1 = tr + (w1 ? 1 : 0);
      const bool w2 = w1 && tr1 == Rk;
      ts = go ? (w1 ? 0 : ts1) : ts;
      tr = go ? (w2 ? 0 : tr1) : tr;
      ksb = go ? ksb + (w2 ? T::BK : 0) : ksb;
      tap_rows(tr, ts);
      return;
    }
    if (!go) return;
    kcur += T::BK;
    kc += T::BK;
    if (kc >= C) {
      do {
        kc -= C;
        if (++ks == S) { ks = 0; ++kr; }
      } while (kc >= C);
      tap_rows(kr, ks);
    }
  };

  // the main loops' per-register-set hook before the split (unused by the forward)
  auto prep = [](int) __attribute__((always_inline)) {};
  const int wm0 = (wave / T::WAVES_N) * T::WM, wn0 = (wave % T::WAVES_N) * T::WN;
  if constexpr (T::M16) {
    f32x4v acc[T::MI16][T::NI16];
    zero_acc4(acc);
    if constexpr (GLDS)
      main_loop16<T>(smem, nk, acc, ra, rbv, rb, kq, load_all, adv, prep, DmaB<decltype(dma_b), GLDS_A>{dma_b});
    else
      main_loop16<T>(smem, nk, acc, ra, rbv, rb, kq, load_all, adv, prep, NoDma{});
    if constexpr (SPLIT) {
      float* sl = slab + (long)zs * (M - m_base) * Cop;
#pragma unroll
      for (int i = 0; i < T::MI16; ++i)
#pragma unroll
        for (int j = 0; j < T::NI16; ++j) {
          const int n = n0 + wn0 + 16 * j + (lane & 15);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int mm = m0 + wm0 + 16 * i + 4 * (lane >> 4) + r;
            if (n < Cop && mm < M) sl[(long)(mm - m_base) * Cop + n] = acc[i][j][r];
          }
        }
      return;
    }
    // 16x16 blocks: lane holds column lane & 15, rows 4 (lane >> 4) + r.  IN partials per 32-row
    // group (block pair 2g, 2g+1): per-lane fixed-order fp64 sums, then over the four lanes of a
    // column (xor 16, xor 32).
    // LDS_EPI: the activated tile goes to LDS (row stride BN + 16 floats: the two rows of a 32-lane
    // write group land 16 banks apart) and leaves as whole float4 rows (coalesced stores).
    // (an addend — the residual gradient of a data gradient — is always added on this path: its float4
    // loads ride with the row stores instead of 4-byte reads per accumulator element)
    constexpr bool LFIT = T::BM * (T::BN + 16) * 4 <= 2 * T::STAGE;
    const bool LEPI = LFIT && (VST_BF_LDS_EPI || addend != nullptr || oph != 0 || inb.part != nullptr);
    constexpr int LDE = T::BN + 16;
    float* ept = reinterpret_cast<float*>(smem);
    // InbArgs: the IN input z (and the addend) of the wave's 32-row group (wave w: rows 32 w .., one group per
    // wave) loaded before the tile goes through LDS, so their latency overlaps the staging
    constexpr int IC4 = T::BN / 4, IRW = 64 / (IC4 > 0 ? IC4 : 1);
    constexpr bool IOK = LFIT && 64 % IC4 == 0 && T::BM == 32 * T::NW && IC4 >= 4;
    float4 izr[IOK ? 32 / IRW : 1], iar[IOK ? 32 / IRW : 1];
    if constexpr (IOK) {
      if (inb.part) {
        const int n = n0 + 4 * (lane % IC4);
#pragma unroll
        for (int k = 0; k < 32 / IRW; ++k) {
          const int mm = m0 + 32 * wave + lane / IC4 + IRW * k;
          const bool ok = n < Cop && mm < M;
          izr[k] = ok ? *reinterpret_cast<const float4*>(inb.z + (long)mm * Cop + n) : make_float4(0.f, 0.f, 0.f, 0.f);
          iar[k] = (ok && addend) ? *reinterpret_cast<const float4*>(addend + (long)mm * Cop + n)
                                  : make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    }
    if (LEPI) __syncthreads();  // every wave is done reading the last stage
#pragma unroll
    for (int g = 0; g < T::MI16 / 2; ++g)
#pragma unroll
      for (int j = 0; j < T::NI16; ++j) {
        const int n = n0 + wn0 + 16 * j + (lane & 15);
        const bool nok = n < Cop;
        const float bv = (bias && nok) ? bias[n] : 0.f;
        double s1 = 0.0, s2 = 0.0;
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int mm = m0 + wm0 + 16 * (2 * g + h) + 4 * (lane >> 4) + r;
            const float ad = (!LEPI && addend && nok && mm < M) ? addend[(long)mm * Cop + n] : 0.f;
            const float v = apply_act(acc[2 * g + h][j][r] + bv, act, slope) + ad;
            if (LEPI)
              ept[(mm - m0) * LDE + (n - n0)] = v;
            else if (nok && mm < M && (!oph || phase_row(mm, oph, Ho, Wo) >= 0))
              y[(long)(oph ? phase_row(mm, oph, Ho, Wo) : mm) * Cop + n] = v;
            s1 += v;
            s2 += (double)v * v;
          }
        if (part) {
          s1 += __shfl_xor(s1, 16);
          s2 += __shfl_xor(s2, 16);
          s1 += __shfl_xor(s1, 32);
          s2 += __shfl_xor(s2, 32);
          const int g0 = m0 + wm0 + 32 * g;
          if (lane < 16 && nok && g0 < M) {
            const int hw = Ho * Wo, img = g0 / hw, z = (g0 - img * hw) >> 5;
            double* d = part + (((long)img * (hw >> 5) + z) * Cop + n) * 2;
            d[0] = s1;
            d[1] = s2;
          }
        }
      }
    if (LEPI) {
      __syncthreads();
      constexpr int C4 = T::BN / 4;
      if constexpr (IOK) {
        if (inb.part) {
          // IN-backward partials (InbArgs): wave w stores the 32-row group w (z / addend prefetched above);
          // lane l owns channels 4 (l % C4) .. + 3 and rows l / C4 + RW k of the group (whole 4*C4-float rows
          // per instruction, as the loop below); per-lane fixed-order fp64 sums, then xor over the RW lanes of
          // a channel group.  Every group lies in one image (HW % 32 == 0, checked by the launcher).
          constexpr int RW = IRW;
          const int c = 4 * (lane % C4), n = n0 + c, hw = Ho * Wo;
          const int gm0 = m0 + 32 * wave;
          if (gm0 < M) {
            const int img = gm0 / hw;
            float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0;
            if (n < Cop) {
              s0 = reinterpret_cast<const float4*>(inb.st)[((long)img * Cop + n) / 2];
              s1 = reinterpret_cast<const float4*>(inb.st)[((long)img * Cop + n) / 2 + 1];
            }
            const float mu[4] = {s0.x, s0.z, s1.x, s1.z}, rs[4] = {s0.y, s0.w, s1.y, s1.w};
            double a0[4] = {0, 0, 0, 0}, a1[4] = {0, 0, 0, 0}, a2[4] = {0, 0, 0, 0};
#pragma unroll
            for (int k = 0; k < 32 / RW; ++k) {
              const int row = 32 * wave + lane / C4 + RW * k, mm = m0 + row;
              if (n < Cop && mm < M) {
                float4 v = *reinterpret_cast<const float4*>(ept + row * LDE + c);
                add_f4(v, iar[k]);
                *reinterpret_cast<float4*>(y + (long)mm * Cop + n) = v;
                const float gv[4] = {v.x, v.y, v.z, v.w}, zv[4] = {izr[k].x, izr[k].y, izr[k].z, izr[k].w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  float gd, xh;
                  inb_term(gv[e], zv[e], mu[e], rs[e], inb.act, inb.slope, gd, xh);
                  a0[e] += gd;
                  a1[e] += (double)gd * xh;
                  a2[e] += xh;
                }
              }
            }
#pragma unroll
            for (int off = C4; off < 64; off <<= 1)
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                a0[e] += __shfl_xor(a0[e], off);
                a1[e] += __shfl_xor(a1[e], off);
                a2[e] += __shfl_xor(a2[e], off);
              }
            if (lane < C4 && n < Cop) {
              double* d = inb.part + (((long)img * inb.ns + ((gm0 - img * hw) >> 5)) * Cop + n) * 3;
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                d[3 * e] = a0[e];
                d[3 * e + 1] = a1[e];
                d[3 * e + 2] = a2[e];
              }
            }
          }
          return;
        }
      }
#pragma unroll 4
      for (int idx = t; idx < T::BM * C4; idx += T::NT) {
        const int row = idx / C4, c = 4 * (idx - row * C4);
        const int mm = m0 + row, n = n0 + c;
        const int orow = oph ? phase_row(mm, oph, Ho, Wo) : mm;
        if (mm < M && n < Cop && orow >= 0) {
          float4 v = *reinterpret_cast<const float4*>(ept + row * LDE + c);
          if (addend) add_f4(v, *reinterpret_cast<const float4*>(addend + (long)mm * Cop + n));
          *reinterpret_cast<float4*>(y + (long)orow * Cop + n) = v;
        }
      }
    }
    return;
  }
  f32x16 acc[T::MI][T::NI];
  zero_acc(acc);
  main_loop<T>(smem, nk, acc, ra, rbv, rb, kq, load_all, adv, prep);
  if constexpr (SPLIT) {
    float* sl = slab + (long)zs * (M - m_base) * Cop;
#pragma unroll
    for (int i = 0; i < T::MI; ++i)
#pragma unroll
      for (int j = 0; j < T::NI; ++j) {
        const int n = n0 + wn0 + 32 * j + (lane & 31);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int mm = m0 + wm0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (n < Cop && mm < M) sl[(long)(mm - m_base) * Cop + n] = acc[i][j][r];
        }
      }
    return;
  }

#pragma unroll
  for (int i = 0; i < T::MI; ++i)
#pragma unroll
    for (int j = 0; j < T::NI; ++j) {
      const int n = n0 + wn0 + 32 * j + (lane & 31);
      const bool nok = n < Cop;
      const float bv = (bias && nok) ? bias[n] : 0.f;
      double s1 = 0.0, s2 = 0.0;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int mm = m0 + wm0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const float ad = (addend && nok && mm < M) ? addend[(long)mm * Cop + n] : 0.f;
        const float v = apply_act(acc[i][j][r] + bv, act, slope) + ad;
        if (nok && mm < M && (!oph || phase_row(mm, oph, Ho, Wo) >= 0))
          y[(long)(oph ? phase_row(mm, oph, Ho, Wo) : mm) * Cop + n] = v;
        s1 += v;
        s2 += (double)v * v;
      }
      if (part) {
        // InstanceNorm statistics partials of this 32-row group (vst_conv2d_fwd_in): lanes l and
        // l ^ 32 hold the group's two row halves of column n; fixed order, fp64.  The launcher
        // guarantees Ho*Wo % 32 == 0, so a group never straddles an image or M.
        s1 += __shfl_xor(s1, 32);
        s2 += __shfl_xor(s2, 32);
        const int g0 = m0 + wm0 + 32 * i;
        if (lane < 32 && nok && g0 < M) {
          const int hw = Ho * Wo, img = g0 / hw, z = (g0 - img * hw) >> 5;
          double* d = part + (((long)img * (hw >> 5) + z) * Cop + n) * 2;
          d[0] = s1;
          d[1] = s2;
        }
      }
    }
}

// APRE: the A operand from apl (x's three bf16 planes, NHWC, plane stride pps elements) by LDS-DMA
template <class T, bool KSL, int REFL, bool SPLIT = false, bool APRE = false>
__global__ __launch_bounds__(T::NT, T::MINB) void conv_fprop_bf_k(
    const float* __restrict__ x, const __bf16* __restrict__ ws, long wps, const float* __restrict__ bias,
    float* __restrict__ y, int H, int W, int C, int Ho, int Wo, int Cop, int S, int st, int padh,
    int padw, int reflect, int act, float slope, int M, int Ktot, int m_base, double* __restrict__ part,
    int spk = 0, float* __restrict__ slab = nullptr, const float* __restrict__ addend = nullptr, int oph = 0,
    const __bf16* __restrict__ apl = nullptr, long pps = 0) {
  conv_fprop_bf_body<T, KSL, REFL, SPLIT, APRE>(blockIdx.x, x, ws, wps, bias, y, H, W, C, Ho, Wo, Cop, S, st, padh,
                                                padw, reflect, act, slope, M, Ktot, m_base, part, spk, slab, addend, oph,
                                                InbArgs{}, apl, pps);
}

// The interior conv of the reflect-pad-1 data gradient (+ addend) with the IN-backward partials of the
// layer below in its epilogue (InbArgs); M = the rows of this launch (whole 256x128 rounds).
template <class T, bool APRE = false>
__global__ __launch_bounds__(T::NT, T::MINB) void conv_fprop_bf_inb_k(
    const float* __restrict__ x, const __bf16* __restrict__ ws, long wps, float* __restrict__ y, int H, int W, int C,
    int Cop, const float* __restrict__ addend, int M, int Ktot, InbArgs inb, const __bf16* __restrict__ apl = nullptr,
    long pps = 0) {
  conv_fprop_bf_body<T, true, 0, false, APRE>(blockIdx.x, x, ws, wps, nullptr, y, H, W, C, H, W, Cop, 3, 1, 1, 1, 0,
                                              VST_ACT_NONE, 0.f, M, Ktot, 0, nullptr, 0, nullptr, addend, 0, inb, apl, pps);
}

// All four phases of a stride-2 ConvTranspose2d(k3, p1, op1) forward in ONE launch, each stored
// straight into the interleaved output (phase_row).  Phase (a, b) is the (1+a) x (1+b) zero-pad (a, b)
// conv over x whose (H+a) x (W+b) pixels map onto y's (2(ph-a)+a, 2(pw-b)+b).  Separately the phases
// are four launches of 256-265 tiles each at N=8 (u0: 256 -> 128 at 64x64 on 128x128 tiles): each
// a CU round plus a few stragglers, with K = 8-32 steps against its prologue / epilogue.  Here the
// grid is their concatenation, the 4-tap phase first (longest first), each job's range starting on a
// multiple of 8 so its XCD-aware tile order holds: ~4 rounds for the four.
struct PhaseJobs {
  const __bf16* ws[4];  // per job (launch order: phases 11, 01, 10, 00), the pack's bf16 planes
  int t0[5];            // job j's blocks [t0[j], t0[j] + tiles_j), t0[j] % 8 == 0; t0[4] = grid
};

// full: the four 2x2 pad-1 phase convs of a Conv2d(k4, s2, p1) data gradient (oph 5..8, (H+1) x (W+1) each)
template <class T>
__global__ __launch_bounds__(T::NT, T::MINB) void conv_convT_phases_k(const float* __restrict__ x, PhaseJobs jobs,
                                                                      const float* __restrict__ bias,
                                                                      float* __restrict__ y, int N, int H, int W,
                                                                      int C, int Cop, int act, float slope,
                                                                      int full) {
  const int bid = blockIdx.x;
  const int j = bid < jobs.t0[1] ? 0 : (bid < jobs.t0[2] ? 1 : (bid < jobs.t0[3] ? 2 : 3));
  const int ph = j == 0 ? 3 : (j == 1 ? 1 : (j == 2 ? 2 : 0));
  const int a = ph >> 1, b = ph & 1;
  const int t0 = j == 0 ? jobs.t0[0] : (j == 1 ? jobs.t0[1] : (j == 2 ? jobs.t0[2] : jobs.t0[3]));
  const __bf16* ws = j == 0 ? jobs.ws[0] : (j == 1 ? jobs.ws[1] : (j == 2 ? jobs.ws[2] : jobs.ws[3]));
  const int R = full ? 2 : 1 + a, S = full ? 2 : 1 + b, pah = full ? 1 : a, paw = full ? 1 : b;
  const int Ho = H + (full ? 1 : a), Wo = W + (full ? 1 : b), M = N * Ho * Wo, K = R * S * C;
  const int tiles = (M + T::BM - 1) / T::BM * ((Cop + T::BN - 1) / T::BN);
  if (bid - t0 >= tiles) return;  // the job's padding to a multiple of 8 blocks
  conv_fprop_bf_body<T, true, 0, false>(bid - t0, x, ws, (long)Cop * K, bias, y, H, W, C, Ho, Wo, Cop, S, 1, pah,
                                        paw, 0, act, slope, M, K, 0, nullptr, 0, nullptr, nullptr,
                                        (full ? 5 : 1) + 2 * a + b);
}

// -------------------------------------------------------------------------- weight gradient
// dW[m = (r, s, ci)][co] = sum_p X[shift_rs(p)][ci] * dY[p][co] over one split-K chunk of output
// pixels p, on the same stage / MMA machinery as the forward:
//   A rows (tap, ci): the padded channel-major fp32 copy xt = [Cx][N][Hp][Wp] of x (reflect / zero
//     border applied; stride 2: each padded row stored as its even then its odd columns), so a
//     thread's 8 consecutive output pixels (one output-row segment: Wo % 8 == 0) are 8 consecutive
//     words; split into bf16 planes in registers like the forward's activations;
//   B rows co: dY as NP pre-split bf16 planes [NP][Cyp][ldy] (nhwc_to_cp_planes_k), copied into the
//     stage image like the forward's weights.
// Replaces the [row][k] fp32-image kernel for the x6 arithmetic: that one split BOTH operands in
// registers for every K-step (the x shifted copy once per tap) and sat at ~0.33 of the x6 ceiling.
// The split-K chunk index comes from an XCD-aware 1-D grid (every tile of one chunk on one XCD, so
// its x / dy rows stay in that XCD's L2); partial tiles land in slab[z][m][Cyp].
// W1 (Wo >= BK): a K-step crosses at most one output-row end, so the pixel cursor advances with
// selects only and the two-stage loop body stays one basic block (as the forward's KSL cursor).
template <class T, bool W1>
__global__ __launch_bounds__(T::NT, T::MINB) void conv_wgrad_bf_k(
    const float* __restrict__ xt, const __bf16* __restrict__ dyp, long dps, float* __restrict__ slab, int H,
    int W, int Cx, int Ho, int Wo, int Cyp, int S, int pad, int st, int Mw, int P, int chunk, long ldx,
    long ldy) {
  __shared__ __attribute__((aligned(16))) char smem[2 * T::STAGE];
  constexpr int A_LD = T::A_LD, B_LD = T::B_LD, RPP = T::RPP, NP = T::NP;
  typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int Mt = (Mw + T::BM - 1) / T::BM, Nt = (Cyp + T::BN - 1) / T::BN, Zt = (P + chunk - 1) / chunk;
  int mx, ny, zz;
  {
    const int tt = xcd_tile(blockIdx.x, Mt * Nt * Zt);
    zz = tt / (Mt * Nt);
    const int rem = tt - zz * Mt * Nt;
    ny = rem / Mt;
    mx = rem - ny * Mt;
  }
  const int m0 = mx * T::BM, n0 = ny * T::BN;
  const int pbeg = zz * chunk, pend = min(P, pbeg + chunk);
  const int kq = t % T::KC, rb = t / T::KC;
  const float* zp = g_zero_page;
  const __bf16* zpb = reinterpret_cast<const __bf16*>(g_zero_page);
  const int Hp = H + 2 * pad, Wp = W + 2 * pad;
  // A rows (rows past Mw read row Mw-1: never stored)
  const float* xrow[A_LD];
#pragma unroll
  for (int j = 0; j < A_LD; ++j) {
    const int m = m0 + rb + RPP * j;
    const int mm = m < Mw ? m : Mw - 1;
    const int tap = mm / Cx, ci = mm - tap * Cx;
    const int r = tap / S, s_ = tap - r * S;
    xrow[j] = xt + (long)ci * ldx + r * Wp + (st == 1 ? s_ : (s_ & 1) * (Wp >> 1) + (s_ >> 1));
  }
  // B rows (channels past Cyp read row Cyp-1: never stored)
  const __bf16* drow[B_LD];
#pragma unroll
  for (int j = 0; j < B_LD; ++j) {
    const int n = n0 + rb + RPP * j;
    drow[j] = dyp + (long)(n < Cyp ? n : Cyp - 1) * ldy;
  }
  // this thread's 8-pixel chunk: output pixel kp = (pn, pho, pwo) and its padded-image offset
  int kp = pbeg + 8 * kq, pho, pwo;
  long poff;
  {
    const int hw = Ho * Wo;
    const int pn = kp / hw;
    const int rem = kp - pn * hw;
    pho = rem / Wo;
    pwo = rem - pho * Wo;
    poff = ((long)pn * Hp + st * pho) * Wp + pwo;
  }
  float4 ra[2][A_LD][2];
  u32x4_t rbv[2][B_LD][NP];
  auto load_all = [&](int set) __attribute__((always_inline)) {
    const bool live = kp < pend;  // 8-pixel chunks never straddle pend (chunk, P multiples of 8)
#pragma unroll
    for (int j = 0; j < A_LD; ++j) {
      const float* p = live ? xrow[j] + poff : zp;
      const f4u u0 = *reinterpret_cast<const f4u*>(p);
      const f4u u1 = *reinterpret_cast<const f4u*>(p + 4);
      ra[set][j][0] = make_float4(u0.x, u0.y, u0.z, u0.w);
      ra[set][j][1] = make_float4(u1.x, u1.y, u1.z, u1.w);
    }
#pragma unroll
    for (int j = 0; j < B_LD; ++j) {
      const __bf16* q = live ? drow[j] + kp : zpb;
      const long ps = live ? dps : 0;
#pragma unroll
      for (int p = 0; p < NP; ++p) rbv[set][j][p] = *reinterpret_cast<const u32x4_t*>(q + p * ps);
    }
  };
  const long row_step = (long)st * Wp - Wo, img_step = (long)(Hp - st * Ho) * Wp;
  auto adv = [&](bool go) __attribute__((always_inline)) {
    if (W1 && VST_WG_SELECT) {
      const int pw1 = pwo + T::BK;
      const bool e1 = pw1 >= Wo;
      const int ph1 = pho + (e1 ? 1 : 0);
      const bool e2 = ph1 == Ho;
      const long po1 = poff + T::BK + (e1 ? row_step : 0) + (e2 ? img_step : 0);
      kp = go ? kp + T::BK : kp;
      pwo = go ? (e1 ? pw1 - Wo : pw1) : pwo;
      pho = go ? (e2 ? 0 : ph1) : pho;
      poff = go ? po1 : poff;
      return;
    }
    if (!go) return;
    kp += T::BK;
    pwo += T::BK;
    poff += T::BK;
    while (pwo >= Wo) {
      pwo -= Wo;
      poff += st * Wp - Wo;
      if (++pho == Ho) { pho = 0; poff += (long)(Hp - st * Ho) * Wp; }
    }
  };
  const int nk = pend > pbeg ? (pend - pbeg + T::BK - 1) / T::BK : 0;
  const int wm0 = (wave / T::WAVES_N) * T::WM, wn0 = (wave % T::WAVES_N) * T::WN;
  float* sl = slab + (long)zz * Mw * Cyp;
  if constexpr (T::M16) {
    f32x4v acc[T::MI16][T::NI16];
    zero_acc4(acc);
    main_loop16<T>(smem, nk, acc, ra, rbv, rb, kq, load_all, adv, [](int) {}, NoDma{});
#pragma unroll
    for (int i = 0; i < T::MI16; ++i)
#pragma unroll
      for (int j = 0; j < T::NI16; ++j) {
        const int n = n0 + wn0 + 16 * j + (lane & 15);
        if (n >= Cyp) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int mm = m0 + wm0 + 16 * i + 4 * (lane >> 4) + r;
          if (mm < Mw) sl[(long)mm * Cyp + n] = acc[i][j][r];
        }
      }
    return;
  }
  f32x16 acc[T::MI][T::NI];
  zero_acc(acc);
  main_loop<T>(smem, nk, acc, ra, rbv, rb, kq, load_all, adv, [](int) {});

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

// ---- The weight gradient over NHWC operands (round 6).  conv_wgrad_bf_k reads x as a padded channel-major fp32
// image and dy as channel-major bf16 planes — layouts with the pixel (the GEMM's K) contiguous, made for it by the
// producing IN passes in addition to the NHWC tensors the convs read.  This kernel reads the NHWC tensors
// themselves: x fp32 NHWC (the activation the forward conv read; reflect / zero padding applied per gathered
// pixel) and dy as its NHWC bf16 planes [3][P][Cyp] (the data gradient's pre-split A operand), both with the
// channels (the GEMM's M / N) contiguous.  The stage image is therefore k-major — per plane, [32 k rows] x
// [128 columns] sub-images — and the MFMA operands are read with ds_read_b64_tr_b16 (cdna_hip_programming.md T10:
// per 16-lane group a 4-row x 16-column block delivered column-major; two reads give a lane its 8 k values).  The
// rows are KM_PITCH = 272 B apart (256 B of data + 16): a 32-lane half of a transposed read touches rows 8g + q and
// 8g + 8 + q (q < 4), whose 32-B pieces then sit 4 banks apart (at most 2-way, as the channel-major kernel's
// 16x16x32 row reads) and, unlike a chunk XOR, a fragment's address differs from the next fragment's by an
// immediate, so the operand reads need one address register per stage.  The K split, the per-stage MFMA sequence
// and the lanes' k assignment are conv_wgrad_bf_k's, so the slabs are bit-identical to it.
constexpr int KM_PITCH = 272, KM_GROUP = 32 * KM_PITCH;
__device__ __forceinline__ int km_off(int grp, int row, int col) { return grp * KM_GROUP + KM_PITCH * row + 2 * col; }
template <class T>
struct KmGeom {
  static constexpr int A_PLANE = (T::BM / 128) * KM_GROUP, B_PLANE = (T::BN / 128) * KM_GROUP;
  static constexpr int A_BYTES = T::NP * A_PLANE, STAGE = T::NP * (A_PLANE + B_PLANE);
  static_assert(2 * STAGE <= 160 * 1024, "LDS");
};

// A chunks (8 consecutive M columns of one k row, fp32 -> split here), B chunks (8 columns of one k row per plane,
// pre-split): thread t's chunk j is c = t + NT j, row c / (cols / 8), chunk c % (cols / 8)
template <class T>
__device__ __forceinline__ void store_stage_km(char* st, const float4 (&ra)[T::A_LD][2],
                                               const u32x4_t (&rbv)[T::B_LD][T::NP], int t) {
  using G = KmGeom<T>;
  char* Bs = st + G::A_BYTES;
  constexpr int AC = T::BM / 8, BC = T::BN / 8;
#pragma unroll
  for (int j = 0; j < T::A_LD; ++j) {
    const int c = t + T::NT * j, k = c / AC, mc = c % AC;
    uint4 sp[T::NP];
    split8<T::NP>(ra[j][0], ra[j][1], sp);
    const int off = km_off(mc >> 4, k, 8 * (mc & 15));
#pragma unroll
    for (int p = 0; p < T::NP; ++p) *reinterpret_cast<uint4*>(st + p * G::A_PLANE + off) = sp[p];
  }
#pragma unroll
  for (int j = 0; j < T::B_LD; ++j) {
    const int c = t + T::NT * j, k = c / BC, nc = c % BC;
    const int off = km_off(nc >> 4, k, 8 * (nc & 15));
#pragma unroll
    for (int p = 0; p < T::NP; ++p) *reinterpret_cast<u32x4_t*>(Bs + p * G::B_PLANE + off) = rbv[j][p];
  }
}

// ... B chunks as fp32 (8 columns of one k row, split here like A)
template <class T>
__device__ __forceinline__ void store_stage_km(char* st, const float4 (&ra)[T::A_LD][2],
                                               const float4 (&rbf)[T::B_LD][2], int t) {
  using G = KmGeom<T>;
  char* Bs = st + G::A_BYTES;
  constexpr int AC = T::BM / 8, BC = T::BN / 8;
#pragma unroll
  for (int j = 0; j < T::A_LD; ++j) {
    const int c = t + T::NT * j, k = c / AC, mc = c % AC;
    uint4 sp[T::NP];
    split8<T::NP>(ra[j][0], ra[j][1], sp);
    const int off = km_off(mc >> 4, k, 8 * (mc & 15));
#pragma unroll
    for (int p = 0; p < T::NP; ++p) *reinterpret_cast<uint4*>(st + p * G::A_PLANE + off) = sp[p];
  }
#pragma unroll
  for (int j = 0; j < T::B_LD; ++j) {
    const int c = t + T::NT * j, k = c / BC, nc = c % BC;
    uint4 sp[T::NP];
    split8<T::NP>(rbf[j][0], rbf[j][1], sp);
    const int off = km_off(nc >> 4, k, 8 * (nc & 15));
#pragma unroll
    for (int p = 0; p < T::NP; ++p) *reinterpret_cast<uint4*>(Bs + p * G::B_PLANE + off) = sp[p];
  }
}

typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4_t lds_bf16x4;

// the 16x16x32 operand of columns cb .. cb + 15 (k = 8 g .. 8 g + 7 for lane group g) from a k-major image:
// lane 4q + p of group g supplies row 8g + q (then 8g + 4 + q), columns cb + 4p .. + 3
__device__ __forceinline__ bf16x8_t read_km16(const char* __restrict__ img, int cb, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const char* a0 = img + km_off(cb >> 7, 8 * g + q, (cb & 127) + 4 * pp);
  const char* a1 = a0 + 4 * KM_PITCH;
  bf16x4_t lo = {}, hi = {};
#if defined(__HIP_DEVICE_COMPILE__)
  lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a0));
  hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a1));
#endif
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

template <class T>
__device__ __forceinline__ void read_plane16_km(Plane16<T>& f, const char* __restrict__ st, int p, int wm0, int wn0,
                                                int lane) {
  using G = KmGeom<T>;
  const char* As = st + p * G::A_PLANE;
  const char* Bs = st + G::A_BYTES + p * G::B_PLANE;
#pragma unroll
  for (int i = 0; i < T::MI16; ++i) f.a[i] = read_km16(As, wm0 + 16 * i, lane);
#pragma unroll
  for (int j = 0; j < T::NI16; ++j) f.b[j] = read_km16(Bs, wn0 + 16 * j, lane);
}

// main_loop16 (same stage / group / MFMA order) on k-major stage images
template <class T, class RB, class LoadAll, class Adv>
__device__ __forceinline__ void main_loop16_km(char* smem, int nk, f32x4v (&acc)[T::MI16][T::NI16],
                                               float4 (&ra)[2][T::A_LD][2], RB (&rbv)[2], LoadAll load_all,
                                               Adv adv) {
  constexpr int STAGE = KmGeom<T>::STAGE;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm0 = (wave / T::WAVES_N) * T::WM, wn0 = (wave % T::WAVES_N) * T::WN;
  if (nk <= 0) return;
  load_all(0);
  store_stage_km<T>(smem, ra[0], rbv[0], t);
  adv(nk > 1);
  load_all(1);
  __syncthreads();
  Plane16<T> hi, mid, lo;
  read_plane16_km<T>(mid, smem, 1, wm0, wn0, lane);
  auto step = [&](int kt, auto par) __attribute__((always_inline)) {
    constexpr int P = decltype(par)::value;
    const char* cur = smem + P * STAGE;
    char* nxt = smem + (P ^ 1) * STAGE;
    read_plane16_km<T>(hi, cur, 0, wm0, wn0, lane);
    adv(kt + 2 < nk);
    load_all(P);
    mma16<T>(mid, mid, acc);
    read_plane16_km<T>(lo, cur, 2, wm0, wn0, lane);
    store_stage_km<T>(nxt, ra[P ^ 1], rbv[P ^ 1], t);
    mma16<T>(mid, hi, acc);
    mma16<T>(hi, mid, acc);
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
    read_plane16_km<T>(mid, nxt, 1, wm0, wn0, lane);
    mma16<T>(hi, hi, acc);
    mma16<T>(lo, hi, acc);
    mma16<T>(hi, lo, acc);
  };
  int kt = 0;
  for (; kt + 1 < nk; kt += 2) {
    step(kt, std::integral_constant<int, 0>());
    step(kt + 1, std::integral_constant<int, 1>());
  }
  if (kt < nk) step(kt, std::integral_constant<int, 0>());
}

// dW = x^T dy over split-K pixel chunks, x fp32 NHWC [N][H][W][Cx], dy NHWC bf16 planes dyp [3][P][Cyp] (plane
// stride pps) or, BF32, dy itself fp32 NHWC [P][Cyp] (split in registers like x); M rows (tap, ci), N columns co;
// the same tile grid / XCD order / chunks / slab layout as conv_wgrad_bf_k.  Needs Wo % 32 == 0 (a 32-pixel K
// step inside one output row), Cx % 8 == 0, Cyp % 8 == 0.  dwd != null (one split only): the tile goes straight
// into the weight gradient dwd[co][m] (co < dco; += when dacc) instead of a slab — rows m are then the weight's
// inner index (the im2col form of vst_conv2d_wgrad_nhwc_f32 orders its columns (ci, r, s)).
template <class T, bool BF32>
__global__ __launch_bounds__(T::NT, T::MINB) void conv_wgrad_nhwc_k(
    const float* __restrict__ x, const void* __restrict__ dyv, long pps, float* __restrict__ slab, int H, int W,
    int Cx, int Ho, int Wo, int Cyp, int S, int pad, int st, int reflect, int Mw, int P, int chunk,
    float* __restrict__ dwd, int dco, int dacc) {
  static_assert(T::M16 && T::BK == 32 && T::BM % 128 == 0 && T::BN % 128 == 0, "k-major images of 128 columns");
  static_assert((T::NT % (T::BM / 8)) == 0 && (T::NT % (T::BN / 8)) == 0, "a thread's chunk column is fixed");
  __shared__ __attribute__((aligned(16))) char smem[2 * KmGeom<T>::STAGE];
  constexpr int A_LD = T::A_LD, B_LD = T::B_LD, NP = T::NP, AC = T::BM / 8, BC = T::BN / 8;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int Mt = (Mw + T::BM - 1) / T::BM, Nt = (Cyp + T::BN - 1) / T::BN, Zt = (P + chunk - 1) / chunk;
  int mx, ny, zz;
  {
    const int tt = xcd_tile(blockIdx.x, Mt * Nt * Zt);
    zz = tt / (Mt * Nt);
    const int rem = tt - zz * Mt * Nt;
    ny = rem / Mt;
    mx = rem - ny * Mt;
  }
  const int m0 = mx * T::BM, n0 = ny * T::BN;
  const int pbeg = zz * chunk, pend = min(P, pbeg + chunk);
  // Both operands through buffer descriptors: a gathered pixel outside the frame (zero padding) or a stage past the
  // split's end gets an offset past the descriptor's range and reads zeros — the loads stay unconditional and
  // their 32-bit offsets cheap (the host keeps both tensors under 2 GiB), so the two-stage loop body stays one
  // basic block (a select between two pointers compiled to branches around 64-bit address arithmetic).
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(x), 0, (int)((long)P / (Ho * Wo) * H * W * Cx * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t drs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(dyv), 0, (int)(BF32 ? (long)P * Cyp * 4 : NP * pps * 2), 0x00020000);
  constexpr int OOB = 0x7ffffff0;
  // this thread's A column chunk (tap, ci .. ci + 7) (columns past Mw read column chunk Mw - 8: never stored)
  int r_, s_, ci;
  {
    const int m = min(m0 + 8 * (t % AC), Mw - 8);
    const int tap = m / Cx;
    ci = m - tap * Cx;
    r_ = tap / S;
    s_ = tap - r_ * S;
  }
  const int ka = t / AC;  // + (NT / AC) j: its pixel rows
  // its B column chunk (channels past Cyp read the last chunk: never stored)
  const int co = min(n0 + 8 * (t % BC), Cyp - 8), kb = t / BC;
  // the stage's first output pixel: (n, ho, wo0), flattened pb
  int pb = pbeg, n, ho, wo0;
  {
    const int hw = Ho * Wo;
    n = pb / hw;
    const int rem = pb - n * hw;
    ho = rem / Wo;
    wo0 = rem - ho * Wo;
  }
  typedef typename std::conditional<BF32, float4[B_LD][2], u32x4_t[B_LD][NP]>::type RBset;
  float4 ra[2][A_LD][2];
  RBset rbv[2];
  auto load_all = [&](int set) __attribute__((always_inline)) {
    const bool live = pb < pend;
    const int hi = ho * st + r_ - pad;
    const int hr = reflect ? reflect_idx(hi, H) : hi;
    const bool hok = live && (unsigned)hr < (unsigned)H;
    const int rowb = (n * H + hr) * W;  // pixel index of (n, hr, 0)
#pragma unroll
    for (int j = 0; j < A_LD; ++j) {
      const int wi = (wo0 + ka + (T::NT / AC) * j) * st + s_ - pad;
      const int wr = reflect ? reflect_idx(wi, W) : wi;
      // (bitwise forms: a short-circuit / select form compiled to a branch around the offset arithmetic)
      const int ok = (int)hok & (int)((unsigned)wr < (unsigned)W), msk = -ok;
      const int off = ((((rowb + wr) * Cx + ci) * 4) & msk) | (OOB & ~msk);
      ra[set][j][0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0));
      ra[set][j][1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xrs, off + 16, 0, 0));
    }
#pragma unroll
    for (int j = 0; j < B_LD; ++j) {
      const int e = (pb + kb + (T::NT / BC) * j) * Cyp + co;
      if constexpr (BF32) {
        const int off = live ? e * 4 : OOB;
        rbv[set][j][0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(drs, off, 0, 0));
        rbv[set][j][1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(drs, off + 16, 0, 0));
      } else {
#pragma unroll
        for (int p = 0; p < NP; ++p)
          rbv[set][j][p] = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(
                                                           drs, live ? (e + p * (int)pps) * 2 : OOB, 0, 0));
      }
    }
  };
  auto adv = [&](bool go) __attribute__((always_inline)) {
    const int w1 = wo0 + T::BK;
    const bool e1 = w1 == Wo;
    const int h1 = ho + (e1 ? 1 : 0);
    const bool e2 = h1 == Ho;
    pb = go ? pb + T::BK : pb;
    wo0 = go ? (e1 ? 0 : w1) : wo0;
    ho = go ? (e2 ? 0 : h1) : ho;
    n = go ? (e2 ? n + 1 : n) : n;
  };
  const int nk = pend > pbeg ? (pend - pbeg + T::BK - 1) / T::BK : 0;
  const int wm0 = (wave / T::WAVES_N) * T::WM, wn0 = (wave % T::WAVES_N) * T::WN;
  float* sl = slab + (long)zz * Mw * Cyp;
  f32x4v acc[T::MI16][T::NI16];
  zero_acc4(acc);
  main_loop16_km<T>(smem, nk, acc, ra, rbv, load_all, adv);
  if (dwd) {  // one split: the transposed tile into the weight gradient itself (4 consecutive m per lane: one float4)
#pragma unroll
    for (int i = 0; i < T::MI16; ++i)
#pragma unroll
      for (int j = 0; j < T::NI16; ++j) {
        const int nn = n0 + wn0 + 16 * j + (lane & 15), mm = m0 + wm0 + 16 * i + 4 * (lane >> 4);
        if (nn >= dco || mm >= Mw) continue;
        float4* d = reinterpret_cast<float4*>(dwd + (long)nn * Mw + mm);
        float4 v = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
        if (dacc) {
          const float4 o = *d;
          v = make_float4(o.x + v.x, o.y + v.y, o.z + v.z, o.w + v.w);
        }
        *d = v;
      }
    return;
  }
#pragma unroll
  for (int i = 0; i < T::MI16; ++i)
#pragma unroll
    for (int j = 0; j < T::NI16; ++j) {
      const int nn = n0 + wn0 + 16 * j + (lane & 15);
      if (nn >= Cyp) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int mm = m0 + wm0 + 16 * i + 4 * (lane >> 4) + r;
        if (mm < Mw) sl[(long)mm * Cyp + nn] = acc[i][j][r];
      }
    }
}

// fprop_splitk_reduce_k of a data gradient's split-K tail (no bias / act) with the IN-backward partials
// of the layer below (InbArgs, one 32-row group per block: slice (m - image start) / 32); same block
// geometry, the 16 row-threads' fp64 sums folded through LDS in a fixed order.
__global__ __launch_bounds__(256) void fprop_splitk_reduce_inb_k(const float* __restrict__ slab, int ks, int m_base,
                                                                 int M, int Cop, float* __restrict__ y, int hw,
                                                                 const float* __restrict__ addend, InbArgs inb) {
  __shared__ double red[3][16][65];
  const int t = threadIdx.x, c4 = (t & 15) * 4, sub = t >> 4;
  const int n = blockIdx.y * 64 + c4;
  const long rows = M - m_base, zst = rows * Cop;
  const int r0 = blockIdx.x * 32;
  const int g0 = m_base + r0, img = g0 / hw;
  double a0[4] = {0, 0, 0, 0}, a1[4] = {0, 0, 0, 0}, a2[4] = {0, 0, 0, 0};
  if (n < Cop) {
    const float4 s0 = reinterpret_cast<const float4*>(inb.st)[((long)img * Cop + n) / 2];
    const float4 s1 = reinterpret_cast<const float4*>(inb.st)[((long)img * Cop + n) / 2 + 1];
    const float mu[4] = {s0.x, s0.z, s1.x, s1.z}, rs[4] = {s0.y, s0.w, s1.y, s1.w};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const long r = r0 + sub + 16 * h;
      if (r >= rows) break;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int z0 = 0; z0 < ks; z0 += 8) {  // batches of 8 loads in flight, summed in slab order
        float4 q[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          q[u] = z0 + u < ks ? *reinterpret_cast<const float4*>(slab + (z0 + u) * zst + r * Cop + n)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (z0 + u >= ks) break;
          add_f4(v, q[u]);
        }
      }
      if (addend) add_f4(v, *reinterpret_cast<const float4*>(addend + (m_base + r) * Cop + n));
      *reinterpret_cast<float4*>(y + (m_base + r) * Cop + n) = v;
      const float4 zz = *reinterpret_cast<const float4*>(inb.z + (m_base + r) * Cop + n);
      const float gv[4] = {v.x, v.y, v.z, v.w}, zv[4] = {zz.x, zz.y, zz.z, zz.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float gd, xh;
        inb_term(gv[e], zv[e], mu[e], rs[e], inb.act, inb.slope, gd, xh);
        a0[e] += gd;
        a1[e] += (double)gd * xh;
        a2[e] += xh;
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    red[0][sub][c4 + e] = a0[e];
    red[1][sub][c4 + e] = a1[e];
    red[2][sub][c4 + e] = a2[e];
  }
  __syncthreads();
  if (t < 192) {
    const int v = t >> 6, c = t & 63, nn = blockIdx.y * 64 + c;
    if (nn >= Cop) return;
    double acc = 0.0;
    for (int q = 0; q < 16; ++q) acc += red[v][q][c];
    inb.part[(((long)img * inb.ns + ((g0 - img * hw) >> 5)) * Cop + nn) * 3 + v] = acc;
  }
}

// Split-K tail: y[m][n] = act(sum_z slab[z][m - m_base][n] + bias[n]) (splits summed in order) and,
// with part, the InstanceNorm partials {sum y, sum y^2} of each 32-row group in the layout of the
// GEMM epilogue's.  A block owns one 32-row group x 64 channels: thread (row pair r, r + 16; 4
// channels) issues all its 2 x ks float4 slab loads together, then the 16 row-threads' fp64 sums
// fold through LDS in a fixed order.  grid (ceil((M - m_base) / 32), ceil(Cop / 64)), 256 threads;
// Cop % 4 == 0.
__global__ __launch_bounds__(256) void fprop_splitk_reduce_k(const float* __restrict__ slab, int ks, int m_base, int M,
                                                             int Cop, const float* __restrict__ bias, int act,
                                                             float slope, float* __restrict__ y,
                                                             double* __restrict__ part, int hw,
                                                             const float* __restrict__ addend = nullptr) {
  __shared__ double red[2][16][65];
  const int t = threadIdx.x, c4 = (t & 15) * 4, sub = t >> 4;
  const int n = blockIdx.y * 64 + c4;
  const long rows = M - m_base, zst = rows * Cop;
  const int r0 = blockIdx.x * 32;
  double s1[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
  if (n < Cop) {
    // scalar loads: a bias may be a view at any 4-byte offset of a network's flat parameter buffer
    const float4 bv = bias ? make_float4(bias[n], bias[n + 1], bias[n + 2], bias[n + 3]) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const long r = r0 + sub + 16 * h;
      if (r >= rows) break;
      float4 v = bv;
      // the slabs in batches of 8 loads in flight, summed in slab order (a load-add chain is a round trip per slab)
      for (int z0 = 0; z0 < ks; z0 += 8) {
        float4 q[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          q[u] = z0 + u < ks ? *reinterpret_cast<const float4*>(slab + (z0 + u) * zst + r * Cop + n)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (z0 + u >= ks) break;
          add_f4(v, q[u]);
        }
      }
      float o[4] = {apply_act(v.x, act, slope), apply_act(v.y, act, slope), apply_act(v.z, act, slope),
                    apply_act(v.w, act, slope)};
      if (addend) {  // added after the activation (the addend of a data gradient: the residual gradient)
        const float4 a = *reinterpret_cast<const float4*>(addend + (m_base + r) * Cop + n);
        o[0] += a.x;
        o[1] += a.y;
        o[2] += a.z;
        o[3] += a.w;
      }
      *reinterpret_cast<float4*>(y + (m_base + r) * Cop + n) = make_float4(o[0], o[1], o[2], o[3]);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        s1[e] += o[e];
        s2[e] += (double)o[e] * o[e];
      }
    }
  }
  if (!part) return;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    red[0][sub][c4 + e] = s1[e];
    red[1][sub][c4 + e] = s2[e];
  }
  __syncthreads();
  if (t < 128) {
    const int v = t >> 6, c = t & 63, nn = blockIdx.y * 64 + c;
    if (nn >= Cop) return;
    double acc = 0.0;
    for (int q = 0; q < 16; ++q) acc += red[v][q][c];
    const int g0 = m_base + r0, img = g0 / hw, zg = (g0 - img * hw) >> 5;
    part[(((long)img * (hw >> 5) + zg) * Cop + nn) * 2 + v] = acc;
  }
}

// NHWC [P][Cs] fp32 -> NP bf16 planes [NP][Cs][ld] (hi, (mid,) lo of each value, the same RNE
// conversions as split8 / split3_k) through a 64x64 LDS transpose tile: the weight gradient's
// pre-split B operand.
// rin / rout (> 0): the plane pixels are rows of rout words holding rin source pixels each, then
// zeros (the Wo-padded weight gradient); P counts plane pixels.
template <int NP>
__global__ __launch_bounds__(256) void nhwc_to_cp_planes_k(const float* __restrict__ x, __bf16* __restrict__ y,
                                                           long P, int Cs, long ld, int rin, int rout) {
  __shared__ float tile[64][65];
  const long p0 = (long)blockIdx.x * 64;
  const int c0 = blockIdx.y * 64;
  const int t = threadIdx.x;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int idx = t + 256 * it, pr = idx >> 4, c4 = (idx & 15) * 4;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    long q = p0 + pr;
    bool ok = q < P && c0 + c4 < Cs;
    if (rout > 0) {
      const long row = q / rout;
      const int col = (int)(q - row * rout);
      ok = ok && col < rin;
      q = row * rin + col;
    }
    if (ok) v = *reinterpret_cast<const float4*>(x + q * Cs + c0 + c4);
    tile[pr][c4] = v.x;
    tile[pr][c4 + 1] = v.y;
    tile[pr][c4 + 2] = v.z;
    tile[pr][c4 + 3] = v.w;
  }
  __syncthreads();
  const long plane = (long)Cs * ld;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int idx = t + 256 * it, cr = idx >> 4, p4 = (idx & 15) * 4;
    if (c0 + cr >= Cs || p0 + p4 >= P) continue;
    float r[4] = {tile[p4][cr], tile[p4 + 1][cr], tile[p4 + 2][cr], tile[p4 + 3][cr]};
    __bf16* dst = y + (long)(c0 + cr) * ld + p0 + p4;
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const uint32_t q0 = pack2(r[0], r[1]), q1 = pack2(r[2], r[3]);
      if (p0 + p4 + 3 < P) {
        *reinterpret_cast<uint2*>(dst + p * plane) = make_uint2(q0, q1);
      } else {  // ragged plane length: element stores, never past P
        const uint16_t h[4] = {(uint16_t)q0, (uint16_t)(q0 >> 16), (uint16_t)q1, (uint16_t)(q1 >> 16)};
        for (int e = 0; e < 4 && p0 + p4 + e < P; ++e)
          reinterpret_cast<uint16_t*>(dst + p * plane)[e] = h[e];
      }
      if (p + 1 < NP) {
        r[0] -= __uint_as_float(q0 << 16);
        r[1] -= __uint_as_float(q0 & 0xffff0000u);
        r[2] -= __uint_as_float(q1 << 16);
        r[3] -= __uint_as_float(q1 & 0xffff0000u);
      }
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
//   6: 64x64, 4 waves of 32x32, BK 32      7: 256x128, 8 waves of 64x64, BK 32
//   8: 64x64, 4 waves of 32x32, BK 32 (x6) / 64 (x3)
//   9: 128x128, 4 waves of 64x64, BK 16 (x6: two blocks / CU)
//  10: 256x64, 4 waves of 64x64, BK 32 (x6: the image-layer weight gradients, M = 147 rows in one tile)
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
    case 9: L(128, 128, 64, 64, 16, np) break;                         \
    case 10: L(256, 64, 64, 64, 32, np) break;                         \
    default: L(128, 128, 64, 32, 32, np) break;                        \
  }

int bf_pick(long M, int Nc, int override_kind) {
  if (override_kind >= 0 && override_kind <= 9) return override_kind;
  if (Nc <= 64) return M / 128 >= 256 ? 1 : 6;
  const long n128 = (Nc + 127) / 128;
  if ((M / 128) * n128 >= 200) return 0;
  if ((M / 64) * n128 >= 200) return 3;
  return 6;
}

// Tile geometry of a kind for NP planes: rows, cols, co-resident blocks per CU (LDS-limited).
static void bf_geom(int kind, int np, int* bm, int* bn, int* slots) {
  int BM = 128, BN = 128, BK = 32;
  switch (kind) {
    case 1: BN = 64; break;
    case 2: break;
    case 3: BM = 64; break;
    case 4: BK = np == 3 ? 32 : 64; break;
    case 5: BN = 64; BK = 64; break;
    case 6: BM = 64; BN = 64; break;
    case 7: BM = 256; break;
    case 8: BM = 64; BN = 64; BK = np == 3 ? 32 : 64; break;
    case 9: BK = 16; break;
    case 10: BM = 256; BN = 64; break;
    default: break;
  }
  const int stage = np * (BM + BN) * BK * 2;
  int sl = (160 * 1024) / (2 * stage);
  const int waves = (kind == 0 || kind == 4 || kind == 7) ? 8 : 4;
  if (sl * waves > 32) sl = 32 / waves;
  *bm = BM;
  *bn = BN;
  *slots = sl < 1 ? 1 : sl;
}

// Launch plan of the split-arithmetic forward for an M x Cop output: the tile kind of the main
// launch and, when the grid is split for wave quantisation, the first pixel row of the tail launch
// (0 = one launch) and the tail's tile kind.  Host-only; exported through vst_conv_plan_fwd.
void bf_plan(long M, int Cop, int math, int kind, int* kind_out, int* m_split_out, int* tail_out) {
  int kd = bf_pick(M, Cop, kind);
  int m_split = 0, tail_kind = VST_BF_TAIL_KIND;
#if VST_BF_X6_256
  // x6 runs one 128x128 or 256x128 block per CU either way (the three-plane stage pairs are 96 /
  // 144 KB): 256x128 tiles of 8 waves x (64x64) halve the LDS fragment reads per MFMA and the
  // barriers per FLOP.  Whole rounds of 256 blocks run as one launch; otherwise the whole rounds
  // of 256x128 tiles run first and the remaining pixel rows (a partial round) as a second launch
  // of smaller tiles chosen to fill the CUs (cost = rounds x tile area / tile efficiency):
  //   N=8 padded-frame dgrad (M = 34848): 256 x 256x128 + 132 x 64x64 blocks (was 546 x 128x128
  //   at one per CU = 3 rounds); N=12 forward (M = 49152): 256 x 256x128 + 512 x 64x128.
  if (kind < 0 && kd == 0 && math == VST_MATH_BF16X6) {
    const long nt = (Cop + 127) / 128;
    const long b256 = (long)((M + 255) / 256) * nt;
    if (b256 % VST_NUM_CUS == 0 || b256 >= 4 * VST_NUM_CUS) {
      kd = 7;
    } else if (b256 > VST_NUM_CUS && (VST_NUM_CUS % nt) == 0) {
      const long ms = (long)(b256 / VST_NUM_CUS) * (VST_NUM_CUS / nt) * 256;  // whole rounds of rows
      const long rest = M - ms;
      static const int cand[4] = {8, 3, 1, 0};
      static const double eff[4] = {0.6, 0.75, 0.75, 0.85};  // relative to the 256x128 tile
      double best = (double)((b256 + VST_NUM_CUS - 1) / VST_NUM_CUS);  // no split: whole 256x128 grid
      int bk = -1;
      for (int c = 0; c < 4; ++c) {
        int bm, bn, sl;
        bf_geom(cand[c], 3, &bm, &bn, &sl);
        const long blocks = ((rest + bm - 1) / bm) * ((Cop + bn - 1) / bn);
        const long rounds = (blocks + (long)sl * VST_NUM_CUS - 1) / ((long)sl * VST_NUM_CUS);
        const double cost = (double)(ms / 256 * nt) / VST_NUM_CUS + rounds * (bm * bn) / (256.0 * 128.0) / eff[c];
        if (cost < best - 1e-9) { best = cost; bk = cand[c]; }
      }
      if (VST_BF_TAIL_FORCE >= 0) bk = VST_BF_TAIL_FORCE;  // developer A/B of the tail tile
      kd = 7;
      if (bk >= 0) {
        m_split = (int)ms;
        tail_kind = bk;
      }
    } else if (b256 < VST_NUM_CUS && b256 > VST_BF_FULLSPLIT_MAX) {
      // one partial round of 256x128 tiles (more than the all-split form takes) against the 128x128 grid's
      // rounds at the same one block per CU (a 32-deep K step ~2.25 vs ~1.5 us): the 436x1024 ResnetBlocks
      // (M = 27904, 218 tiles) ran 436 128x128 blocks = 2 rounds
      const long r128 = ((M + 127) / 128 * nt + VST_NUM_CUS - 1) / VST_NUM_CUS;
      if (2.25 < 1.5 * r128) kd = 7;
    }
  }
#endif
#if VST_BF_TAIL
  // Wave quantisation: 128x128 x3 blocks run two per CU, so a grid a few tiles past a whole
  // number of blocks per CU (the padded-frame dgrad: 546 = 2 x 256 + 34 blocks at N = 8) keeps
  // most CUs idle for one extra block time.  Such a tail (<= 1/4 of the CUs) runs as a second
  // launch of 64x64 tiles over the remaining pixel rows (4x as many, 4x smaller blocks).
  if (kind < 0 && kd == 0 && math != VST_MATH_BF16X6) {
    const long nt = (Cop + 127) / 128, blocks = (long)((M + 127) / 128) * nt;
    const long per = blocks / VST_NUM_CUS, tail = blocks - per * VST_NUM_CUS;
    if (per >= 1 && tail > 0 && 4 * tail <= VST_NUM_CUS && (per * VST_NUM_CUS) % nt == 0) {
      m_split = (int)(per * VST_NUM_CUS / nt) * 128;
      tail_kind = VST_BF_TAIL_KIND;
    }
  }
#endif
  *kind_out = kd;
  *m_split_out = m_split;
  *tail_out = m_split ? tail_kind : -1;
}

// Split-K count for the wave-quantisation tail of a whole-round x6 plan (the rows past m_split as
// 256x128 tiles, K split ks ways, + fprop_splitk_reduce_k), 0 = none; cost model in microseconds:
// rounds x (K-steps x 2.25 + 4) for the GEMM (the 256x128 x6 tile runs ~2.25 us per 32-deep K-step
// per round) + the reduction's slab traffic at 4 TB/s + a launch.  N=8 ResnetBlock data gradient
// (2080 tail rows): 14 splits of 6 K-steps; N=12 forward (16384 rows): 2 splits.
int bf_tail_ks(long M, int Cop, int m_split, int nk) {
  const long rest = M - m_split;
  if (m_split <= 0 || rest <= 0) return 0;
  const long Tt = ((rest + 255) / 256) * ((Cop + 127) / 128);
  double best = 1e30;
  int bk = 0;
  for (int ks = 2; ks <= 16; ++ks) {
    const int steps = (nk + ks - 1) / ks;
    if ((long)(ks - 1) * steps >= nk) continue;  // a split would be empty
    const long rounds = (Tt * ks + VST_NUM_CUS - 1) / VST_NUM_CUS;
    const double us = rounds * (steps * 2.25 + 4.0) + (double)(ks + 1) * rest * Cop * 4.0 / 4.0e6 + 3.0;
    if (us < best) {
      best = us;
      bk = ks;
    }
  }
  return bk;
}

// Split-K plan of an x6 forward with a workspace: (first split row, splits), splits = 0 for none.
//   * tail: a whole-round 256x128 plan with a partial last round -> that round as splits (bf_tail_ks);
//   * full: a grid of at most VST_BF_FULLSPLIT_MAX 256x128 tiles (the PatchGAN layers, half-batch
//     passes) -> the whole conv as ks K-range splits of 256x128 tiles filling the CUs, instead of
//     small tiles that cannot fill them either; same cost model.
void bf_split_plan(long M, int Cop, int C, int R, int S, int math, int kind, int* m_first, int* ks_out) {
  *m_first = 0;
  *ks_out = 0;
  if (math != VST_MATH_BF16X6 || !VST_BF_KSLICE || C % 32 || !VST_BF_SPLITK || kind >= 0) return;
  const int nk = (R * S * C + 31) / 32;
  int kd, m_split, tail_kind;
  bf_plan(M, Cop, math, -1, &kd, &m_split, &tail_kind);
  if (kd == 7 && m_split) {
    *m_first = m_split;
    *ks_out = bf_tail_ks(M, Cop, m_split, nk);
    return;
  }
  const long b256 = ((M + 255) / 256) * ((Cop + 127) / 128);
  if (kd == 7 || b256 > VST_BF_FULLSPLIT_MAX) return;
  // the small-tile plan it would replace: rounds x K-steps x the tile's per-round K-step time (x6,
  // 16x16x32; measured on the ResnetBlock / PatchGAN shapes: 256x128 2.25 us, 128x128 1.5 us,
  // 64x128 at two per CU 1.8 us; the 64-wide tiles assumed 1.2 us)
  int bm, bn, sl;
  bf_geom(kd, 3, &bm, &bn, &sl);
  const long blocks = ((M + bm - 1) / bm) * ((Cop + bn - 1) / bn);
  const long rounds_small = (blocks + (long)sl * VST_NUM_CUS - 1) / ((long)sl * VST_NUM_CUS);
  const double t_small = (kd == 0 || kd == 2 || kd == 4 || kd == 9) ? 1.5 : (kd == 3 ? 1.8 : 1.2);
  const double small_us = rounds_small * nk * t_small + 3.0;
  double best = 0.85 * small_us;
  int bk = 0;
  for (int ks = 2; ks <= 32; ++ks) {
    const int steps = (nk + ks - 1) / ks;
    if (steps < 4 || (long)(ks - 1) * steps >= nk) continue;
    const long rounds = (b256 * ks + VST_NUM_CUS - 1) / VST_NUM_CUS;
    const double us = rounds * (steps * 2.25 + 4.0) + (double)(ks + 1) * M * Cop * 4.0 / 4.0e6 + 3.0;
    if (us < best) {
      best = us;
      bk = ks;
    }
  }
  *ks_out = bk;
}

size_t bf_fprop_ws_floats(long M, int Cop, int C, int R, int S, int math) {
  int mf, ks;
  bf_split_plan(M, Cop, C, R, S, math, -1, &mf, &ks);
  return ks ? (size_t)ks * (M - mf) * Cop : 0;
}

int bf_fprop_launch(const float* x, const void* wsplit, long wps, const float* bias, float* y, int N,
                    int H, int W, int C, int Ho, int Wo, int Cop, int R, int S, int st, int padh, int padw,
                    int reflect, int act, float slope, int math, int kind, hipStream_t s, double* part,
                    float* tws, size_t tws_floats, const float* addend, int oph) {
  if (oph) tws = nullptr;  // phase stores: no split-K slabs (their reduce stores unmapped)
  // the epilogue routes differ on whether an addend enters the IN partials (the per-element store
  // counts it, the LDS-staged one adds it at the row store): no caller needs both, so refuse it
  VST_REQUIRE(!(part && addend), "conv fprop: IN partials together with an addend are not supported");
  const int M = N * Ho * Wo, K = R * S * C;
  // 4-channel inputs with 64 outputs (the generator's 7x7 image convs): the direct patch-staged kernel
  if (kind < 0 && padh == padw && !addend && !oph && c4_direct_ok(C, Cop, R, S, st, Ho, Wo, math))
    return c4_direct_launch(x, wsplit, wps, bias, y, N, H, W, Ho, Wo, R, S, padh, reflect, act, slope, math, part, s);
  const __bf16* ws = reinterpret_cast<const __bf16*>(wsplit);
  int kd, m_split, tail_kind;
  bf_plan(M, Cop, math, kind, &kd, &m_split, &tail_kind);
  int ks = 0, m_first = 0;
  if (tws) {
    bf_split_plan(M, Cop, C, R, S, math, kind, &m_first, &ks);
    if ((size_t)ks * (M - m_first) * Cop > tws_floats) ks = 0;
    if (ks && !m_first) {  // the whole conv as split-K 256x128 tiles: the split launch alone
      m_split = 0;
      kd = -1;
    }
  }
#define VST_BF(BM_, BN_, WM_, WN_, BK_, NP_)                                                       \
  {                                                                                                 \
    using T = bf::Tile<BM_, BN_, WM_, WN_, BK_, NP_>;                                              \
    const dim3 grid(ceil_div(Mend - mb, BM_) * ceil_div(Cop, BN_));                                 \
    if (C == 4)                                                                                     \
      hipLaunchKernelGGL((bf::conv_fprop_bf_k<T, false, 3>), grid, dim3(T::NT), 0, s, x, ws, wps, bias, y, \
                         H, W, C, Ho, Wo, Cop, S, st, padh, padw, reflect, act, slope, Mend, K, mb, part, 0,      \
                         nullptr, addend, oph);                                                          \
    else if (VST_BF_KSLICE && C % BK_ == 0 && reflect)                                              \
      hipLaunchKernelGGL((bf::conv_fprop_bf_k<T, true, 1>), grid, dim3(T::NT), 0, s, x, ws, wps, bias, y, \
                         H, W, C, Ho, Wo, Cop, S, st, padh, padw, reflect, act, slope, Mend, K, mb, part, 0,      \
                         nullptr, addend, oph);                                                          \
    else if (VST_BF_KSLICE && C % BK_ == 0)                                                         \
      hipLaunchKernelGGL((bf::conv_fprop_bf_k<T, true, 0>), grid, dim3(T::NT), 0, s, x, ws, wps, bias, y, \
                         H, W, C, Ho, Wo, Cop, S, st, padh, padw, reflect, act, slope, Mend, K, mb, part, 0,      \
                         nullptr, addend, oph);                                                          \
    else                                                                                            \
      hipLaunchKernelGGL((bf::conv_fprop_bf_k<T, false, 2>), grid, dim3(T::NT), 0, s, x, ws, wps, bias, y, \
                         H, W, C, Ho, Wo, Cop, S, st, padh, padw, reflect, act, slope, Mend, K, mb, part, 0,      \
                         nullptr, addend, oph);                                                          \
  }
  for (int ph = (ks && !m_first) ? 1 : 0; ph < ((m_split || (ks && !m_first)) ? 2 : 1); ++ph) {
    const int mb = ph ? m_split : 0, Mend = (m_split && !ph) ? m_split : M;
    const int kp = ph ? tail_kind : kd;
    if (ph == 1 && ks) {
      using T = bf::Tile<256, 128, 64, 64, 32, 3>;
      const int nk = (K + T::BK - 1) / T::BK, spk = (nk + ks - 1) / ks;
      const dim3 grid(ceil_div(M - mb, 256) * ceil_div(Cop, 128) * ks);
      if (reflect)
        hipLaunchKernelGGL((bf::conv_fprop_bf_k<T, true, 1, true>), grid, dim3(T::NT), 0, s, x, ws, wps, bias, y, H,
                           W, C, Ho, Wo, Cop, S, st, padh, padw, reflect, act, slope, M, K, mb, part, spk, tws,
                           nullptr);
      else
        hipLaunchKernelGGL((bf::conv_fprop_bf_k<T, true, 0, true>), grid, dim3(T::NT), 0, s, x, ws, wps, bias, y, H,
                           W, C, Ho, Wo, Cop, S, st, padh, padw, reflect, act, slope, M, K, mb, part, spk, tws,
                           nullptr);
      hipLaunchKernelGGL(bf::fprop_splitk_reduce_k, dim3(ceil_div(M - mb, 32), ceil_div(Cop, 64)), dim3(256), 0, s,
                         tws, ks, mb, M, Cop, bias, act, slope, y, part, Ho * Wo, addend);
      continue;
    }
    if (math == VST_MATH_BF16X6) {
      VST_BF_DISPATCH(kp, 3, VST_BF)
    } else {
      VST_BF_DISPATCH(kp, 2, VST_BF)
    }
  }
#undef VST_BF
  return check_launch("conv2d_fwd(bf16 split)");
}


// Border GEMM of the reflect-pad-1 data gradient (dgrad_border_pos rows): K-split count and slab
// floats.  The rows (2(H+W)+8..+16 per image) are few, so the 256x128 (x6) / 128x128 (x3) tiles run
// as ks K-range splits filling the CUs; the slabs are summed by dgrad_border_add_k.
static void bf_border_plan(int N, int H, int W, int Cy, int Cx, int math, int* ks_out, long* mb_out) {
  const int NB = bf::dgrad_border_rows(H, W);
  const long Mb = (long)N * NB;
  const int bm = math == VST_MATH_BF16X6 ? 256 : 128;
  const long tiles = ((Mb + bm - 1) / bm) * ((Cx + 127) / 128);
  const int nk = (9 * Cy + 31) / 32;
  int ks = (int)(VST_NUM_CUS / (tiles > 0 ? tiles : 1));
  ks = ks < 1 ? 1 : (ks > 16 ? 16 : ks);
  while (ks > 1 && (ks - 1) * ((nk + ks - 1) / ks) >= nk) --ks;  // no empty split
  *ks_out = ks;
  *mb_out = Mb;
}

// The K-restricted border GEMM (REFL 5, 128x128 tiles): segment lengths and K-split count.  ks: at
// least 4 K-steps per split and at most one CU round (g_border_ks overrides; g_border5 = false keeps the
// full-K border rows of bf_border_plan).
static constexpr bool g_border5 = true;
static constexpr int g_border_ks = 0;
static void bf_border5_plan(int N, int H, int W, int Cy, int Cx, int* ks_out, int* lt, int* ll) {
  *lt = bf::border5_seg_rows(N, W + 2, 128);
  *ll = bf::border5_seg_rows(N, H, 128);
  const long tiles = (long)(2 * *lt + 2 * *ll) / 128 * ((Cx + 127) / 128);
  const int nk = (3 * Cy + 31) / 32;
  int ks = g_border_ks > 0 ? g_border_ks : (int)(VST_NUM_CUS / (tiles > 0 ? tiles : 1));
  if (g_border_ks <= 0 && ks > nk / 4) ks = nk / 4;
  ks = ks < 1 ? 1 : (ks > 16 ? 16 : ks);
  while (ks > 1 && (ks - 1) * ((nk + ks - 1) / ks) >= nk) --ks;  // no empty split
  *ks_out = ks;
}

bool bf_dgrad_refl1_ok(int N, int H, int W, int Cy, int Cx, int math) {
  return math != VST_MATH_F32 && VST_BF_KSLICE && Cy % 32 == 0 && Cx % 4 == 0 && H >= 4 && W >= 4 && N > 0;
}

// where the border GEMM's slabs sit in the dgrad workspace (floats) and their split count / rows per image
size_t bf_dgrad_refl1_slabs(int N, int H, int W, int Cy, int Cx, int math, BorderSlabs* b) {
  if (g_border5) {
    bf_border5_plan(N, H, W, Cy, Cx, &b->ks, &b->Lt, &b->Ll);
    b->Mb = 2 * b->Lt + 2 * b->Ll;
  } else {
    long Mb;
    bf_border_plan(N, H, W, Cy, Cx, math, &b->ks, &Mb);
    b->Mb = (int)Mb;
    b->Lt = bf::dgrad_border_rows(H, W);
    b->Ll = 0;
  }
  return bf_fprop_ws_floats((long)N * H * W, Cx, Cy, 3, 3, math);
}

size_t bf_dgrad_refl1_ws_floats(int N, int H, int W, int Cy, int Cx, int math) {
  int ks, ks5, lt, ll;
  long Mb;
  bf_border_plan(N, H, W, Cy, Cx, math, &ks, &Mb);
  bf_border5_plan(N, H, W, Cy, Cx, &ks5, &lt, &ll);
  const size_t b4 = (size_t)ks * Mb * Cx, b5 = g_border5 ? (size_t)ks5 * (2 * lt + 2 * ll) * Cx : 0;
  return bf_fprop_ws_floats((long)N * H * W, Cx, Cy, 3, 3, math) + (b4 > b5 ? b4 : b5);
}

// dx = data gradient of ReflectionPad2d(1) + 3x3 conv (stride 1) from dy (+ addend), wsplit = the
// VST_PACK_IKF planes of the conv weight: the interior as the zero-pad-1 forward conv (addend in its
// epilogue), then the border GEMM (split-K slabs) and dgrad_border_add_k (add_border with VST_BORDER5
// on: the K-restricted border GEMM and dgrad_border5_add_k).  Replaces the conv over the
// (H+2) x (W+2) zero-padded frame + reflect fold.  add_border = false: the slabs (bf_dgrad_refl1_slabs)
// are left for the caller (vst_conv2d_dgrad_refl_in adds them in its InstanceNorm-backward partial pass).
int bf_dgrad_refl1_launch(const float* dy, const void* wsplit, long wps, const float* addend, float* dx, int N, int H,
                          int W, int Cy, int Cx, int math, hipStream_t s, float* ws, size_t ws_floats, bool add_border) {
  int ks;
  long Mb;
  bf_border_plan(N, H, W, Cy, Cx, math, &ks, &Mb);
  const size_t main_ws = bf_fprop_ws_floats((long)N * H * W, Cx, Cy, 3, 3, math);
  VST_REQUIRE(ws_floats >= main_ws + (size_t)ks * Mb * Cx, "dgrad_refl: workspace too small");
  if (int e = bf_fprop_launch(dy, wsplit, wps, nullptr, dx, N, H, W, Cy, H, W, Cx, 3, 3, 1, 1, 1, 0, VST_ACT_NONE, 0.f,
                              math, -1, s, nullptr, main_ws ? ws : nullptr, main_ws, addend))
    return e;
  float* slab = ws + main_ws;
  const __bf16* wb = reinterpret_cast<const __bf16*>(wsplit);
  if (g_border5) {
    int ks5, lt, ll;
    bf_border5_plan(N, H, W, Cy, Cx, &ks5, &lt, &ll);
    const int Mt = 2 * lt + 2 * ll, K = 3 * Cy;
    VST_REQUIRE(ws_floats >= main_ws + (size_t)ks5 * Mt * Cx, "dgrad_refl: workspace too small");
#define VST_B5(NP_)                                                                                            {                                                                                                             using T = bf::Tile<128, 128, 64, 32, 32, NP_>;                                                              const int nk = (K + T::BK - 1) / T::BK, spk = (nk + ks5 - 1) / ks5;                                         const dim3 grid(Mt / 128 * ceil_div(Cx, 128) * ks5);                                                        hipLaunchKernelGGL((bf::conv_fprop_bf_k<T, true, 5, true>), grid, dim3(T::NT), 0, s, dy, wb, wps, nullptr,                          dx, H, W, Cy, lt, ll, Cx, 3, N, 1, 1, 0, VST_ACT_NONE, 0.f, Mt, K, 0, nullptr, spk,                           slab, nullptr);                                                                        }
    if (math == VST_MATH_BF16X6)
      VST_B5(3)
    else
      VST_B5(2)
#undef VST_B5
    const int T = 2 * W + 2 * H;
    if (add_border)
      hipLaunchKernelGGL(bf::dgrad_border5_add_k, dim3(ceil_div((long)N * T, 16), ceil_div(Cx, 64)), dim3(256), 0, s,
                       slab, ks5, Mt, Cx, dx, N, H, W, lt, ll);
    return check_launch("conv2d_dgrad_refl");
  }
  const int NB = bf::dgrad_border_rows(H, W), K = 9 * Cy;
  if (math == VST_MATH_BF16X6) {
    using T = bf::Tile<256, 128, 64, 64, 32, 3>;
    const int nk = (K + T::BK - 1) / T::BK, spk = (nk + ks - 1) / ks;
    const dim3 grid(ceil_div(Mb, 256) * ceil_div(Cx, 128) * ks);
    hipLaunchKernelGGL((bf::conv_fprop_bf_k<T, true, 4, true>), grid, dim3(T::NT), 0, s, dy, wb, wps, nullptr, dx, H,
                       W, Cy, H, NB, Cx, 3, 1, 1, 1, 0, VST_ACT_NONE, 0.f, (int)Mb, K, 0, nullptr, spk, slab, nullptr);
  } else {
    using T = bf::Tile<128, 128, 64, 32, 32, 2>;
    const int nk = (K + T::BK - 1) / T::BK, spk = (nk + ks - 1) / ks;
    const dim3 grid(ceil_div(Mb, 128) * ceil_div(Cx, 128) * ks);
    hipLaunchKernelGGL((bf::conv_fprop_bf_k<T, true, 4, true>), grid, dim3(T::NT), 0, s, dy, wb, wps, nullptr, dx, H,
                       W, Cy, H, NB, Cx, 3, 1, 1, 1, 0, VST_ACT_NONE, 0.f, (int)Mb, K, 0, nullptr, spk, slab, nullptr);
  }
  if (add_border)
    hipLaunchKernelGGL(bf::dgrad_border_add_k, dim3(ceil_div(Mb, 16), ceil_div(Cx, 64)), dim3(256), 0, s, slab, ks,
                       (int)Mb, Cx, dx, H, W, NB);
  return check_launch("conv2d_dgrad_refl");
}

// vst_conv2d_dgrad_refl_in_epi's data-gradient half: the interior conv (whole 256x128 x6 rounds; a split-K
// tail, or the all-split form, through fprop_splitk_reduce_inb_k) with the IN-backward partials of the layer
// below in its epilogue (InbArgs), the K-restricted border GEMM, and dgrad_border5_add_inb_k (the border add
// + the partials' correction slices).  part = [N][ns][Cx][3], ns = bf_dgrad_refl1_inb_slices: the H W / 32
// row groups, then ceil((2W + 2H) / 16) border slices.
int bf_dgrad_refl1_inb_slices(int H, int W) { return H * W / 32 + (2 * W + 2 * H + 15) / 16; }

bool bf_dgrad_refl1_inb_ok(int N, int H, int W, int Cy, int Cx, int math) {
  if (math != VST_MATH_BF16X6 || !g_border5 || !bf_dgrad_refl1_ok(N, H, W, Cy, Cx, math) || (H * W) % 32) return false;
  int kd, m_split, tail_kind, m_first, fks;
  const long M = (long)N * H * W;
  if (M > (1L << 30)) return false;
  bf_plan(M, Cx, math, -1, &kd, &m_split, &tail_kind);
  bf_split_plan(M, Cx, Cy, 3, 3, math, -1, &m_first, &fks);
  if (fks && !m_first) return true;  // the whole conv as split-K 256x128 tiles
  return kd == 7 && (!m_split || (fks && m_first == m_split));
}

int bf_dgrad_refl1_inb_launch(const float* dy, const void* wsplit, long wps, const float* addend, float* dx, int N,
                              int H, int W, int Cy, int Cx, int math, hipStream_t s, float* ws, size_t ws_floats,
                              const float* z, const float* st, double* part, int act, float slope,
                              const __bf16* apl, long pps) {
  VST_REQUIRE(bf_dgrad_refl1_inb_ok(N, H, W, Cy, Cx, math), "conv2d_dgrad_refl_in_epi: unsupported shape / arithmetic");
  const long M = (long)N * H * W;
  int kd, m_split, tail_kind, m_first, fks;
  bf_plan(M, Cx, math, -1, &kd, &m_split, &tail_kind);
  bf_split_plan(M, Cx, Cy, 3, 3, math, -1, &m_first, &fks);
  const size_t main_ws = bf_fprop_ws_floats(M, Cx, Cy, 3, 3, math);
  int ks5, lt, ll;
  bf_border5_plan(N, H, W, Cy, Cx, &ks5, &lt, &ll);
  const int Mt = 2 * lt + 2 * ll, K5 = 3 * Cy, K = 9 * Cy;
  VST_REQUIRE(ws_floats >= main_ws + (size_t)ks5 * Mt * Cx, "conv2d_dgrad_refl_in_epi: workspace too small");
  const bf::InbArgs inb{z, st, part, act, slope, bf_dgrad_refl1_inb_slices(H, W)};
  const __bf16* wb = reinterpret_cast<const __bf16*>(wsplit);
  using T = bf::Tile<256, 128, 64, 64, 32, 3>;
  // rows [0, mb): whole rounds with the partials in the epilogue; [mb, M): split-K + the reducing pass
  const long mb = (fks && !m_first) ? 0 : (m_split ? m_split : M);
  if (mb > 0) {
    const dim3 grid(ceil_div(mb, 256) * ceil_div(Cx, 128));
    if (apl)
      hipLaunchKernelGGL((bf::conv_fprop_bf_inb_k<T, true>), grid, dim3(T::NT), 0, s, dy, wb, wps, dx, H, W, Cy, Cx,
                         addend, (int)mb, K, inb, apl, pps);
    else
      hipLaunchKernelGGL((bf::conv_fprop_bf_inb_k<T>), grid, dim3(T::NT), 0, s, dy, wb, wps, dx, H, W, Cy, Cx, addend,
                         (int)mb, K, inb);
  }
  if (mb < M) {
    const int nk = (K + T::BK - 1) / T::BK, spk = (nk + fks - 1) / fks;
    const dim3 grid(ceil_div(M - mb, 256) * ceil_div(Cx, 128) * fks);
    if (apl)
      hipLaunchKernelGGL((bf::conv_fprop_bf_k<T, true, 0, true, true>), grid, dim3(T::NT), 0, s, dy, wb, wps, nullptr, dx,
                         H, W, Cy, H, W, Cx, 3, 1, 1, 1, 0, VST_ACT_NONE, 0.f, (int)M, K, (int)mb, nullptr, spk, ws,
                         nullptr, 0, apl, pps);
    else
      hipLaunchKernelGGL((bf::conv_fprop_bf_k<T, true, 0, true>), grid, dim3(T::NT), 0, s, dy, wb, wps, nullptr, dx, H,
                         W, Cy, H, W, Cx, 3, 1, 1, 1, 0, VST_ACT_NONE, 0.f, (int)M, K, (int)mb, nullptr, spk, ws,
                         nullptr);
    hipLaunchKernelGGL(bf::fprop_splitk_reduce_inb_k, dim3(ceil_div(M - mb, 32), ceil_div(Cx, 64)), dim3(256), 0, s, ws,
                       fks, (int)mb, (int)M, Cx, dx, H * W, addend, inb);
  }
  float* slab = ws + main_ws;
  {
    using T5 = bf::Tile<128, 128, 64, 32, 32, 3>;
    const int nk = (K5 + T5::BK - 1) / T5::BK, spk = (nk + ks5 - 1) / ks5;
    const dim3 grid(Mt / 128 * ceil_div(Cx, 128) * ks5);
    if (apl)  // dy given as planes only (its fp32 image is not written): the border rows read them
      hipLaunchKernelGGL((bf::conv_fprop_bf_k<T5, true, 5, true, true>), grid, dim3(T5::NT), 0, s, dy, wb, wps, nullptr,
                         dx, H, W, Cy, lt, ll, Cx, 3, N, 1, 1, 0, VST_ACT_NONE, 0.f, Mt, K5, 0, nullptr, spk, slab,
                         nullptr, 0, apl, pps);
    else
      hipLaunchKernelGGL((bf::conv_fprop_bf_k<T5, true, 5, true>), grid, dim3(T5::NT), 0, s, dy, wb, wps, nullptr, dx,
                         H, W, Cy, lt, ll, Cx, 3, N, 1, 1, 0, VST_ACT_NONE, 0.f, Mt, K5, 0, nullptr, spk, slab, nullptr);
  }
  hipLaunchKernelGGL(bf::dgrad_border5_add_inb_k, dim3(ceil_div(2 * W + 2 * H, 16), N, ceil_div(Cx, 64)), dim3(256), 0,
                     s, slab, ks5, Mt, Cx, dx, H, W, lt, ll, inb, H * W / 32);
  return check_launch("conv2d_dgrad_refl_in_epi");
}

// The four phases of a stride-2 ConvTranspose2d(k3, p1, op1) forward as one conv_convT_phases_k launch
// (ws[ph], ph = 2a + b: the phase packs' bf16 planes).  128x128 tiles (128x64 for Cop <= 64); C a
// multiple of the K-slice (32).
bool bf_convT_phases_ok(int C, int Cop, int math) {
  return math != VST_MATH_F32 && VST_BF_KSLICE && C % 32 == 0 && Cop % 4 == 0;
}

// The phase tile (x6): Cop > 64 on 256x128 (8 waves of 64x64) unless its grid's rounds cost more than the
// 128x128 tile's (the N = 4 PatchGAN data gradients: 68 blocks, 77 us vs 51 us), Cop <= 64 on 64x64 (4 waves of
// 32x32).  Round 5
// sweep (profiles/r05e_convT_wgrad_tiles.jsonl, same box): the 256 -> 128 ConvTranspose / stride-2 data
// gradient 144 -> 124 us at N = 8 (188 -> 167 at N = 12) against 128x128 tiles of 8 x (64x32) waves; the
// 128 -> 64 one 150 -> 145 us against 128x64.  g_convt_tile (developer A/B): 0 = the round-4 tiles
// (128x128 8 waves / 128x64 4 waves), 1 = 256x128 / 128x64, 2 = 128x128 4 waves / 64x64; -1 = the default.
static constexpr int g_convt_tile = -1;

int bf_convT_phases_launch(const float* x, const void* const ws[4], const float* bias, float* y, int N, int H, int W,
                           int C, int Cop, int act, float slope, int math, hipStream_t s, int full) {
  VST_REQUIRE(bf_convT_phases_ok(C, Cop, math), "convT phases: unsupported shape / arithmetic");
  const int bn = Cop <= 64 ? 64 : 128;
  // the concatenated grid of the four phases on bm-row tiles (each job on a multiple of 8 blocks)
  auto grid_of = [&](int bm_, bf::PhaseJobs* jb) {
    int tt = 0;
    for (int j = 0; j < 4; ++j) {
      const int ph = j == 0 ? 3 : (j == 1 ? 1 : (j == 2 ? 2 : 0)), a = ph >> 1, b = ph & 1;
      if (jb) {
        jb->ws[j] = reinterpret_cast<const __bf16*>(ws[ph]);
        jb->t0[j] = tt;
      }
      const long rows = (long)N * (H + (full ? 1 : a)) * (W + (full ? 1 : b));
      const long tiles = (rows + bm_ - 1) / bm_ * ((Cop + bn - 1) / bn);
      tt += (int)((tiles + 7) / 8 * 8);
    }
    if (jb) jb->t0[4] = tt;
    return tt;
  };
  int tk = math != VST_MATH_BF16X6 ? 0 : (g_convt_tile >= 0 ? g_convt_tile : (bn == 128 ? 1 : 2));
  if (math == VST_MATH_BF16X6 && g_convt_tile < 0 && bn == 128) {
    // 256x128 only where its rounds cost less than the 8-wave 128x128 tile's (one block per CU either way;
    // a 32-deep K-step ~2.25 vs ~1.5 us): the small grids (the PatchGAN k4s2 data gradients at N = 4, 68
    // blocks of 256x128) keep 128x128
    const long r256 = (grid_of(256, nullptr) + VST_NUM_CUS - 1) / VST_NUM_CUS;
    const long r128 = (grid_of(128, nullptr) + VST_NUM_CUS - 1) / VST_NUM_CUS;
    tk = r256 * 2.25 <= r128 * 1.5 ? 1 : 0;
  }
  const int bm = (tk == 1 && bn == 128) ? 256 : ((tk == 2 && bn == 64) ? 64 : 128);
  bf::PhaseJobs jobs;
  const int t = grid_of(bm, &jobs);
#define VST_CTB(BM_, BN_, WM_, WN_)                                                                       \
  {                                                                                                        \
    using T = bf::Tile<BM_, BN_, WM_, WN_, 32, 3>;                                                         \
    hipLaunchKernelGGL(bf::conv_convT_phases_k<T>, dim3(t), dim3(T::NT), 0, s, x, jobs, bias, y, N, H, W, C, Cop, \
                       act, slope, full);                                                                  \
  }
#define VST_CT(BN_, WN_, NP_)                                                                             \
  {                                                                                                        \
    using T = bf::Tile<128, BN_, 64, WN_, 32, NP_>;                                                        \
    hipLaunchKernelGGL(bf::conv_convT_phases_k<T>, dim3(t), dim3(T::NT), 0, s, x, jobs, bias, y, N, H, W, C, Cop, \
                       act, slope, full);                                                                  \
  }
  if (math == VST_MATH_BF16X6 && tk == 1) {
    if (bn == 64) VST_CT(64, 32, 3) else VST_CTB(256, 128, 64, 64)
  } else if (math == VST_MATH_BF16X6 && tk == 2) {
    if (bn == 64) VST_CTB(64, 64, 32, 32) else VST_CTB(128, 128, 64, 64)
  } else if (math == VST_MATH_BF16X6) {
    if (bn == 64) VST_CT(64, 32, 3) else VST_CT(128, 32, 3)
  } else {
    if (bn == 64) VST_CT(64, 32, 2) else VST_CT(128, 32, 2)
  }
#undef VST_CT
#undef VST_CTB
  return check_launch("conv2d_convT_s2");
}

void bf_nhwc_to_planes(const float* x, void* y, long P, int Cs, int np, hipStream_t s, int row_in, int row_out) {
  const dim3 g((unsigned)((P + 63) / 64), ceil_div(Cs, 64));
  __bf16* yb = reinterpret_cast<__bf16*>(y);
  if (np == 3)
    hipLaunchKernelGGL(bf::nhwc_to_cp_planes_k<3>, g, dim3(256), 0, s, x, yb, P, Cs, rk_cp_ld(P), row_in, row_out);
  else
    hipLaunchKernelGGL(bf::nhwc_to_cp_planes_k<2>, g, dim3(256), 0, s, x, yb, P, Cs, rk_cp_ld(P), row_in, row_out);
}

void bf_wgrad_launch(const float* xt, const void* dyp, float* slab, int N, int H, int W, int Cx, int Ho,
                     int Wo, int Cyp, int S, int pad, int st, int Mw, int chunk, int nsplit, int kind, int math,
                     hipStream_t s) {
  const int P = N * Ho * Wo;
  const long ldx = rk_cp_ld((long)N * (H + 2 * pad) * (W + 2 * pad)), ldy = rk_cp_ld(P);
  const __bf16* d = reinterpret_cast<const __bf16*>(dyp);
  const long dps = (long)Cyp * ldy;
#define VST_BW(BM_, BN_, WM_, WN_, BK_, NP_)                                                          \
  {                                                                                                 \
    using T = bf::Tile<BM_, BN_, WM_, WN_, BK_, NP_>;                                              \
    const dim3 grid(ceil_div(Mw, BM_) * ceil_div(Cyp, BN_) * nsplit);                              \
    if (Wo >= BK_)                                                                                  \
      hipLaunchKernelGGL((bf::conv_wgrad_bf_k<T, true>), grid, dim3(T::NT), 0, s, xt, d, dps, slab, H, W, \
                         Cx, Ho, Wo, Cyp, S, pad, st, Mw, P, chunk, ldx, ldy);                      \
    else                                                                                            \
      hipLaunchKernelGGL((bf::conv_wgrad_bf_k<T, false>), grid, dim3(T::NT), 0, s, xt, d, dps, slab, H, W, \
                         Cx, Ho, Wo, Cyp, S, pad, st, Mw, P, chunk, ldx, ldy);                      \
  }
  if (math == VST_MATH_BF16X6) {
    VST_BF_DISPATCH(kind, 3, VST_BW)
  } else {
    VST_BF_DISPATCH(kind, 2, VST_BW)
  }
#undef VST_BW
}

bool bf_wgrad_nhwc_ok(int kind, int Wo, int Cx, int Cyp) {
  return VST_BF_MF16 && (kind == 7 || kind == 0) && Wo % 32 == 0 && Cx % 8 == 0 && Cyp % 8 == 0;
}

// kind 7: 256x128 tiles (8 waves of 64x64); kind 0: 128x128 (8 waves of 64x32).  bf32: dy fp32 NHWC (pps unused)
void bf_wgrad_nhwc_launch(const float* x, const void* dy, long pps, bool bf32, float* slab, int N, int H, int W,
                          int Cx, int Ho, int Wo, int Cyp, int S, int pad, int st, int reflect, int Mw, int chunk,
                          int nsplit, int kind, hipStream_t s, float* dwd, int dco, int dacc) {
  const int P = N * Ho * Wo;
#define VST_WN(BM_, WN_)                                                                                         \
  {                                                                                                              \
    using T = bf::Tile<BM_, 128, 64, WN_, 32, 3>;                                                                \
    const dim3 grid(ceil_div(Mw, T::BM) * ceil_div(Cyp, T::BN) * nsplit);                                       \
    if (bf32)                                                                                                    \
      hipLaunchKernelGGL((bf::conv_wgrad_nhwc_k<T, true>), grid, dim3(T::NT), 0, s, x, dy, pps, slab, H, W, Cx,  \
                         Ho, Wo, Cyp, S, pad, st, reflect, Mw, P, chunk, dwd, dco, dacc);                        \
    else                                                                                                         \
      hipLaunchKernelGGL((bf::conv_wgrad_nhwc_k<T, false>), grid, dim3(T::NT), 0, s, x, dy, pps, slab, H, W, Cx, \
                         Ho, Wo, Cyp, S, pad, st, reflect, Mw, P, chunk, dwd, dco, dacc);                        \
  }
  if (kind == 7) VST_WN(256, 64) else VST_WN(128, 32)
#undef VST_WN
}

void bf_wgrad_geom(int kind, int math, int* bm, int* bn, int* bk, int* slots) {
  int sl;
  bf_geom(kind, math == VST_MATH_BF16X6 ? 3 : 2, bm, bn, &sl);
  *bk = 32;
  *slots = sl * VST_NUM_CUS;
}

}  // namespace vst

using namespace vst;

extern "C" const char* vst_build_info(void) {
#define VST_STR2(x) #x
#define VST_STR(x) VST_STR2(x)
#if VST_BF_MF16
#define VST_X6_MFMA "16x16x32"
#else
#define VST_X6_MFMA "32x32x16"
#endif
  return "x6_mfma=" VST_X6_MFMA " x3_mfma=32x32x16 kslice=" VST_STR(VST_BF_KSLICE) " x6_256=" VST_STR(VST_BF_X6_256)
         " m16_store=" VST_STR(VST_M16_STORE) " m16_sched=" VST_STR(VST_M16_SCHED);
#undef VST_X6_MFMA
#undef VST_STR
#undef VST_STR2
}

extern "C" int vst_weight_split(const float* w, void* out, long n, void* stream) {
  VST_REQUIRE(w && out && n > 0, "weight_split: bad args");
  hipLaunchKernelGGL(bf::split3_k, dim3(ceil_div(n, 256)), dim3(256), 0, (hipStream_t)stream, w,
                     reinterpret_cast<__bf16*>(out), n);
  return check_launch("weight_split");
}

extern "C" size_t vst_conv2d_dgrad_refl_ws_bytes(int N, int H, int W, int Cy, int Cx, int math) {
  if (!bf_dgrad_refl1_ok(N, H, W, Cy, Cx, math)) return 0;
  return bf_dgrad_refl1_ws_floats(N, H, W, Cy, Cx, math) * sizeof(float);
}

extern "C" int vst_conv2d_dgrad_refl(const float* dy, const void* wsplit, const float* addend, float* dx, float* ws,
                                     size_t ws_bytes, int N, int H, int W, int Cy, int Cx, int math, void* stream) {
  VST_REQUIRE(dy && wsplit && dx && ws, "conv2d_dgrad_refl: null pointer");
  if (!bf_dgrad_refl1_ok(N, H, W, Cy, Cx, math)) {
    ::vst::set_error("conv2d_dgrad_refl: needs split-bf16 math, Cy %% 32 == 0, Cx %% 4 == 0, H, W >= 4");
    return VST_EUNSUPPORTED;
  }
  return bf_dgrad_refl1_launch(dy, wsplit, (long)Cx * 9 * Cy, addend, dx, N, H, W, Cy, Cx, math, (hipStream_t)stream,
                               ws, ws_bytes / sizeof(float), true);
}
