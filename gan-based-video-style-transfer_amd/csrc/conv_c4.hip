// Direct (patch-staged) split-bf16 MFMA convolution of a 4-channel NHWC input: the generator's image
// convs — ReflectionPad2d(3) + Conv2d(3 -> 64, 7x7) (reference networks.py:340-343, the first layer)
// and the data gradient of its last layer (ReflectionPad2d(3) + Conv2d(64 -> 3, 7x7), networks.py:
// 365-366, run as a forward conv over the 4-channel output gradient with the rotated taps).
//
// The implicit-GEMM kernel (conv_fprop_bf_k<.., REFL = 3>) gathers every 8-deep K chunk of every
// output row from global memory and splits it into bf16 planes in registers: for a 7x7 filter each
// input value is gathered and split 49 times, and K = 196 is only 7 K-steps, so the per-tile pipeline
// fill and epilogue dominate (153-164 us per N = 8 call at 256^2, ~4x its MFMA time).  Here a block
// owns one output-row segment (<= 256 pixels): it stages the R input rows the segment reads (with the
// reflect / zero border applied) ONCE as pre-split bf16 planes in LDS, keeps all 64 x R x 8 x 4 weight
// planes resident in LDS for the whole (persistent) launch, and builds every A fragment straight from
// the patch: an MFMA K-step is one kernel row r — 8 taps (S padded to 8 with zero weights) x 4
// channels, the two taps of a lane's 8-deep chunk being adjacent pixels of the patch row (16
// contiguous bytes per plane).  No barrier inside the K loop; the next segment's patch is loaded into
// registers while the current one computes.
//
// Products: the x6 / x3 sums of conv_fprop_bf_k (same terms, same per-K-step order); accumulation
// fp32.  Epilogue: bias, activation, optional InstanceNorm statistics partials per 32-pixel group in
// the layout of vst_conv2d_fwd_in ([img][HW/32][Cop][2] fp64).
#include "common.h"

#include <type_traits>

#ifndef VST_C4_NOCOMPUTE
#define VST_C4_NOCOMPUTE 0  // developer timing experiment only: no MFMAs (WRONG results)
#endif
#ifndef VST_C4_NOSTORE
#define VST_C4_NOSTORE 0    // developer timing experiment only: every output / partial store dropped
#endif
#ifndef VST_C4_NOEPI
#define VST_C4_NOEPI 0      // developer timing experiment only (ring kernel): no epilogue at all
#endif
#ifndef VST_C4_NOWLDS
#define VST_C4_NOWLDS 0     // developer timing experiment only (ring kernel): weight fragments read once per segment
#endif
#if (VST_C4_NOCOMPUTE || VST_C4_NOSTORE || VST_C4_NOEPI || VST_C4_NOWLDS) && !defined(VST_DEV_VARIANT)
#error "VST_C4_NOCOMPUTE / VST_C4_NOSTORE are developer-only timing modes: build them with tools/build_variant.py"
#endif

namespace vst {
namespace c4 {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));

constexpr int NT = 512;          // 8 waves
constexpr int SEG = 256;         // output pixels per segment: 8 waves x 32 rows
constexpr int MAXR = 8;          // kernel rows (and taps per row, S padded to 8)
constexpr int COP = 64;          // output channels (one 64-wide GEMM column tile)
constexpr int PW = SEG + 8;      // patch row width in pixels (segment + 7 taps, rounded)
constexpr int PATCH_PLANE = MAXR * PW * 8;          // bytes per plane: [R][PW][4] bf16
constexpr int W_PLANE = MAXR * 4 * COP * 16;        // bytes per plane: [R][kq][64][8] bf16
constexpr int LDS_BYTES = 3 * (PATCH_PLANE + W_PLANE);
static_assert(LDS_BYTES <= 160 * 1024, "LDS");
constexpr int PF = 5;            // patch float4s prefetched per thread (R * (L + 7) <= PF * NT)
static_assert(MAXR * PW <= PF * NT, "patch prefetch coverage");

__device__ __forceinline__ uint32_t pack2(float a, float b) {
  const f32x2_t v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

#ifndef VST_C4_GRP
#define VST_C4_GRP 0  // ring kernel wave groups: 0 = waves {0-3} / {4-7}, 1 = even / odd waves
#endif
// one output-row segment: image n, output row ho, columns [wo0, wo0 + L)
struct Seg {
  int n, ho, wo0, L;
};

__device__ __forceinline__ Seg seg_of(int t, int Ho, int Wo, int nseg) {
  Seg s;
  const int row = t / nseg, q = t - row * nseg;
  s.n = row / Ho;
  s.ho = row - s.n * Ho;
  s.wo0 = q * SEG;
  s.L = q == nseg - 1 ? Wo - s.wo0 : SEG;
  return s;
}

// y[n][ho][wo][co] = act(bias[co] + sum_{r,s,c} xpad[n][ho + r][wo + s][c] * w[co][r][s][c]),
// xpad = x with a `pad` border (reflect or zero); stride 1, 4 input channels, Cop = 64.
// ws: split weight planes [NP][64][R*S*4] (plane stride wps), the VST_PACK_OK layout of the
// implicit-GEMM kernels.  grid = min(tiles, CUs), persistent over the segments t = blockIdx.x + k*grid.
template <int NP, int R, int ACT>
__global__ __launch_bounds__(NT, 1) void conv_c4_direct_k(const float* __restrict__ x, const __bf16* __restrict__ ws,
                                                           long wps, const float* __restrict__ bias,
                                                           float* __restrict__ y, int H, int W, int Ho, int Wo,
                                                           int S, int pad, int reflect, float slope,
                                                           int nseg, int T, int nimg, double* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  char* patch = smem;                      // [NP][R][PW][4] bf16
  char* wl = smem + 3 * PATCH_PLANE;       // [NP][R][kq 4][64][8] bf16
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int K = R * S * 4;

  // weights -> LDS once: 16-B chunk (r, kq, co) = taps s = 2kq, 2kq + 1 (zero past S) x 4 channels.
  // Branch-free buffer loads (a tap past S gets an out-of-range offset and reads zero), all in flight
  // together: one round trip per block instead of one per chunk.
  {
    constexpr int NCH = NP * R * 4 * COP, PER = (NCH + NT - 1) / NT;
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<__bf16*>(ws), 0, (int)((NP - 1) * wps * 2 + (long)COP * K * 2), 0x00020000);
    u32x2v lo[PER], hi[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int e = t + u * NT;
      const int p = e / (R * 4 * COP), rem = e - p * R * 4 * COP;
      const int r = rem / (4 * COP), kq = (rem / COP) & 3, co = rem % COP;
      const int base = (int)((p * wps + (long)co * K + r * S * 4) * 2);  // bytes
      const bool in = e < NCH;
      lo[u] = __builtin_amdgcn_raw_buffer_load_b64(wrs, in && 2 * kq < S ? base + 2 * kq * 8 : 0x7ffffff0, 0, 0);
      hi[u] = __builtin_amdgcn_raw_buffer_load_b64(wrs, in && 2 * kq + 1 < S ? base + (2 * kq + 1) * 8 : 0x7ffffff0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int e = t + u * NT;
      if (e >= NCH) continue;
      const int p = e / (R * 4 * COP), rem = e - p * R * 4 * COP;
      const int r = rem / (4 * COP), kq = (rem / COP) & 3, co = rem % COP;
      *reinterpret_cast<uint4*>(wl + p * W_PLANE + ((r * 4 + kq) * COP + co) * 16) =
          make_uint4(lo[u][0], lo[u][1], hi[u][0], hi[u][1]);
    }
  }

  // patch element e = (r, c): input row ho - pad + r, column wo0 - pad + c of image n
  float4 pf[PF];
  // Buffer loads through a descriptor over x: an element outside the frame (zero padding, the rows
  // past R) gets an offset past the descriptor's range and reads as zero — no branch around any load
  // (loads under branches make the wait-count pass drain vmcnt(0) at their use, behind the previous
  // segment's output stores).
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(x), 0, nimg * H * W * 16, 0x00020000);
  auto prefetch = [&](const Seg& g) __attribute__((always_inline)) {
    const int cols = g.L + 7;
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int e = t + i * NT;
      const int r = e / cols, c = e - r * cols;
      int hi = g.ho - pad + r, wi = g.wo0 - pad + c;
      bool ok;
      if (reflect) {
        hi = reflect_idx(hi, H);
        wi = reflect_idx(wi, W);
        ok = (unsigned)wi < (unsigned)W;  // columns past the last tap's reach may leave the frame
      } else {
        ok = (unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W;
      }
      ok = ok && r < R;
      const int off = ok ? ((g.n * H + hi) * W + wi) * 16 : (int)0x7ffffff0;
      pf[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0));
    }
  };
  auto store_patch = [&](const Seg& g) __attribute__((always_inline)) {
    const int cols = g.L + 7;
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int e = t + i * NT;
      const int r = e / cols, c = e - r * cols;
      // no branch (see prefetch): elements past the R rows land in row MAXR - 1, which no K-step reads
      static_assert(R < MAXR, "a spare patch row");
      float a[4] = {pf[i].x, pf[i].y, pf[i].z, pf[i].w};
      char* dst = patch + ((r < R ? r : MAXR - 1) * PW + c) * 8;
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const uint32_t q0 = pack2(a[0], a[1]), q1 = pack2(a[2], a[3]);
        *reinterpret_cast<uint2*>(dst + p * PATCH_PLANE) = make_uint2(q0, q1);
        if (p + 1 < NP) {
          a[0] -= __uint_as_float(q0 << 16);
          a[1] -= __uint_as_float(q0 & 0xffff0000u);
          a[2] -= __uint_as_float(q1 << 16);
          a[3] -= __uint_as_float(q1 & 0xffff0000u);
        }
      }
    }
  };

  // this lane's bias values (channels 16 j + 4 (lane >> 4) + q), loaded once before any prefetch so
  // the epilogue never waits behind the patch loads; scalar loads: a bias view may sit at any 4-byte
  // offset of a flat parameter buffer
  float4 bvs[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c0 = 16 * j + 4 * (lane >> 4);
    bvs[j] = bias ? make_float4(bias[c0], bias[c0 + 1], bias[c0 + 2], bias[c0 + 3]) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const int kq = lane >> 4;
  const int sub = wave;  // this wave's 32-pixel sub-tile of every segment (SEG = 8 waves x 32)
  const int HWo = Ho * Wo;
  f32x4v acc[2][4];

  // the fragments of kernel row r: A = the weight planes (4 blocks of 16 channels), B = the patch
  // pixels (2 blocks of 16).  D^T = W . X^T: a lane's accumulator holds 4 consecutive channels of one
  // pixel (pixel 16 i + (lane & 15), channels 16 j + 4 (lane >> 4) + q) and leaves as one float4.
  struct Fr {
    bf16x8_t w[NP][4], x[NP][2];
  };
  auto load_fr = [&](Fr& f, int r) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      // pixel (segment-local) 32 sub + 16 i + (lane & 15); taps 2 kq, 2 kq + 1 -> patch columns
      const int pc = 32 * sub + 16 * i + (lane & 15) + 2 * kq;
      const char* src = patch + (r * PW + pc) * 8;
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const uint2 lo = *reinterpret_cast<const uint2*>(src + p * PATCH_PLANE);
        const uint2 hi = *reinterpret_cast<const uint2*>(src + p * PATCH_PLANE + 8);
        f.x[p][i] = __builtin_bit_cast(bf16x8_t, make_uint4(lo.x, lo.y, hi.x, hi.y));
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int p = 0; p < NP; ++p)
        f.w[p][j] = *reinterpret_cast<const bf16x8_t*>(wl + p * W_PLANE + ((r * 4 + kq) * COP + 16 * j + (lane & 15)) * 16);
  };
  auto compute = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};
    Fr fr[2];  // double-buffered: row r + 1's LDS reads run under row r's MFMAs
    load_fr(fr[0], 0);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const Fr& f = fr[r & 1];
      if (r + 1 < R) load_fr(fr[(r + 1) & 1], r + 1);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          // (x-plane, w-plane) products in conv_fprop_bf_k's per-K-step order
#define VST_C4MF(pa, pb) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.w[pb][j], f.x[pa][i], acc[i][j], 0, 0, 0)
          if constexpr (NP == 3) {
            VST_C4MF(1, 1); VST_C4MF(1, 0); VST_C4MF(0, 1); VST_C4MF(0, 0); VST_C4MF(2, 0); VST_C4MF(0, 2);
          } else {
            VST_C4MF(1, 0); VST_C4MF(0, 1); VST_C4MF(0, 0);
          }
#undef VST_C4MF
        }
      __builtin_amdgcn_sched_barrier(0);  // at most two fragment sets live
    }
  };
  // bias, activation, the output float4s and the InstanceNorm partials of segment `cs`.  Stores go
  // through buffer descriptors whose range check drops the pixels past the segment (and every partial
  // of a launch without them, or of a sub-tile past the segment): no branch around any store.
  // live = false (the first pass, before any segment was computed): every store is dropped.
  auto epilogue = [&](const Seg& cs, bool live) __attribute__((always_inline)) {
    const float* yseg = y + (((long)cs.n * Ho + cs.ho) * Wo + cs.wo0) * COP;
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(yseg), 0, live && !VST_C4_NOSTORE ? cs.L * COP * (int)sizeof(float) : 0, 0x00020000);
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
        part ? part + (long)cs.n * (HWo >> 5) * COP * 2 : nullptr, 0,
        part && live && !VST_C4_NOSTORE ? (HWo >> 5) * COP * 2 * (int)sizeof(double) : 0, 0x00020000);
    const int pskip = 32 * sub < cs.L ? 0 : (1 << 30);  // a sub-tile past the segment: no partials
    const int z = (cs.ho * Wo + cs.wo0 + 32 * sub) >> 5;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c0 = 16 * j + 4 * kq;
      const float4 bv = bvs[j];
      float v[2][4];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int px = 32 * sub + 16 * i + (lane & 15);  // segment-local pixel
        v[i][0] = apply_act(acc[i][j][0] + bv.x, ACT, slope);
        v[i][1] = apply_act(acc[i][j][1] + bv.y, ACT, slope);
        v[i][2] = apply_act(acc[i][j][2] + bv.z, ACT, slope);
        v[i][3] = apply_act(acc[i][j][3] + bv.w, ACT, slope);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, f32x4v{v[i][0], v[i][1], v[i][2], v[i][3]}),
                                               yrs, (px * COP + c0) * (int)sizeof(float), 0, 0);
      }
      // InstanceNorm partials of the sub-tile's 32 pixels (one group: a launch with partials has
      // Wo % 32 == 0): d = {sum v, sum v^2} of channel c0 + q over this lane's two pixels, then a
      // butterfly reduce-scatter over the row's 16 lanes (xor 8, 4, 2 halve the 8 values, xor 1
      // completes the last): lane l ends with index 4 b3 + 2 b2 + b1 (b = bits of l), i.e. channel
      // c0 + 2 b3 + b2, value b1 (sum / sum of squares)
      double d[8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        d[2 * q] = (double)v[0][q] + (double)v[1][q];
        d[2 * q + 1] = (double)v[0][q] * v[0][q] + (double)v[1][q] * v[1][q];
      }
      // (written out: a loop over (m, n) that the compiler leaves rolled indexes d[] at run time)
      auto half = [&](auto M, auto Nn) __attribute__((always_inline)) {
        constexpr int m = decltype(M)::value, n = decltype(Nn)::value;
        const bool up = (lane & m) != 0;
#pragma unroll
        for (int u = 0; u < n / 2; ++u) {
          const double send = up ? d[u] : d[u + n / 2];
          const double keep = up ? d[u + n / 2] : d[u];
          d[u] = keep + __shfl_xor(send, m);
        }
      };
      half(std::integral_constant<int, 8>(), std::integral_constant<int, 8>());
      half(std::integral_constant<int, 4>(), std::integral_constant<int, 4>());
      half(std::integral_constant<int, 2>(), std::integral_constant<int, 2>());
      d[0] += __shfl_xor(d[0], 1);
      // lanes l and l ^ 1 hold the same value: both store it (no lane branch)
      const int co = c0 + 2 * ((lane >> 3) & 1) + ((lane >> 2) & 1);
      const int off = ((z * COP + co) * 2 + ((lane >> 1) & 1)) * (int)sizeof(double) + pskip;
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2v, d[0]), prs, off, 0, 0);
    }
  };

  // Pipeline per segment: [barrier] patch(cur) -> LDS [barrier] prefetch(next) loads, epilogue(prev)
  // stores, MFMAs(cur).  The next patch's loads and the previous segment's output stores are both
  // issued before the MFMAs, so the waits at the next patch write find them done.
  int tile = blockIdx.x;
  Seg g = seg_of(tile, Ho, Wo, nseg);
  prefetch(g);
  Seg prev = g;
  bool have_prev = false;
  // a dropped epilogue behind the first loads: the loop is entered with the same loads-then-stores
  // queue as its back edge, so the waits at the patch write stay counted (a merge with an entry state
  // without the stores makes the last one vmcnt(0))
  __builtin_amdgcn_sched_barrier(0);
  epilogue(prev, false);
  for (;;) {
    __syncthreads();  // every wave is done reading the previous patch (and the weights are in)
    store_patch(g);   // past the last segment: a re-load of the last one, never read
    __syncthreads();
    const Seg cur = g;
    const int nxt = tile + gridDim.x;
    // the loads first: the epilogue's store data registers are then never a load's destination (a
    // register an in-flight store still reads is only reusable after vmcnt(0)).  No branch around the
    // loads or the stores either, so every wait for a load stays a counted one.
    g = seg_of(nxt < T ? nxt : (tile < T ? tile : T - 1), Ho, Wo, nseg);  // past the end: a re-load
    prefetch(g);
    __builtin_amdgcn_sched_barrier(0);  // keep the loads ahead of the stores
    epilogue(prev, have_prev);
    if (tile >= T) break;
    if (32 * sub < cur.L && !VST_C4_NOCOMPUTE) compute();  // no VMEM inside: a branch here costs no wait
    prev = cur;
    have_prev = true;
    tile = nxt;
  }
}

// Row-ring form of the same conv (VST_C4_RING, default): a block owns a run of consecutive output rows
// of one image column segment, so segment ho + 1 reads six of segment ho's seven input rows.  The patch
// is a ring of MAXR = 8 row slots (padded row pr in slot pr & 7): each segment stages ONE new input row
// (segment ho + 1's last, into the slot segment ho - 1 freed) while segment ho computes, instead of all
// seven rows between two barriers — one barrier per segment, 1/7 of the split / ds_write work.  The
// eight waves run as two groups, one wave of each per SIMD: group 0 computes segment ho then runs its
// epilogue, group 1 runs segment ho - 1's epilogue then computes segment ho, so one wave's MFMAs overlap
// the other's epilogue VALU and stores on every SIMD (the lock-step form serialised them: the MFMAs
// were ~55 of 102 us at N = 8, everything else ~48).  A run that enters a new (image, column segment)
// restages all seven rows behind a barrier.  Same products, order and epilogue as conv_c4_direct_k.
template <int NP, int R, int ACT>
__global__ __launch_bounds__(NT, 1) void conv_c4_ring_k(const float* __restrict__ x, const __bf16* __restrict__ ws,
                                                         long wps, const float* __restrict__ bias,
                                                         float* __restrict__ y, int H, int W, int Ho, int Wo,
                                                         int S, int pad, int reflect, float slope, int nseg, int T,
                                                         int per, int nimg, double* __restrict__ part) {
  static_assert(R < MAXR && MAXR == 8, "ring: a free slot, slot = padded row & 7");
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  char* patch = smem;                      // [NP][8 slots][PW][4] bf16
  char* wl = smem + 3 * PATCH_PLANE;       // [NP][R][kq 4][64][8] bf16
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int K = R * S * 4;
  const int tb = blockIdx.x * per;
  const int te = tb + per < T ? tb + per : T;

  {  // weights -> LDS once (as conv_c4_direct_k)
    constexpr int NCH = NP * R * 4 * COP, PER = (NCH + NT - 1) / NT;
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<__bf16*>(ws), 0, (int)((NP - 1) * wps * 2 + (long)COP * K * 2), 0x00020000);
    u32x2v lo[PER], hi[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int e = t + u * NT;
      const int p = e / (R * 4 * COP), rem = e - p * R * 4 * COP;
      const int r = rem / (4 * COP), kq = (rem / COP) & 3, co = rem % COP;
      const int base = (int)((p * wps + (long)co * K + r * S * 4) * 2);
      const bool in = e < NCH;
      lo[u] = __builtin_amdgcn_raw_buffer_load_b64(wrs, in && 2 * kq < S ? base + 2 * kq * 8 : 0x7ffffff0, 0, 0);
      hi[u] = __builtin_amdgcn_raw_buffer_load_b64(wrs, in && 2 * kq + 1 < S ? base + (2 * kq + 1) * 8 : 0x7ffffff0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int e = t + u * NT;
      if (e >= NCH) continue;
      const int p = e / (R * 4 * COP), rem = e - p * R * 4 * COP;
      const int r = rem / (4 * COP), kq = (rem / COP) & 3, co = rem % COP;
      *reinterpret_cast<uint4*>(wl + p * W_PLANE + ((r * 4 + kq) * COP + co) * 16) =
          make_uint4(lo[u][0], lo[u][1], hi[u][0], hi[u][1]);
    }
  }

  // segment s -> image n, column segment q, output row ho (ho fastest: a block's run walks rows)
  auto segof = [&](int s) __attribute__((always_inline)) {
    Seg g;
    g.ho = s % Ho;
    const int rest = s / Ho, q = rest % nseg;
    g.n = rest / nseg;
    g.wo0 = q * SEG;
    g.L = q == nseg - 1 ? Wo - g.wo0 : SEG;
    return g;
  };
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(x), 0, nimg * H * W * 16, 0x00020000);
  // byte offset of patch element (padded row pr, column c) of segment g; out of the frame (zero padding)
  // or past the columns the segment reads: an offset past the descriptor's range (reads zero)
  auto xoff = [&](const Seg& g, int pr, int c) __attribute__((always_inline)) {
    int hi = pr - pad, wi = g.wo0 - pad + c;
    bool ok;
    if (reflect) {
      hi = reflect_idx(hi, H);
      wi = reflect_idx(wi, W);
      ok = (unsigned)wi < (unsigned)W;
    } else {
      ok = (unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W;
    }
    ok = ok && c < g.L + 7;
    return ok ? ((g.n * H + hi) * W + wi) * 16 : (int)0x7ffffff0;
  };
  // split one float4 (4 channels of a patch pixel) into the NP planes of slot pr & 7, column c
  auto put = [&](int pr, int c, const float4& v) __attribute__((always_inline)) {
    char* dst = patch + ((pr & 7) * PW + c) * 8;
    float a[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const uint32_t q0 = pack2(a[0], a[1]), q1 = pack2(a[2], a[3]);
      *reinterpret_cast<uint2*>(dst + p * PATCH_PLANE) = make_uint2(q0, q1);
      if (p + 1 < NP) {
        a[0] -= __uint_as_float(q0 << 16);
        a[1] -= __uint_as_float(q0 & 0xffff0000u);
        a[2] -= __uint_as_float(q1 << 16);
        a[3] -= __uint_as_float(q1 & 0xffff0000u);
      }
    }
  };
  // all R rows of segment g (elements past them land in the free slot g.ho + R)
  auto full_stage = [&](const Seg& g) __attribute__((always_inline)) {
    constexpr int FP = (R * (SEG + 7) + NT - 1) / NT;
    const int cols = g.L + 7;
    float4 pf[FP];
#pragma unroll
    for (int i = 0; i < FP; ++i) {
      const int e = t + i * NT, r = e / cols, c = e - r * cols;
      pf[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                             xrs, r < R ? xoff(g, g.ho + r, c) : (int)0x7ffffff0, 0, 0));
    }
#pragma unroll
    for (int i = 0; i < FP; ++i) {
      const int e = t + i * NT, r = e / cols, c = e - r * cols;
      put(g.ho + (r < R ? r : R), c < PW ? c : PW - 1, pf[i]);
    }
  };
  // one padded row of segment g's columns: thread t = column t (threads past the row write column
  // PW - 1 with zeros, a column no fragment reads)
  auto load_row = [&](const Seg& g, int pr) __attribute__((always_inline)) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xrs, xoff(g, pr, t), 0, 0));
  };
  auto put_row = [&](int pr, const float4& v) __attribute__((always_inline)) { put(pr, t < PW ? t : PW - 1, v); };

  float4 bvs[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c0 = 16 * j + 4 * (lane >> 4);
    bvs[j] = bias ? make_float4(bias[c0], bias[c0 + 1], bias[c0 + 2], bias[c0 + 3]) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const int kq = lane >> 4;
  const int sub = wave;      // this wave's 32-pixel sub-tile of every segment
  // one wave of each group per SIMD; an SGPR value, so `grp` branches are scalar (two exclusive paths,
  // each with its own counted waits) rather than exec-masked sequences of both
  const int grp = __builtin_amdgcn_readfirstlane(VST_C4_GRP ? (wave & 1) : (wave >> 2));
  const int HWo = Ho * Wo;
  f32x4v acc[2][4];

  struct Fr {
    bf16x8_t w[NP][4], x[NP][2];
  };
  auto load_fr = [&](Fr& f, int ho, int r) __attribute__((always_inline)) {
    const char* rowp = patch + ((ho + r) & 7) * PW * 8;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int pc = 32 * sub + 16 * i + (lane & 15) + 2 * kq;
      const char* src = rowp + pc * 8;
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const uint2 lo = *reinterpret_cast<const uint2*>(src + p * PATCH_PLANE);
        const uint2 hi = *reinterpret_cast<const uint2*>(src + p * PATCH_PLANE + 8);
        f.x[p][i] = __builtin_bit_cast(bf16x8_t, make_uint4(lo.x, lo.y, hi.x, hi.y));
      }
    }
    if (VST_C4_NOWLDS && r > 0) return;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int p = 0; p < NP; ++p)
        f.w[p][j] = *reinterpret_cast<const bf16x8_t*>(wl + p * W_PLANE + ((r * 4 + kq) * COP + 16 * j + (lane & 15)) * 16);
  };
  auto compute = [&](int ho) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};
    Fr fr[2];
    load_fr(fr[0], ho, 0);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const Fr& f = fr[r & 1];
      if (r + 1 < R) load_fr(fr[(r + 1) & 1], ho, r + 1);
      // product-major: the 8 accumulators' MFMAs of one (x-plane, w-plane) product back to back, so
      // consecutive MFMAs are independent (an accumulator's six products in a row wait on each other);
      // each accumulator still takes its products in conv_fprop_bf_k's order
#define VST_C4MF(pa, pb)                                                                                       \
  _Pragma("unroll") for (int i = 0; i < 2; ++i) _Pragma("unroll") for (int j = 0; j < 4; ++j) acc[i][j] =     \
      __builtin_amdgcn_mfma_f32_16x16x32_bf16((VST_C4_NOWLDS ? fr[0].w : f.w)[pb][j], f.x[pa][i], acc[i][j], 0, 0, 0);
      if constexpr (NP == 3) {
        VST_C4MF(1, 1) VST_C4MF(1, 0) VST_C4MF(0, 1) VST_C4MF(0, 0) VST_C4MF(2, 0) VST_C4MF(0, 2)
      } else {
        VST_C4MF(1, 0) VST_C4MF(0, 1) VST_C4MF(0, 0)
      }
#undef VST_C4MF
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  auto epilogue = [&](const Seg& cs, bool live) __attribute__((always_inline)) {
    if (VST_C4_NOEPI) return;
    const float* yseg = y + (((long)cs.n * Ho + cs.ho) * Wo + cs.wo0) * COP;
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(yseg), 0, live && !VST_C4_NOSTORE ? cs.L * COP * (int)sizeof(float) : 0, 0x00020000);
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
        part ? part + (long)cs.n * (HWo >> 5) * COP * 2 : nullptr, 0,
        part && live && !VST_C4_NOSTORE ? (HWo >> 5) * COP * 2 * (int)sizeof(double) : 0, 0x00020000);
    const int pskip = 32 * sub < cs.L ? 0 : (1 << 30);
    const int z = (cs.ho * Wo + cs.wo0 + 32 * sub) >> 5;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c0 = 16 * j + 4 * kq;
      const float4 bv = bvs[j];
      float v[2][4];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int px = 32 * sub + 16 * i + (lane & 15);
        v[i][0] = apply_act(acc[i][j][0] + bv.x, ACT, slope);
        v[i][1] = apply_act(acc[i][j][1] + bv.y, ACT, slope);
        v[i][2] = apply_act(acc[i][j][2] + bv.z, ACT, slope);
        v[i][3] = apply_act(acc[i][j][3] + bv.w, ACT, slope);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, f32x4v{v[i][0], v[i][1], v[i][2], v[i][3]}),
                                               yrs, (px * COP + c0) * (int)sizeof(float), 0, 0);
      }
      // partials of the sub-tile's 32 pixels: a lane's two pixels and the butterfly in fp32 (each
      // partial is a 32-term sum: relative error <= 32 * 2^-24 of its magnitude), stored as fp64 and
      // combined over the image in fp64 by in_finalize_k
      float d[8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        d[2 * q] = v[0][q] + v[1][q];
        d[2 * q + 1] = v[0][q] * v[0][q] + v[1][q] * v[1][q];
      }
      // reduce-scatter over the row's 16 lanes: levels pair lane l with 15 - l, 7 - l (in its half),
      // l ^ 2, l ^ 1 (DPP moves; each level's partner differs in the bit the level halves on, so lane l
      // ends with index 4 b3 + 2 b2 + b1, as the xor butterfly of conv_c4_direct_k)
      auto half = [&](auto M, auto Nn) __attribute__((always_inline)) {
        constexpr int m = decltype(M)::value, n = decltype(Nn)::value;
        constexpr int ctrl = m == 8 ? 0x140 : m == 4 ? 0x141 : m == 2 ? 0x4E : 0xB1;
        const bool up = (lane & m) != 0;
#pragma unroll
        for (int u = 0; u < n / 2; ++u) {
          const float send = up ? d[u] : d[u + n / 2];
          const float keep = up ? d[u + n / 2] : d[u];
          d[u] = keep + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, send),
                                                                                ctrl, 0xf, 0xf, false));
        }
      };
      half(std::integral_constant<int, 8>(), std::integral_constant<int, 8>());
      half(std::integral_constant<int, 4>(), std::integral_constant<int, 4>());
      half(std::integral_constant<int, 2>(), std::integral_constant<int, 2>());
      d[0] += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, d[0]), 0xB1, 0xf, 0xf, false));
      const int co = c0 + 2 * ((lane >> 3) & 1) + ((lane >> 2) & 1);
      const int off = ((z * COP + co) * 2 + ((lane >> 1) & 1)) * (int)sizeof(double) + pskip;
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2v, (double)d[0]), prs, off, 0, 0);
    }
  };

  if (tb >= T) return;  // block-uniform, before any barrier
  Seg g = segof(tb);
  full_stage(g);
  __syncthreads();
  Seg prev = g;
  bool have_prev = false;
  for (int s = tb; s < te; ++s) {
    const Seg cur = g;
    // segment s + 1's last row (padded row cur.ho + R; junk when s + 1 starts a new run, restaged
    // below): loaded here, written at the end of this iteration into slot (cur.ho + R) & 7 =
    // (cur.ho - 1) & 7, which segment s does not read — the load's wait then sits behind this
    // iteration's own work, with no load live across the loop edge
    // (put_row inside each group's path: after the group-0 / group-1 branches merge, the compiler's
    // wait for prow would also count the path that skips both, and drain every store: vmcnt(0))
    const float4 prow = load_row(cur, cur.ho + R);
    if (grp == 0) {
      if (32 * sub < cur.L && !VST_C4_NOCOMPUTE) compute(cur.ho);
      put_row(cur.ho + R, prow);
      epilogue(cur, true);
    } else {
      epilogue(prev, have_prev);
      if (32 * sub < cur.L && !VST_C4_NOCOMPUTE) compute(cur.ho);
      put_row(cur.ho + R, prow);
    }
    prev = cur;
    have_prev = true;
    __syncthreads();  // segment s read, segment s + 1's last row written
    if (s + 1 < te) {
      g = segof(s + 1);
      if (g.ho == 0) {  // a new image / column segment: all R rows (block-uniform)
        full_stage(g);
        __syncthreads();
      }
    }
  }
  if (grp == 1) epilogue(prev, have_prev);
}

}  // namespace c4

// Routing: does the direct kernel take this forward conv?  4 input channels, 64 outputs, stride 1,
// 7 x S (S <= 8) filters, split-bf16 math, and rows that split into whole 256-pixel segments (or one
// shorter one): a short last segment would cost a whole segment's time.  Its InstanceNorm partials
// are per 32-pixel row piece, so an image whose H*W is a multiple of 32 (the callers then ask for
// partials) must also have Wo % 32 == 0: a conv is routed the same way with and without partials.
static constexpr bool g_c4_direct = true;
static constexpr bool g_c4_ring = true;

bool c4_direct_ok(int C, int Cop, int R, int S, int st, int Ho, int Wo, int math) {
  return g_c4_direct && C == 4 && Cop == c4::COP && st == 1 && R == 7 && S >= 1 && S <= c4::MAXR &&
         (math == VST_MATH_BF16X6 || math == VST_MATH_BF16X3) && (Wo <= c4::SEG || Wo % c4::SEG == 0) &&
         (Wo % 32 == 0 || ((long)Ho * Wo) % 32 != 0);
}

int c4_direct_launch(const float* x, const void* wsplit, long wps, const float* bias, float* y, int N, int H, int W,
                     int Ho, int Wo, int R, int S, int pad, int reflect, int act, float slope, int math, double* part,
                     hipStream_t s) {
  const int nseg = (Wo + c4::SEG - 1) / c4::SEG;
  VST_REQUIRE(R == 7 && S <= c4::MAXR, "conv_c4_direct: 7 x S (S <= 8) filters only");
  VST_REQUIRE((long)N * Ho * nseg < (1L << 31), "conv_c4_direct: too many segments");
  VST_REQUIRE((long)N * H * W * 16 < 0x7ffffff0L, "conv_c4_direct: input over 2 GB (32-bit buffer offsets)");
  const int T = N * Ho * nseg;
  const int grid = T < VST_NUM_CUS ? T : VST_NUM_CUS;
  const int per = (T + VST_NUM_CUS - 1) / VST_NUM_CUS, rgrid = (T + per - 1) / per;
  const __bf16* ws = reinterpret_cast<const __bf16*>(wsplit);
  // the activation is a template argument: a runtime one makes every epilogue element evaluate all
  // of them (tanh included) and select
#define VST_C4D(NP_, ACT_)                                                                                      \
  if (g_c4_ring)                                                                                                \
    hipLaunchKernelGGL((c4::conv_c4_ring_k<NP_, 7, ACT_>), dim3(rgrid), dim3(c4::NT), 0, s, x, ws, wps, bias, y, H,  \
                       W, Ho, Wo, S, pad, reflect, slope, nseg, T, per, N, part);                                \
  else                                                                                                          \
    hipLaunchKernelGGL((c4::conv_c4_direct_k<NP_, 7, ACT_>), dim3(grid), dim3(c4::NT), 0, s, x, ws, wps, bias, y, H, \
                       W, Ho, Wo, S, pad, reflect, slope, nseg, T, N, part)
#define VST_C4D_ACT(NP_)                                \
  switch (act) {                                        \
    case VST_ACT_RELU: VST_C4D(NP_, VST_ACT_RELU); break;   \
    case VST_ACT_LRELU: VST_C4D(NP_, VST_ACT_LRELU); break; \
    case VST_ACT_TANH: VST_C4D(NP_, VST_ACT_TANH); break;   \
    default: VST_C4D(NP_, VST_ACT_NONE); break;             \
  }
  if (math == VST_MATH_BF16X6) {
    VST_C4D_ACT(3)
  } else {
    VST_C4D_ACT(2)
  }
#undef VST_C4D_ACT
#undef VST_C4D
  return check_launch("conv2d_fwd(4-channel direct)");
}

// ------------------------------------------------- reflect-pad data gradient of a 4-channel 7x7 conv
// The data gradient of ReflectionPad2d(p) + Conv2d(C -> 4, R x R) (the generator's last layer,
// networks.py:365-366) is dx = fold(dxp), dxp = the zero-pad-(R-1) full correlation of dy with the
// rotated taps over the (H+2p) x (W+2p) padded frame, fold = the reflect map back onto H x W.  Its
// interior dxp[i+p][j+p] is the zero-pad-p conv of dy (the direct 4-channel kernel, 256-wide rows);
// this pass adds the frame: every pixel whose row or column reflects a frame position (rows 1..p and
// H-1-p..H-2, columns likewise) gets, in a fixed order (q, then p ascending), the dxp values of the
// frame positions folding onto it — computed here in fp32 from dy (only the taps that reach dy: row
// q of the frame reads dy rows q - (R-1) .. q).  One writer per dx element: deterministic.
// grid (ceil(N * B / 64), C / 16), 256 threads: thread = (border pixel, 4-channel group of 16).
__global__ __launch_bounds__(256) void c4_dgrad_frame_k(const float* __restrict__ dy, const float* __restrict__ w,
                                                        float* __restrict__ dx, int N, int H, int W, int C, int R,
                                                        int pad) {
  const int rows = 2 * pad * W, B = rows + 2 * pad * (H - 2 * pad);
  const long b = (long)blockIdx.x * 64 + (threadIdx.x >> 2);
  const int cg = blockIdx.y * 16 + (threadIdx.x & 3) * 4;
  if (b >= (long)N * B || cg >= C) return;
  const int n = (int)(b / B), k = (int)(b - (long)n * B);
  int i, j;
  if (k < rows) {
    const int rr = k / W;
    i = rr < pad ? 1 + rr : H - 1 - pad + (rr - pad);
    j = k - rr * W;
  } else {  // the column bands over the rows the row bands do not hold: 0, pad + 1 .. H - 2 - pad, H - 1
    const int kk = k - rows, hr = H - 2 * pad, cc = kk / hr, t = kk - cc * hr;
    j = cc < pad ? 1 + cc : W - 1 - pad + (cc - pad);
    i = t == 0 ? 0 : (t == hr - 1 ? H - 1 : t + pad);
  }
  // padded rows / columns folding onto i / j: the direct one (i + pad) and the mirror, if any
  int qs[2], ps[2], nq = 0, np = 0;
  if (i >= 1 && i <= pad) qs[nq++] = pad - i;
  qs[nq++] = i + pad;
  if (i >= H - 1 - pad && i <= H - 2) qs[nq++] = 2 * H - 2 + pad - i;
  if (j >= 1 && j <= pad) ps[np++] = pad - j;
  ps[np++] = j + pad;
  if (j >= W - 1 - pad && j <= W - 2) ps[np++] = 2 * W - 2 + pad - j;
  const int off = R - 1;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int a = 0; a < nq; ++a)
    for (int c = 0; c < np; ++c) {
      const int q = qs[a], pp = ps[c];
      if (q == i + pad && pp == j + pad) continue;  // the interior term: the conv already wrote it
      float v[4] = {0.f, 0.f, 0.f, 0.f};  // (plain arrays: HIP's float4 members are accessor objects)
      for (int r = 0; r < R; ++r) {
        const int h = q + r - off;
        if ((unsigned)h >= (unsigned)H) continue;
        for (int s = 0; s < R; ++s) {
          const int x = pp + s - off;
          if ((unsigned)x >= (unsigned)W) continue;
          const float4 d = *reinterpret_cast<const float4*>(dy + (((long)n * H + h) * W + x) * 4);
          const float* wp = w + ((long)cg * R * R + r * R + s) * 4;
          const long cs = (long)R * R * 4;  // next output channel's taps
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const float4 ww = *reinterpret_cast<const float4*>(wp + u * cs);
            v[u] += d.x * ww.x + d.y * ww.y + d.z * ww.z + d.w * ww.w;
          }
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] += v[u];
    }
  float4* o = reinterpret_cast<float4*>(dx + (((long)n * H + i) * W + j) * C + cg);
  float4 y = *o;
  y.x += acc[0];
  y.y += acc[1];
  y.z += acc[2];
  y.w += acc[3];
  *o = y;
}

}  // namespace vst

using namespace vst;

// dx (N, H, W, C; the interior conv's output) += the reflect-fold frame terms of the data gradient of
// ReflectionPad2d(pad) + Conv2d(C -> 4, R x R); dy NHWC4, w = the VST_PACK_IKF pack [C][R][R][4] fp32.
extern "C" int vst_c4_dgrad_frame(const float* dy, const float* w, float* dx, int N, int H, int W, int C, int R,
                                  int pad, void* stream) {
  VST_REQUIRE(dy && w && dx && N > 0 && C % 16 == 0 && R >= 1 && pad >= 1 && 2 * pad + 2 <= H && 2 * pad + 2 <= W &&
                  R - 1 == 2 * pad,
              "c4_dgrad_frame: bad args (C %% 16 == 0, R = 2 pad + 1, H, W > 2 pad + 1)");
  const long B = 2L * pad * W + 2L * pad * (H - 2 * pad);
  hipLaunchKernelGGL(c4_dgrad_frame_k, dim3((unsigned)ceil_div((long)N * B, 64), C / 16), dim3(256), 0,
                     (hipStream_t)stream, dy, w, dx, N, H, W, C, R, pad);
  return check_launch("c4_dgrad_frame");
}
