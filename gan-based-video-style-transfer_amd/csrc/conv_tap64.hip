// Direct kernel for the generator's 64 -> 3 (padded 4) 7x7 convolutions: the last layer's forward
// (ReflectionPad2d(3) + Conv2d(64 -> 3, 7x7) + Tanh, reference networks.py:365-367) and the data
// gradient of the first layer (ReflectionPad2d(3) + Conv2d(3 -> 64, 7x7), networks.py:340-343: the full
// correlation of the 64-channel output gradient with the rotated taps over a zero-padded frame, folded
// afterwards).  Same contraction as vst_tapconv_h_fwd — the (r, ci) part as an R x 1 conv whose 28
// outputs are (column tap s, channel co), then the 7 column taps summed — in ONE kernel:
//
//   z[q][s*4 + co] = sum_{r, ci} x[row(ho + r - pad)][q][ci] * w[(s, co)][r][ci]      (MFMA, x6 / x3)
//   y[ho][p][co]   = act(bias[co] + sum_s z[src(p + s - pad)][s*4 + co])              (epilogue, LDS)
//
// The implicit-GEMM route ran the R x 1 conv with 64-wide column tiles for 28 columns and wrote the
// 28-wide z to HBM for a separate tap-sum pass (~190 us + 16 us per N = 8 call at 256^2).  Here:
//   * a block (8 waves) owns a group of 1024 z columns = 1024 / W output rows; each wave 8 M-blocks of
//     16 columns x both 16-wide N-blocks (28 of 32 columns live) on v_mfma_f32_16x16x32_bf16;
//   * A (the 64-channel activations, the big operand) goes global -> registers straight as fragments
//     (a lane's 8 consecutive channels of one pixel = two 16-byte loads), split into bf16 planes in
//     registers; each M-block's next K-step load is issued as soon as its current one is split, so a
//     whole K-step (96 MFMAs) covers every load's latency; no LDS staging, no barrier in the K loop;
//   * B (the 28 x 448 pre-split weights) is read from L2 per K-step, one step ahead, into registers
//     shared by the wave's 8 M-blocks;
//   * z goes to LDS once per group and the column taps are summed there (bias + activation), the
//     output leaving as one float4 per pixel.  Summation order of the taps: tapsum_h_k's (bias, then
//     s = 0..6), so with the same z this is its result bit for bit.
#include "common.h"

namespace vst {
namespace tap64 {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));

constexpr int NT = 512;          // 8 waves
constexpr int MBW = 8;           // M-blocks (16 z columns) per wave
constexpr int GQ = 8 * MBW * 16;  // z columns per group: 1024
constexpr int CI = 64;           // input channels
constexpr int R = 7;             // kernel rows = column taps
constexpr int NZ = 4 * R;        // live z columns (s, co)
constexpr int KS = R * CI / 32;  // K-steps of 32: (r, channel half)
constexpr int ZS = 36;           // LDS floats per z column (32 + pad: 16-byte aligned float4 reads)
static_assert(GQ * ZS * 4 <= 160 * 1024, "LDS");

__device__ __forceinline__ uint32_t pack2(float a, float b) {
  const f32x2_t v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

// 8 fp32 values -> NP bf16x8 planes (hi, mid, lo: each the exact remainder's rounding)
template <int NP>
__device__ __forceinline__ void split(const float4& a, const float4& b, bf16x8_t (&o)[NP]) {
  float r[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    uint32_t q[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) q[e] = pack2(r[2 * e], r[2 * e + 1]);
    o[p] = __builtin_bit_cast(bf16x8_t, make_uint4(q[0], q[1], q[2], q[3]));
    if (p + 1 < NP) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        r[2 * e] -= __uint_as_float(q[e] << 16);
        r[2 * e + 1] -= __uint_as_float(q[e] & 0xffff0000u);
      }
    }
  }
}

// x: NHWC [N][H][W][64]; ws: the VST_PACK_SOK pack's NP bf16 planes [28][R][64] (plane stride wps);
// y: NHWC4 [N][Ho][Wo][4].  Rows of the R x 1 conv are padded by `pad` (reflect or zero), Ho = H + 2 pad
// - R + 1; the column taps read z column src(p + s - pad) (reflected, or zero outside [0, W)), Wo = W +
// 2 pad - R + 1.  A group is RI = GQ / W consecutive output rows of one image (gpi groups per image, the
// last one's rows past Ho computed and dropped).  Wave w owns z column blocks [w CBW, (w+1) CBW) of all
// RI rows, so output row rho's K-step (r, c) reads input row ho0 + rho + r - pad: the split fragments of
// input row j = rho + r are shared by the RI rows as r advances (a window of RI rows, one new row split
// per K-step instead of RI), and the loads / split VALU per MFMA drop RI-fold.
template <int NP, int ACT, bool REFL, int RI>
__global__ __launch_bounds__(NT, 1) void tap64_k(const float* __restrict__ x, const __bf16* __restrict__ ws, long wps,
                                                 const float* __restrict__ bias, float* __restrict__ y, int H, int W,
                                                 int Ho, int Wo, int pad, float slope, int gpi, int groups, int nimg,
                                                 int nseg, int outw) {
  constexpr int CBW = MBW / RI;  // column blocks per wave
  constexpr int WS = GQ / RI;    // z columns per group row: W, or a column segment of a wider row
  static_assert(CBW * RI == MBW, "RI divides the wave's M-blocks");
  __shared__ __attribute__((aligned(16))) float zl[GQ * ZS];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(x), 0, nimg * H * W * CI * (int)sizeof(float), 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<__bf16*>(ws), 0, (int)(((NP - 1) * wps + (long)NZ * R * CI) * 2), 0x00020000);
  const float4 bv = bias ? make_float4(bias[0], bias[1], bias[2], bias[3]) : make_float4(0.f, 0.f, 0.f, 0.f);
  const int kc = lane >> 4;  // this lane's 8-channel chunk of a K-step
  // B: z column n = 16 j + (lane & 15); past the 28 live ones the loads read zero
  int boff[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = 16 * j + (lane & 15);
    boff[j] = n < NZ ? (n * R * CI + 8 * kc) * 2 : -1;  // bytes
  }
  const int wpsb = (int)(wps * 2);
  auto load_b = [&](int r, int c, bf16x8_t (&b)[2][NP]) __attribute__((always_inline)) {
    const int kb = (r * CI + 32 * c) * 2;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const int off = boff[j] >= 0 ? p * wpsb + boff[j] + kb : 0x7ffffff0;
        b[j][p] = __builtin_bit_cast(bf16x8_t, __builtin_amdgcn_raw_buffer_load_b128(wrs, off, 0, 0));
      }
  };
  // this lane's z columns (one per column block, local to the group's segment)
  int colq[CBW];
#pragma unroll
  for (int cb = 0; cb < CBW; ++cb) colq[cb] = 16 * (wave * CBW + cb) + (lane & 15);
  const int rowb = W * CI * (int)sizeof(float);

  for (int g = blockIdx.x; g < groups; g += gridDim.x) {
    // group g = (image n, row group, column segment k): output columns [k outw, k outw + outw) from the WS z columns
    // starting at image column zc0 (one segment per row when WS == W: zc0 = 0, outw = Wo)
    const int k = g % nseg, gr = g / nseg;
    const int n = gr / gpi, ho0 = (gr - n * gpi) * RI;
    const int zc0 = nseg > 1 ? k * outw - pad : 0;
    // byte offsets of this lane's z columns inside an input row, or -1 outside the image (their z is never read)
    int colb[CBW];
#pragma unroll
    for (int cb = 0; cb < CBW; ++cb) {
      const int ci_ = zc0 + colq[cb];
      colb[cb] = (unsigned)ci_ < (unsigned)W ? (ci_ * CI + 8 * kc) * (int)sizeof(float) : -1;
    }
    // byte offset of window row j (input row ho0 + j - pad) of image n, or -1 for a zero-padding row
    auto row_off = [&](int j) __attribute__((always_inline)) {
      int h = ho0 + j - pad;
      bool ok = true;
      if constexpr (REFL) {
        h = reflect_idx(h, H);
      } else {
        ok = (unsigned)h < (unsigned)H;
      }
      return ok ? (n * H + h) * rowb : -1;
    };
    auto load_raw = [&](int j, int c, float4 (&raw)[CBW][2]) __attribute__((always_inline)) {
      const int ro = row_off(j);
#pragma unroll
      for (int cb = 0; cb < CBW; ++cb) {
        const int off = (ro >= 0 && colb[cb] >= 0) ? ro + colb[cb] + 128 * c : (int)0x7ffffff0;
        raw[cb][0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0));
        raw[cb][1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xrs, off + 16, 0, 0));
      }
    };
    f32x4v acc[RI][CBW][2];
#pragma unroll
    for (int rho = 0; rho < RI; ++rho)
#pragma unroll
      for (int cb = 0; cb < CBW; ++cb)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[rho][cb][j] = f32x4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int c = 0; c < 2; ++c) {
      bf16x8_t F[RI + R - 1][CBW][NP];  // window rows j = rho + r (live: RI at a time)
      {
        float4 raw[RI][CBW][2];
#pragma unroll
        for (int j = 0; j < RI; ++j) load_raw(j, c, raw[j]);
#pragma unroll
        for (int j = 0; j < RI; ++j)
#pragma unroll
          for (int cb = 0; cb < CBW; ++cb) split<NP>(raw[j][cb][0], raw[j][cb][1], F[j][cb]);
      }
      bf16x8_t b[2][NP], bn[2][NP];
      load_b(0, c, b);
      float4 rn[CBW][2];
      load_raw(RI, c, rn);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (r + 1 < R) load_b(r + 1, c, bn);
        if (r >= 1) {
#pragma unroll
          for (int cb = 0; cb < CBW; ++cb) split<NP>(rn[cb][0], rn[cb][1], F[r + RI - 1][cb]);
          if (r + 1 < R) load_raw(r + RI, c, rn);
        }
#pragma unroll
        for (int rho = 0; rho < RI; ++rho)
#pragma unroll
          for (int cb = 0; cb < CBW; ++cb)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const bf16x8_t(&ap)[NP] = F[rho + r][cb];
              // (A plane, B plane) terms of the x6 / x3 sums (conv_fprop_bf_k's set)
#define VST_T64(pa, pb) acc[rho][cb][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ap[pa], b[j][pb], acc[rho][cb][j], 0, 0, 0)
              if constexpr (NP == 3) {
                VST_T64(1, 1); VST_T64(1, 0); VST_T64(0, 1); VST_T64(0, 0); VST_T64(2, 0); VST_T64(0, 2);
              } else {
                VST_T64(1, 0); VST_T64(0, 1); VST_T64(0, 0);
              }
#undef VST_T64
            }
        if (r + 1 < R) {
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int p = 0; p < NP; ++p) b[j][p] = bn[j][p];
        }
      }
    }
    // z -> LDS: lane (column 16 j + (lane & 15), rows 4 (lane >> 4) + i) of each accumulator block
#pragma unroll
    for (int rho = 0; rho < RI; ++rho)
#pragma unroll
      for (int cb = 0; cb < CBW; ++cb)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int qq = rho * WS + 16 * (wave * CBW + cb) + 4 * (lane >> 4) + i;
            zl[qq * ZS + 16 * j + (lane & 15)] = acc[rho][cb][j][i];
          }
    __syncthreads();
    // column taps: output pixel (rho, p) of the group, bias then s = 0..6 in order (tapsum_h_k)
    const int rows = Ho - ho0 < RI ? Ho - ho0 : RI;
    const int p0 = nseg > 1 ? k * outw : 0, ow = nseg > 1 ? min(outw, Wo - p0) : Wo;
    const int outs = rows * ow;
    for (int e = t; e < outs; e += NT) {
      const int rho = e / ow, p = p0 + (e - rho * ow);
      float4 v = bv;
#pragma unroll
      for (int s = 0; s < R; ++s) {
        int c = p + s - pad;
        if constexpr (REFL) {
          c = c < 0 ? -c : (c >= W ? 2 * (W - 1) - c : c);
        }
        const bool in = (unsigned)c < (unsigned)W;  // then c - zc0 lies in [0, WS) (the segment's halo)
        const float4 zv = in ? *reinterpret_cast<const float4*>(zl + (rho * WS + c - zc0) * ZS + 4 * s)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
        v.x += zv.x;
        v.y += zv.y;
        v.z += zv.z;
        v.w += zv.w;
      }
      const long o = (((long)n * Ho + ho0 + rho) * Wo + p) * 4;
      *reinterpret_cast<float4*>(y + o) = make_float4(apply_act(v.x, ACT, slope), apply_act(v.y, ACT, slope),
                                                      apply_act(v.z, ACT, slope), apply_act(v.w, ACT, slope));
    }
    __syncthreads();  // the next group's z writes wait for every read of this one
  }
}

}  // namespace tap64

static constexpr bool g_tap64 = true;
// 1024-wide rows as column segments: groups of 4 rows x 256 z columns (250 output columns + the taps' 6-column halo)
// instead of one whole row per group — a row's K-steps each split a new input row for only one output row
// (RI = 1), 4x the operand-split VALU per MFMA of the 4-row groups (the C3 / Sintel-size last layer and the
// first layer's data gradient ran ~3.5x slower per pixel than at 256 wide).
#ifndef VST_TAP64_SEG
#define VST_TAP64_SEG 1
#endif

// Does the direct kernel take this tap conv?  64 input channels, 7 x 7, 4 (padded) outputs, x6 / x3
// math, W in {256, 512, 1024} (a group is 1024 / W whole rows, or 4 rows of a 1024-wide row's column segment),
// reflect 'same' or zero padding.
bool tap64_ok(int Cx, int R, int W, int math) {
  return g_tap64 && Cx == tap64::CI && R == tap64::R && W % 256 == 0 && tap64::GQ % W == 0 &&
         (math == VST_MATH_BF16X6 || math == VST_MATH_BF16X3);
}

int tap64_launch(const float* x, const void* wsplit, long wps, const float* bias, float* y, int N, int H, int W,
                 int pad, int reflect, int act, float slope, int math, hipStream_t s) {
  const int Ho = H + 2 * pad - tap64::R + 1, Wo = W + 2 * pad - tap64::R + 1;
  VST_REQUIRE(Ho > 0 && Wo > 0 && (!reflect || (pad < H && pad < W)), "tap64: bad padding");
  VST_REQUIRE(W % 256 == 0 && tap64::GQ % W == 0, "tap64: W must be 256, 512 or 1024");
  VST_REQUIRE((long)N * H * W * tap64::CI * 4 < 0x7ffffff0L, "tap64: input over 2 GB (32-bit buffer offsets)");
  const bool seg = VST_TAP64_SEG && W == 1024;
  const int RI = seg ? 4 : tap64::GQ / W, gpi = (Ho + RI - 1) / RI;
  const int outw = seg ? tap64::GQ / 4 - (tap64::R - 1) : Wo, nseg = seg ? (Wo + outw - 1) / outw : 1;
  const int groups = N * gpi * nseg;
  const int grid = groups < VST_NUM_CUS ? groups : VST_NUM_CUS;
  const __bf16* ws = reinterpret_cast<const __bf16*>(wsplit);
#define VST_T64K_R(NP_, ACT_, REFL_, RI_)                                                                          \
  hipLaunchKernelGGL((tap64::tap64_k<NP_, ACT_, REFL_, RI_>), dim3(grid), dim3(tap64::NT), 0, s, x, ws, wps, bias, y, \
                     H, W, Ho, Wo, pad, slope, gpi, groups, N, nseg, outw)
#define VST_T64K(NP_, ACT_)                                  \
  switch (RI * 2 + (reflect ? 1 : 0)) {                       \
    case 2: VST_T64K_R(NP_, ACT_, false, 1); break;           \
    case 3: VST_T64K_R(NP_, ACT_, true, 1); break;            \
    case 4: VST_T64K_R(NP_, ACT_, false, 2); break;           \
    case 5: VST_T64K_R(NP_, ACT_, true, 2); break;            \
    case 8: VST_T64K_R(NP_, ACT_, false, 4); break;           \
    default: VST_T64K_R(NP_, ACT_, true, 4); break;           \
  }
#define VST_T64K_ACT(NP_)                                    \
  switch (act) {                                             \
    case VST_ACT_TANH: VST_T64K(NP_, VST_ACT_TANH); break;   \
    case VST_ACT_NONE: VST_T64K(NP_, VST_ACT_NONE); break;   \
    default: return VST_EUNSUPPORTED;                        \
  }
  if (math == VST_MATH_BF16X6) {
    VST_T64K_ACT(3)
  } else {
    VST_T64K_ACT(2)
  }
#undef VST_T64K_ACT
#undef VST_T64K
#undef VST_T64K_R
  return check_launch("tapconv64 (direct)");
}

}  // namespace vst
