// Convolutions with at most 4 output channels on the fp32 VALU (v_fma_f32 runs at the same
// 64 FLOP/clk/SIMD as fp32 MFMA on gfx950, without padding N=3 or N=1 up to an MFMA tile).
//
// These are the image-facing layers of the reference networks
// (methods/GAN-based/CycleGAN/models/networks.py): the generator's last ReflectionPad2d(3) +
// Conv2d(ngf, 3, 7) (:365-366), the PatchGAN head Conv2d(8*ndf, 1, 4) (:578), and the data
// gradients that flow back into 3-channel images (first generator conv :340-343, first PatchGAN
// conv :556).  On the MFMA path they wasted 8-32x of their tile and, for the 30x30 PatchGAN head,
// ran on 15 workgroups.
//
//   skinny_out_k   out[p][0..3] = act(bias + sum_{tap, c} in[gather(p, tap)][c] * w[tap][c][0..3])
//                  MODE 0: forward conv gather (stride, zero/reflect pad);
//                  MODE 1: transposed-conv / data-gradient gather (per parity class in blockIdx.z,
//                          reflect mirrors for stride 1) — the same index rules as conv_tconv_k.
//                  One output pixel per KS consecutive lanes: the KS lanes split the channel loop
//                  (K-split for the 30x30 PatchGAN head, KS = 1 for the 256x256 image layers) and
//                  are combined with wave shuffles.  Weights are wave-uniform (scalar loads); the
//                  channel loop is unrolled so several 16-byte gathers are in flight per lane.
//   skinny_wgrad_k dw slab for Cyp == 4: each thread owns one (tap, 4 input channels) block of 16
//                  accumulators over a split-K pixel range (4 pixels per iteration, loads first);
//                  dy[p] is wave-uniform.
#include "common.h"

namespace vst {

// acc.{x,y,z,w} += dot(v, w_{0,1,2,3}); w_j = the 4 input-channel weights of output channel j
// (weights are the VST_PACK_OK / VST_PACK_IK packs: output channel major, k = (r, s, c) inside).
__device__ __forceinline__ void fma4x4(float4& acc, const float4& v, const float4& w0, const float4& w1,
                                       const float4& w2, const float4& w3) {
  acc.x += v.x * w0.x + v.y * w0.y + v.z * w0.z + v.w * w0.w;
  acc.y += v.x * w1.x + v.y * w1.y + v.z * w1.z + v.w * w1.w;
  acc.z += v.x * w2.x + v.y * w2.y + v.z * w2.z + v.w * w2.w;
  acc.w += v.x * w3.x + v.y * w3.y + v.z * w3.z + v.w * w3.w;
}

// C1 (MODE 0): only output channel 0 is real (the PatchGAN head, 1 channel padded to 4): the padded
// channels' weight rows are zero, so their sums are exactly 0 and are not computed — one weight
// float4 and 4 FMAs per input float4 instead of four and 16.
template <int MODE, int ST, int KS, bool C1 = false>
__global__ __launch_bounds__(256) void skinny_out_k(
    const float* __restrict__ in, const float* __restrict__ wp, const float* __restrict__ bias,
    const float* __restrict__ addend, float* __restrict__ out, int Nimg, int Hi, int Wi, int Cin,
    int Ho, int Wo, int R, int S, int st_rt, int pad, int reflect, int act, float slope) {
  const int st = ST > 0 ? ST : st_rt;
  const int ca = MODE == 1 ? blockIdx.z / st : 0, cb = MODE == 1 ? blockIdx.z % st : 0;
  const int Hc = MODE == 1 ? (Ho > ca ? (Ho - ca + st - 1) / st : 0) : Ho;
  const int Wc = MODE == 1 ? (Wo > cb ? (Wo - cb + st - 1) / st : 0) : Wo;
  const long total = (long)Nimg * Hc * Wc;
  const long gid = ((long)blockIdx.x * blockDim.x + threadIdx.x) / KS;
  const int ks = threadIdx.x % KS;
  const bool valid = gid < total;
  const long gq = valid ? gid : 0;
  const int ww = gq % Wc;
  const long q = gq / Wc;
  const int hh = q % Hc, n = q / Hc;
  const float* ib = in + (long)n * Hi * Wi * Cin;
  const long wstride = (long)R * S * Cin;  // between output channels of the OK / IK pack
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);

  if (valid) {
    if (MODE == 0) {
      for (int r = 0; r < R; ++r) {
        int hi = hh * st - pad + r;
        bool hok = true;
        if (reflect) hi = reflect_idx(hi, Hi);
        else hok = (unsigned)hi < (unsigned)Hi;
        for (int s = 0; s < S; ++s) {
          int wi = ww * st - pad + s;
          bool ok = hok;
          if (reflect) wi = reflect_idx(wi, Wi);
          else ok = ok && (unsigned)wi < (unsigned)Wi;
          if (!ok) continue;
          const float* wt = wp + (long)(r * S + s) * Cin;
          const float* src = ib + ((long)hi * Wi + wi) * Cin;
          if (C1) {
#pragma unroll 8
            for (int c = 4 * ks; c < Cin; c += 4 * KS) {
              const float4 v = *reinterpret_cast<const float4*>(src + c);
              const float4 w0 = *reinterpret_cast<const float4*>(wt + c);
              acc.x += v.x * w0.x + v.y * w0.y + v.z * w0.z + v.w * w0.w;
            }
            continue;
          }
#pragma unroll 4
          for (int c = 4 * ks; c < Cin; c += 4 * KS) {
            const float4 v = *reinterpret_cast<const float4*>(src + c);
            fma4x4(acc, v, *reinterpret_cast<const float4*>(wt + c),
                   *reinterpret_cast<const float4*>(wt + wstride + c),
                   *reinterpret_cast<const float4*>(wt + 2 * wstride + c),
                   *reinterpret_cast<const float4*>(wt + 3 * wstride + c));
          }
        }
      }
    } else {
      // transposed gather: h = ca + st*hh; taps r = r0 + st*i at ho = (h + pad - r)/st
      const int h = ca + st * hh, w = cb + st * ww;
      const int r0 = (ca + pad) % st, s0 = (cb + pad) % st;
      int hc[2] = {h + pad, -(1 << 20)}, wc[2] = {w + pad, -(1 << 20)};
      if (reflect) {
        if (h >= 1 && h <= pad) hc[1] = pad - h;
        else if (h >= Ho - 1 - pad && h <= Ho - 2) hc[1] = 2 * Ho - 2 - h + pad;
        if (w >= 1 && w <= pad) wc[1] = pad - w;
        else if (w >= Wo - 1 - pad && w <= Wo - 2) wc[1] = 2 * Wo - 2 - w + pad;
      }
      for (int r = r0; r < R; r += st) {
        for (int s = s0; s < S; s += st) {
          const float* wt = wp + (long)(r * S + s) * Cin;
#pragma unroll
          for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b) {
              const int dh = hc[a] - r, dw = wc[b] - s;
              if (dh < 0 || dw < 0) continue;
              const int ho = dh / st, wo = dw / st;
              if (ho >= Hi || wo >= Wi) continue;
              const float* src = ib + ((long)ho * Wi + wo) * Cin;
#pragma unroll 4
              for (int c = 4 * ks; c < Cin; c += 4 * KS) {
                const float4 v = *reinterpret_cast<const float4*>(src + c);
                fma4x4(acc, v, *reinterpret_cast<const float4*>(wt + c),
                       *reinterpret_cast<const float4*>(wt + wstride + c),
                       *reinterpret_cast<const float4*>(wt + 2 * wstride + c),
                       *reinterpret_cast<const float4*>(wt + 3 * wstride + c));
              }
            }
        }
      }
    }
  }
  if (KS > 1) {
#pragma unroll
    for (int o = KS / 2; o > 0; o >>= 1) {
      acc.x += __shfl_xor(acc.x, o, 64);
      acc.y += __shfl_xor(acc.y, o, 64);
      acc.z += __shfl_xor(acc.z, o, 64);
      acc.w += __shfl_xor(acc.w, o, 64);
    }
  }
  if (!valid || ks != 0) return;
  const float4 b4 = bias ? *reinterpret_cast<const float4*>(bias) : make_float4(0.f, 0.f, 0.f, 0.f);
  const int h = MODE == 1 ? ca + st * hh : hh, w = MODE == 1 ? cb + st * ww : ww;
  const long o = (((long)n * Ho + h) * Wo + w) * 4;
  float4 v;
  v.x = apply_act(acc.x + b4.x, act, slope);
  v.y = apply_act(acc.y + b4.y, act, slope);
  v.z = apply_act(acc.z + b4.z, act, slope);
  v.w = apply_act(acc.w + b4.w, act, slope);
  if (addend) add_f4(v, *reinterpret_cast<const float4*>(addend + o));
  *reinterpret_cast<float4*>(out + o) = v;
}

// skinny_out_k MODE 0 for few output pixels over a long K (the StarGAN discriminator heads: 3x3 / 4x4 taps over
// 2048 channels at 4x4, <= 128 pixels — one workgroup of the per-pixel kernel ran 150-360 us): the K range split
// over blockIdx.y = (tap, channel chunk of CC) blocks, thread (pixel, KS lane) as skinny_out_k, the lane sums
// shuffled together and the raw partial stored to g_skinny_slab[z][pixel][4]; skinny_split_reduce_k sums the
// splits in order + bias + act (+ addend).  Deterministic.
constexpr long SKINNY_SLAB = 1L << 18;  // floats
__device__ float g_skinny_slab[SKINNY_SLAB];

template <int KS>
__global__ __launch_bounds__(256) void skinny_split_k(const float* __restrict__ in, const float* __restrict__ wp,
                                                      int Nimg, int Hi, int Wi, int Cin, int Ho, int Wo, int S, int st,
                                                      int pad, int reflect, int CC) {
  const int CB = Cin / CC, z = blockIdx.y, tap = z / CB, cb = z - tap * CB;
  const int r = tap / S, s = tap - r * S;
  const long total = (long)Nimg * Ho * Wo;
  const long gid = ((long)blockIdx.x * blockDim.x + threadIdx.x) / KS;
  const int ks = threadIdx.x % KS;
  const bool valid = gid < total;
  const long gq = valid ? gid : 0;
  const int ww = gq % Wo;
  const long q = gq / Wo;
  const int hh = q % Ho, n = q / Ho;
  const long wstride = (long)gridDim.y / CB * Cin;  // R*S*Cin: between output channels of the OK pack
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  int hi = hh * st - pad + r, wi = ww * st - pad + s;
  bool ok = valid;
  if (reflect) {
    hi = reflect_idx(hi, Hi);
    wi = reflect_idx(wi, Wi);
  } else {
    ok = ok && (unsigned)hi < (unsigned)Hi && (unsigned)wi < (unsigned)Wi;
  }
  if (ok) {
    const float* wt = wp + (long)tap * Cin;
    const float* src = in + (((long)n * Hi + hi) * Wi + wi) * Cin;
#pragma unroll 4
    for (int c = cb * CC + 4 * ks; c < (cb + 1) * CC; c += 4 * KS) {
      const float4 v = *reinterpret_cast<const float4*>(src + c);
      fma4x4(acc, v, *reinterpret_cast<const float4*>(wt + c), *reinterpret_cast<const float4*>(wt + wstride + c),
             *reinterpret_cast<const float4*>(wt + 2 * wstride + c),
             *reinterpret_cast<const float4*>(wt + 3 * wstride + c));
    }
  }
#pragma unroll
  for (int o = KS / 2; o > 0; o >>= 1) {
    acc.x += __shfl_xor(acc.x, o, 64);
    acc.y += __shfl_xor(acc.y, o, 64);
    acc.z += __shfl_xor(acc.z, o, 64);
    acc.w += __shfl_xor(acc.w, o, 64);
  }
  if (valid && ks == 0) *reinterpret_cast<float4*>(g_skinny_slab + ((long)z * total + gid) * 4) = acc;
}

__global__ __launch_bounds__(256) void skinny_split_reduce_k(const float* __restrict__ bias,
                                                             const float* __restrict__ addend, float* __restrict__ out,
                                                             long total, int nsplit, int act, float slope) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= total) return;
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int z = 0; z < nsplit; ++z) add_f4(v, *reinterpret_cast<const float4*>(g_skinny_slab + ((long)z * total + p) * 4));
  const float4 b4 = bias ? *reinterpret_cast<const float4*>(bias) : make_float4(0.f, 0.f, 0.f, 0.f);
  v.x = apply_act(v.x + b4.x, act, slope);
  v.y = apply_act(v.y + b4.y, act, slope);
  v.z = apply_act(v.z + b4.z, act, slope);
  v.w = apply_act(v.w + b4.w, act, slope);
  if (addend) add_f4(v, *reinterpret_cast<const float4*>(addend + p * 4));
  *reinterpret_cast<float4*>(out + p * 4) = v;
}

// slab[z][(r*S+s)*Cx + ci][co] for co < 4, ci block of 4 per thread, pixels of split z.
__global__ __launch_bounds__(256) void skinny_wgrad_k(
    const float* __restrict__ x, const float* __restrict__ dy, float* __restrict__ slab, int H,
    int W, int Cx, int Ho, int Wo, int S, int st, int pad, int reflect, int Mw, int P, int chunk) {
  const int m4 = blockIdx.x * blockDim.x + threadIdx.x;  // (tap, ci4) block
  const int z = blockIdx.y;
  if (4 * m4 >= Mw) return;
  const int m = 4 * m4;
  const int ci = m % Cx, rs = m / Cx, r = rs / S, s = rs - (rs / S) * S;
  const int p0 = z * chunk, p1 = min(P, p0 + chunk);
  float acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = 0.f;
  const int hw = Ho * Wo;
  int n = p0 / hw, rem = p0 - (p0 / hw) * hw, ho = rem / Wo, wo = rem - (rem / Wo) * Wo;
  constexpr int U = 4;
  for (int p = p0; p < p1; p += U) {
    float4 v[U], g[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      g[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (p + u < p1) {
        int hi = ho * st - pad + r, wi = wo * st - pad + s;
        bool ok = true;
        if (reflect) {
          hi = reflect_idx(hi, H);
          wi = reflect_idx(wi, W);
        } else {
          ok = (unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W;
        }
        g[u] = *reinterpret_cast<const float4*>(dy + (long)(p + u) * 4);  // wave-uniform
        if (ok) v[u] = *reinterpret_cast<const float4*>(x + (((long)n * H + hi) * W + wi) * Cx + ci);
      }
      if (++wo == Wo) {
        wo = 0;
        if (++ho == Ho) { ho = 0; ++n; }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float vv[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        acc[a][0] += vv[a] * g[u].x;
        acc[a][1] += vv[a] * g[u].y;
        acc[a][2] += vv[a] * g[u].z;
        acc[a][3] += vv[a] * g[u].w;
      }
    }
  }
  float* sl = slab + ((long)z * Mw + m) * 4;
#pragma unroll
  for (int a = 0; a < 4; ++a)
    *reinterpret_cast<float4*>(sl + 4 * a) = make_float4(acc[a][0], acc[a][1], acc[a][2], acc[a][3]);
}

// few-pixel long-K forwards on the split kernel (skinny_split_k); g_skinny_split = false: the per-pixel kernel
static constexpr bool g_skinny_split = true;

// the PatchGAN head's one-channel forward on its row kernel (patch.hip); g_head = false: the per-pixel gather here
const bool g_head = true;

int skinny_out_launch(int mode, const float* in, const float* wp, const float* bias,
                      const float* addend, float* out, int N, int Hi, int Wi, int Cin, int Ho,
                      int Wo, int R, int S, int st, int pad, int reflect, int act, float slope,
                      hipStream_t s, int co_real) {
  const int classes = mode == 1 ? st * st : 1;
  const int Hc = mode == 1 ? (Ho + st - 1) / st : Ho, Wc = mode == 1 ? (Wo + st - 1) / st : Wo;
  const long pix = (long)N * Hc * Wc;
  // split the channel loop over lanes when there are too few output pixels to fill the chip
  int ks = 1;
  while (ks < 16 && pix * ks * classes < 256L * 1024 && 4 * ks * 2 <= Cin) ks *= 2;
#define VST_SK(M_, ST_, KS_)                                                                       \
  hipLaunchKernelGGL((skinny_out_k<M_, ST_, KS_>), dim3(ceil_div(pix * KS_, 256), 1, classes),       \
                     dim3(256), 0, s, in, wp, bias, addend, out, N, Hi, Wi, Cin, Ho, Wo, R, S, st,  \
                     pad, reflect, act, slope)
#define VST_SK_KS(M_, ST_)                      \
  switch (ks) {                                 \
    case 1: VST_SK(M_, ST_, 1); break;          \
    case 2: VST_SK(M_, ST_, 2); break;          \
    case 4: VST_SK(M_, ST_, 4); break;          \
    case 8: VST_SK(M_, ST_, 8); break;          \
    default: VST_SK(M_, ST_, 16); break;        \
  }
  if (mode == 0 && co_real == 1 && g_head && head_ok(Cin, R, S, st, reflect, Wo) && !addend)
    return head_fwd_launch(in, wp, bias, out, N, Hi, Wi, Cin, Ho, Wo, R, S, pad, act, slope, s);
  if (mode == 0 && g_skinny_split && pix * 16 <= 4096 && (long)R * S * Cin >= 4096 && Cin % 64 == 0) {
    // few pixels, long K: split the K range over workgroups (skinny_split_k)
    int CC = Cin;
    while (CC > 256 && CC % 2 == 0 && (CC / 2) % 64 == 0) CC /= 2;
    const int nsplit = R * S * (Cin / CC);
    if ((long)nsplit * pix * 4 <= SKINNY_SLAB) {
      hipLaunchKernelGGL(skinny_split_k<16>, dim3(ceil_div(pix * 16, 256), nsplit), dim3(256), 0, s, in, wp, N, Hi, Wi,
                         Cin, Ho, Wo, S, st, pad, reflect, CC);
      hipLaunchKernelGGL(skinny_split_reduce_k, dim3(ceil_div(pix, 256)), dim3(256), 0, s, bias, addend, out, pix,
                         nsplit, act, slope);
      return check_launch("skinny_out(split)");
    }
  }
  if (mode == 0 && co_real == 1) {
#define VST_SK1(KS_)                                                                                  \
  hipLaunchKernelGGL((skinny_out_k<0, 0, KS_, true>), dim3(ceil_div(pix * KS_, 256), 1, classes), dim3(256), 0, s, \
                     in, wp, bias, addend, out, N, Hi, Wi, Cin, Ho, Wo, R, S, st, pad, reflect, act, slope)
    switch (ks) {
      case 1: VST_SK1(1); break;
      case 2: VST_SK1(2); break;
      case 4: VST_SK1(4); break;
      case 8: VST_SK1(8); break;
      default: VST_SK1(16); break;
    }
#undef VST_SK1
  } else if (mode == 0) {
    VST_SK_KS(0, 0)
  } else if (st == 1) {
    VST_SK_KS(1, 1)
  } else if (st == 2) {
    VST_SK_KS(1, 2)
  } else {
    VST_SK_KS(1, 0)
  }
#undef VST_SK_KS
#undef VST_SK
  return check_launch("skinny_out");
}

int skinny_wgrad_launch(const float* x, const float* dy, float* slab, int H, int W, int Cx, int Ho,
                        int Wo, int S, int st, int pad, int reflect, int Mw, int P, int chunk,
                        int nsplit, hipStream_t s) {
  hipLaunchKernelGGL(skinny_wgrad_k, dim3(ceil_div(Mw / 4, 256), nsplit), dim3(256), 0, s, x, dy, slab,
                     H, W, Cx, Ho, Wo, S, st, pad, reflect, Mw, P, chunk);
  return check_launch("skinny_wgrad");
}

}  // namespace vst
