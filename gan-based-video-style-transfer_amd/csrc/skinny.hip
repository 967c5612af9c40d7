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
//                  Each thread owns P consecutive output pixels of one class row and keeps the
//                  4xP accumulators in registers; weights are wave-uniform (scalar loads).
//   skinny_wgrad_k dw slab for Cyp == 4: each thread owns one (tap, 4 input channels) block of 16
//                  accumulators over a split-K pixel range; dy[p] is wave-uniform.
#include "common.h"

namespace vst {

template <int P, int MODE, int ST>
__global__ __launch_bounds__(256) void skinny_out_k(
    const float* __restrict__ in, const float* __restrict__ wp, const float* __restrict__ bias,
    const float* __restrict__ addend, float* __restrict__ out, int Nimg, int Hi, int Wi, int Cin,
    int Ho, int Wo, int R, int S, int st_rt, int pad, int reflect, int act, float slope) {
  const int st = ST > 0 ? ST : st_rt;
  const int ca = MODE == 1 ? blockIdx.z / st : 0, cb = MODE == 1 ? blockIdx.z % st : 0;
  const int Hc = MODE == 1 ? (Ho > ca ? (Ho - ca + st - 1) / st : 0) : Ho;
  const int Wc = MODE == 1 ? (Wo > cb ? (Wo - cb + st - 1) / st : 0) : Wo;
  const int wgroups = (Wc + P - 1) / P;
  const long total = (long)Nimg * Hc * wgroups;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= total) return;
  const int wg = gid % wgroups;
  const long q = gid / wgroups;
  const int hh = q % Hc, n = q / Hc;
  const float* ib = in + (long)n * Hi * Wi * Cin;
  float4 acc[P];
#pragma unroll
  for (int j = 0; j < P; ++j) acc[j] = make_float4(0.f, 0.f, 0.f, 0.f);

  if (MODE == 0) {
    for (int r = 0; r < R; ++r) {
      int hi = hh * st - pad + r;
      bool hok = true;
      if (reflect) hi = reflect_idx(hi, Hi);
      else hok = (unsigned)hi < (unsigned)Hi;
      for (int s = 0; s < S; ++s) {
        const float* wt = wp + (long)(r * S + s) * Cin * 4;
        long off[P];
        bool ok[P];
#pragma unroll
        for (int j = 0; j < P; ++j) {
          const int wo = wg * P + j;
          int wi = wo * st - pad + s;
          bool wok = wo < Wo;
          if (reflect) wi = reflect_idx(wi, Wi);
          else wok = wok && (unsigned)wi < (unsigned)Wi;
          ok[j] = hok && wok;
          off[j] = ((long)hi * Wi + wi) * Cin;
        }
#pragma unroll 4
        for (int c = 0; c < Cin; c += 4) {
          const float4 w0 = *reinterpret_cast<const float4*>(wt + (c + 0) * 4);
          const float4 w1 = *reinterpret_cast<const float4*>(wt + (c + 1) * 4);
          const float4 w2 = *reinterpret_cast<const float4*>(wt + (c + 2) * 4);
          const float4 w3 = *reinterpret_cast<const float4*>(wt + (c + 3) * 4);
#pragma unroll
          for (int j = 0; j < P; ++j) {
            if (!ok[j]) continue;
            const float4 v = *reinterpret_cast<const float4*>(ib + off[j] + c);
            acc[j].x += v.x * w0.x + v.y * w1.x + v.z * w2.x + v.w * w3.x;
            acc[j].y += v.x * w0.y + v.y * w1.y + v.z * w2.y + v.w * w3.y;
            acc[j].z += v.x * w0.z + v.y * w1.z + v.z * w2.z + v.w * w3.z;
            acc[j].w += v.x * w0.w + v.y * w1.w + v.z * w2.w + v.w * w3.w;
          }
        }
      }
    }
  } else {
    // transposed gather: h = ca + st*hh; taps r = r0 + st*i at ho = (h + pad - r)/st
    const int h = ca + st * hh;
    const int r0 = (ca + pad) % st, s0 = (cb + pad) % st;
    int hcand[2] = {h + pad, -(1 << 20)};
    if (reflect) {
      if (h >= 1 && h <= pad) hcand[1] = pad - h;
      else if (h >= Ho - 1 - pad && h <= Ho - 2) hcand[1] = 2 * Ho - 2 - h + pad;
    }
    for (int r = r0; r < R; r += st) {
      for (int s = s0; s < S; s += st) {
        const float* wt = wp + (long)(r * S + s) * Cin * 4;
        long off[P][4];
        bool ok[P][4];
#pragma unroll
        for (int j = 0; j < P; ++j) {
          const int w = cb + st * (wg * P + j);
          int wcand[2] = {w + pad, -(1 << 20)};
          if (reflect) {
            if (w >= 1 && w <= pad) wcand[1] = pad - w;
            else if (w >= Wo - 1 - pad && w <= Wo - 2) wcand[1] = 2 * Wo - 2 - w + pad;
          }
#pragma unroll
          for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b) {
              const int dh = hcand[a] - r, dw = wcand[b] - s;
              const int ho = dh / st, wo = dw / st;
              ok[j][2 * a + b] = (w < Wo) && dh >= 0 && dw >= 0 && ho < Hi && wo < Wi;
              off[j][2 * a + b] = ((long)ho * Wi + wo) * Cin;
            }
        }
#pragma unroll 4
        for (int c = 0; c < Cin; c += 4) {
          const float4 w0 = *reinterpret_cast<const float4*>(wt + (c + 0) * 4);
          const float4 w1 = *reinterpret_cast<const float4*>(wt + (c + 1) * 4);
          const float4 w2 = *reinterpret_cast<const float4*>(wt + (c + 2) * 4);
          const float4 w3 = *reinterpret_cast<const float4*>(wt + (c + 3) * 4);
#pragma unroll
          for (int j = 0; j < P; ++j) {
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (ok[j][e]) {
                const float4 u = *reinterpret_cast<const float4*>(ib + off[j][e] + c);
                v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
              }
            acc[j].x += v.x * w0.x + v.y * w1.x + v.z * w2.x + v.w * w3.x;
            acc[j].y += v.x * w0.y + v.y * w1.y + v.z * w2.y + v.w * w3.y;
            acc[j].z += v.x * w0.z + v.y * w1.z + v.z * w2.z + v.w * w3.z;
            acc[j].w += v.x * w0.w + v.y * w1.w + v.z * w2.w + v.w * w3.w;
          }
        }
      }
    }
  }
  const float4 b4 = bias ? *reinterpret_cast<const float4*>(bias) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int j = 0; j < P; ++j) {
    const int ww = wg * P + j;
    if (ww >= Wc) continue;
    const int h = MODE == 1 ? ca + st * hh : hh, w = MODE == 1 ? cb + st * ww : ww;
    const long o = (((long)n * Ho + h) * Wo + w) * 4;
    float4 v;
    v.x = apply_act(acc[j].x + b4.x, act, slope);
    v.y = apply_act(acc[j].y + b4.y, act, slope);
    v.z = apply_act(acc[j].z + b4.z, act, slope);
    v.w = apply_act(acc[j].w + b4.w, act, slope);
    if (addend) add_f4(v, *reinterpret_cast<const float4*>(addend + o));
    *reinterpret_cast<float4*>(out + o) = v;
  }
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
  for (int p = p0; p < p1; ++p) {
    int hi = ho * st - pad + r, wi = wo * st - pad + s;
    bool ok = true;
    if (reflect) {
      hi = reflect_idx(hi, H);
      wi = reflect_idx(wi, W);
    } else {
      ok = (unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W;
    }
    const float4 g = *reinterpret_cast<const float4*>(dy + (long)p * 4);  // wave-uniform
    if (ok) {
      const float4 v = *reinterpret_cast<const float4*>(x + (((long)n * H + hi) * W + wi) * Cx + ci);
      const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        acc[a][0] += vv[a] * g.x;
        acc[a][1] += vv[a] * g.y;
        acc[a][2] += vv[a] * g.z;
        acc[a][3] += vv[a] * g.w;
      }
    }
    if (++wo == Wo) {
      wo = 0;
      if (++ho == Ho) { ho = 0; ++n; }
    }
  }
  float* sl = slab + ((long)z * Mw + m) * 4;
#pragma unroll
  for (int a = 0; a < 4; ++a)
    *reinterpret_cast<float4*>(sl + 4 * a) = make_float4(acc[a][0], acc[a][1], acc[a][2], acc[a][3]);
}

int skinny_out_launch(int mode, const float* in, const float* wp, const float* bias,
                      const float* addend, float* out, int N, int Hi, int Wi, int Cin, int Ho,
                      int Wo, int R, int S, int st, int pad, int reflect, int act, float slope,
                      hipStream_t s) {
  const int classes = mode == 1 ? st * st : 1;
  const int Hc = mode == 1 ? (Ho + st - 1) / st : Ho, Wc = mode == 1 ? (Wo + st - 1) / st : Wo;
  // few output pixels (PatchGAN head) -> one pixel per thread for parallelism
  const long pix = (long)N * Hc * Wc * classes;
  const bool small = mode == 1 || pix < 256L * 1024;  // P=1: more waves in flight (latency-bound)
#define VST_SK(P_, M_, ST_)                                                                        \
  {                                                                                                \
    const long tot = (long)N * Hc * ((Wc + P_ - 1) / P_);                                          \
    hipLaunchKernelGGL((skinny_out_k<P_, M_, ST_>), dim3(ceil_div(tot, 256), 1, classes), dim3(256), \
                       0, s, in, wp, bias, addend, out, N, Hi, Wi, Cin, Ho, Wo, R, S, st, pad,      \
                       reflect, act, slope);                                                        \
  }
  if (mode == 0) {
    if (small) VST_SK(1, 0, 0) else VST_SK(4, 0, 0)
  } else if (st == 1) {
    if (small) VST_SK(1, 1, 1) else VST_SK(4, 1, 1)
  } else if (st == 2) {
    if (small) VST_SK(1, 1, 2) else VST_SK(4, 1, 2)
  } else {
    VST_SK(1, 1, 0)
  }
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
