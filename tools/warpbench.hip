// Developer A/B of warp kernel variants (standalone, no torch): times each variant over the bench
// shape (N=32, C=64, 436x1024) on three flows — the bench's i.i.d. N(0, 3^2) px per pixel, a smooth
// field (sum of low-frequency sinusoids, ~16 px amplitude) and zero flow — and
// checks every variant bit for bit against the product kernel (flow.hip warp_fwd_k).
// build: hipcc -O3 --offload-arch=gfx950 -o tools/warpbench tools/warpbench.hip
#include "../gan-based-video-style-transfer_amd/csrc/flow.hip"

#include <math.h>
#include <stdlib.h>

#include <vector>

namespace vst {
void set_error(const char* fmt, ...) { (void)fmt; }
}  // namespace vst

using namespace vst;

#ifndef WB_PIX
#define WB_PIX 1
#endif

// V1: XCD-banded 1-D grid (each XCD a contiguous range of (image, row, chunk) units: rows that share
// source rows run on one XCD's L2); NT: non-temporal output stores; PIX pixels per thread (w, w + 16/PIX..)
template <int CT, bool NT, int PIX>
__global__ __launch_bounds__(256) void warp_v1_k(const float* __restrict__ x, const float* __restrict__ flow,
                                                 float* __restrict__ out, int N, int H, int W, int chunks,
                                                 int align) {
  constexpr int C4 = CT;
  const int T = N * H * chunks;
  const int u = xcd_tile(blockIdx.x, T);
  const int row = u / chunks, ch = u - row * chunks;
  const int n = row / H, h = row - n * H;
  const int c4 = threadIdx.x % C4;
  const int p0 = threadIdx.x / C4;                 // 0 .. 256/C4
  constexpr int PPB = 256 / C4;                    // pixels per pass
  const long plane = (long)H * W;
  const float4* xs = reinterpret_cast<const float4*>(x) + (long)n * plane * C4 + c4;
  float4 v[PIX][4];
  Bilin b[PIX];
  int wq[PIX];
#pragma unroll
  for (int q = 0; q < PIX; ++q) {
    const int w = ch * PPB * PIX + p0 + q * PPB;
    wq[q] = w;
    const int wc = w < W ? w : W - 1;
    const long fo = (long)n * 2 * plane + (long)h * W + wc;
    b[q] = bilin(h, wc, flow[fo], flow[fo + plane], H, W, align);
  }
#pragma unroll
  for (int q = 0; q < PIX; ++q) {
    // unconditional loads from clamped corners, zeroed by select (no branches: all in flight)
    const int ya = min(max(b[q].y0, 0), H - 1), yb = min(max(b[q].y0 + 1, 0), H - 1);
    const int xa = min(max(b[q].x0, 0), W - 1), xb = min(max(b[q].x0 + 1, 0), W - 1);
    const float4 z = make_float4(0, 0, 0, 0);
    const float4 l0 = xs[(long)(ya * W + xa) * C4], l1 = xs[(long)(ya * W + xb) * C4];
    const float4 l2 = xs[(long)(yb * W + xa) * C4], l3 = xs[(long)(yb * W + xb) * C4];
    v[q][0] = inb(b[q].y0, b[q].x0, H, W) ? l0 : z;
    v[q][1] = inb(b[q].y0, b[q].x0 + 1, H, W) ? l1 : z;
    v[q][2] = inb(b[q].y0 + 1, b[q].x0, H, W) ? l2 : z;
    v[q][3] = inb(b[q].y0 + 1, b[q].x0 + 1, H, W) ? l3 : z;
  }
#pragma unroll
  for (int q = 0; q < PIX; ++q) {
    if (wq[q] >= W) continue;
    float4 o;
    o.x = bilerp(v[q][0].x, v[q][1].x, v[q][2].x, v[q][3].x, b[q].nw, b[q].ne, b[q].sw, b[q].se);
    o.y = bilerp(v[q][0].y, v[q][1].y, v[q][2].y, v[q][3].y, b[q].nw, b[q].ne, b[q].sw, b[q].se);
    o.z = bilerp(v[q][0].z, v[q][1].z, v[q][2].z, v[q][3].z, b[q].nw, b[q].ne, b[q].sw, b[q].se);
    o.w = bilerp(v[q][0].w, v[q][1].w, v[q][2].w, v[q][3].w, b[q].nw, b[q].ne, b[q].sw, b[q].se);
    float4* op = reinterpret_cast<float4*>(out) + ((long)n * plane + (long)h * W + wq[q]) * C4 + c4;
    if (NT)
      __builtin_nontemporal_store(f32x4v{o.x, o.y, o.z, o.w}, reinterpret_cast<f32x4v*>(op));
    else
      *op = o;
  }
}


// V2: the product kernel's 3-D grid (chunk, row, image) with PIX pixels per thread and optional
// non-temporal output stores
template <int CT, bool NT, int PIX>
__global__ __launch_bounds__(256) void warp_v2_k(const float* __restrict__ x, const float* __restrict__ flow,
                                                 float* __restrict__ out, int N, int H, int W, int align) {
  constexpr int C4 = CT, PPB = 256 / C4;
  const int h = blockIdx.y, n = blockIdx.z;
  const int c4 = threadIdx.x % C4, p0 = threadIdx.x / C4;
  const long plane = (long)H * W;
  const float4* xs = reinterpret_cast<const float4*>(x) + (long)n * plane * C4 + c4;
  float4 v[PIX][4];
  Bilin b[PIX];
  int wq[PIX];
#pragma unroll
  for (int q = 0; q < PIX; ++q) {
    const int w = blockIdx.x * PPB * PIX + p0 + q * PPB;
    wq[q] = w;
    const int wc = w < W ? w : W - 1;
    const long fo = (long)n * 2 * plane + (long)h * W + wc;
    b[q] = bilin(h, wc, flow[fo], flow[fo + plane], H, W, align);
  }
#pragma unroll
  for (int q = 0; q < PIX; ++q) {
    // unconditional loads from clamped corners, zeroed by select (no branches: all in flight)
    const int ya = min(max(b[q].y0, 0), H - 1), yb = min(max(b[q].y0 + 1, 0), H - 1);
    const int xa = min(max(b[q].x0, 0), W - 1), xb = min(max(b[q].x0 + 1, 0), W - 1);
    const float4 z = make_float4(0, 0, 0, 0);
    const float4 l0 = xs[(long)(ya * W + xa) * C4], l1 = xs[(long)(ya * W + xb) * C4];
    const float4 l2 = xs[(long)(yb * W + xa) * C4], l3 = xs[(long)(yb * W + xb) * C4];
    v[q][0] = inb(b[q].y0, b[q].x0, H, W) ? l0 : z;
    v[q][1] = inb(b[q].y0, b[q].x0 + 1, H, W) ? l1 : z;
    v[q][2] = inb(b[q].y0 + 1, b[q].x0, H, W) ? l2 : z;
    v[q][3] = inb(b[q].y0 + 1, b[q].x0 + 1, H, W) ? l3 : z;
  }
#pragma unroll
  for (int q = 0; q < PIX; ++q) {
    if (wq[q] >= W) continue;
    float4 o;
    o.x = bilerp(v[q][0].x, v[q][1].x, v[q][2].x, v[q][3].x, b[q].nw, b[q].ne, b[q].sw, b[q].se);
    o.y = bilerp(v[q][0].y, v[q][1].y, v[q][2].y, v[q][3].y, b[q].nw, b[q].ne, b[q].sw, b[q].se);
    o.z = bilerp(v[q][0].z, v[q][1].z, v[q][2].z, v[q][3].z, b[q].nw, b[q].ne, b[q].sw, b[q].se);
    o.w = bilerp(v[q][0].w, v[q][1].w, v[q][2].w, v[q][3].w, b[q].nw, b[q].ne, b[q].sw, b[q].se);
    float4* op = reinterpret_cast<float4*>(out) + ((long)n * plane + (long)h * W + wq[q]) * C4 + c4;
    if (NT)
      __builtin_nontemporal_store(f32x4v{o.x, o.y, o.z, o.w}, reinterpret_cast<f32x4v*>(op));
    else
      *op = o;
  }
}

#define CK(e)                                                          \
  do {                                                                 \
    hipError_t r_ = (e);                                               \
    if (r_ != hipSuccess) {                                            \
      fprintf(stderr, "%s: %s\n", #e, hipGetErrorString(r_));          \
      exit(1);                                                         \
    }                                                                  \
  } while (0)

int main() {
  const int N = 32, H = 436, W = 1024, C = 64, C4 = C / 4;
  const long npx = (long)N * H * W, nx = npx * C;
  std::vector<float> hx(nx), hf(npx * 2);
  unsigned long long s = 12345;
  auto rnd = [&]() {
    s = s * 6364136223846793005ULL + 1442695040888963407ULL;
    return ((s >> 40) & 0xffffff) / 16777216.0f;
  };
  for (long i = 0; i < nx; ++i) hx[i] = rnd() * 2.f - 1.f;
  float *dx, *df, *dout, *dref;
  CK(hipMalloc(&dx, nx * 4));
  CK(hipMalloc(&df, npx * 8));
  CK(hipMalloc(&dout, nx * 4));
  CK(hipMalloc(&dref, nx * 4));
  CK(hipMemcpy(dx, hx.data(), nx * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double bytes = npx * (8.0 * C + 8.0);
  for (int fk = 0; fk < 3; ++fk) {
    const char* fname = fk == 0 ? "iid3" : (fk == 1 ? "smooth16" : "zero");
    for (int n = 0; n < N; ++n)
      for (int h = 0; h < H; ++h)
        for (int w = 0; w < W; ++w) {
          float fx = 0.f, fy = 0.f;
          if (fk == 0) {
            const float u1 = rnd() + 1e-7f, u2 = rnd(), u3 = rnd() + 1e-7f, u4 = rnd();
            fx = 3.f * sqrtf(-2.f * logf(u1)) * cosf(6.2831853f * u2);
            fy = 3.f * sqrtf(-2.f * logf(u3)) * cosf(6.2831853f * u4);
          } else if (fk == 1) {
            fx = 16.f * sinf(0.011f * w + 0.7f * n) * cosf(0.017f * h);
            fy = 12.f * cosf(0.009f * w - 0.3f * n) * sinf(0.013f * h + 0.5f);
          }
          hf[((long)n * 2 + 0) * H * W + (long)h * W + w] = fx;
          hf[((long)n * 2 + 1) * H * W + (long)h * W + w] = fy;
        }
    CK(hipMemcpy(df, hf.data(), npx * 8, hipMemcpyHostToDevice));
    for (int v = 0; v < 6; ++v) {
      auto launch = [&](float* o) {
        const int chunks1 = (W * C4 + 255) / 256;
        switch (v) {
          case 0: warp_fwd_launch<0>(dx, df, o, N, H, W, C, 0, 0); break;
          case 1: hipLaunchKernelGGL((warp_v2_k<16, false, 1>), dim3(W / 16, H, N), dim3(256), 0, 0, dx, df, o, N, H, W, 0); break;
          case 2: hipLaunchKernelGGL((warp_v2_k<16, false, 2>), dim3(W / 32, H, N), dim3(256), 0, 0, dx, df, o, N, H, W, 0); break;
          case 3: hipLaunchKernelGGL((warp_v2_k<16, true, 2>), dim3(W / 32, H, N), dim3(256), 0, 0, dx, df, o, N, H, W, 0); break;
          case 4: hipLaunchKernelGGL((warp_v2_k<16, true, 4>), dim3(W / 64, H, N), dim3(256), 0, 0, dx, df, o, N, H, W, 0); break;
          case 5: { const int c2 = (W + 31) / 32; hipLaunchKernelGGL((warp_v1_k<16, true, 2>), dim3(N * H * c2), dim3(256), 0, 0, dx, df, o, N, H, W, c2, 0); break; }
        }
      };
      launch(v == 0 ? dref : dout);
      CK(hipDeviceSynchronize());
      bool same = true;
      if (v) {
        std::vector<float> a(nx), r(nx);
        CK(hipMemcpy(a.data(), dout, nx * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(r.data(), dref, nx * 4, hipMemcpyDeviceToHost));
        same = memcmp(a.data(), r.data(), nx * 4) == 0;
      }
      float best = 1e9;
      for (int rep = 0; rep < 3; ++rep) {
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < 10; ++i) launch(v == 0 ? dref : dout);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = fminf(best, ms / 10);
      }
      printf("{\"flow\": \"%s\", \"variant\": %d, \"ms\": %.4f, \"TBs\": %.3f, \"exact\": %s}\n", fname, v, best,
             bytes / best / 1e9, same ? "true" : "false");
      fflush(stdout);
    }
  }
  return 0;
}
