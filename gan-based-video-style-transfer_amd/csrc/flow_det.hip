// Deterministic warp backward (SURVEY §7 item 4, §5 "deterministic debug path"): the input gradient
// of the reference warp (utils/flowtools.py:18-32; CycleGANCon/models/cycle_gan_model.py:191-204,
// F.grid_sample bilinear / zeros padding) without floating-point atomics.  The product kernels
// (flow.hip warp_bwd_k, temporal_k) scatter with fp32 atomicAdd, whose summation order changes from
// run to run; this path fixes the order so a run can be diffed against another bit for bit:
//   1. emit:   every (output pixel p, corner k in nw, ne, sw, se order) that lands inside the frame
//              writes one 64-bit key (target pixel << 32 | 4p + k); out-of-frame corners (and, for
//              the fs_lib masked warp, invalid samples) write the sentinel ~0;
//   2. sort:   rocprim radix sort of the keys, so each target's contributions are contiguous and in
//              ascending (p, k) order;
//   3. gather: the first key of each target's run walks the run and adds w * gout[p] (negated for the
//              temporal loss, whose input gradient is -scatter(gb)) onto gx in that order, one rounding
//              per add — the order of a sequential loop over output pixels and corners.
// Debug path: selected by ops.set_deterministic(True) / VST_DETERMINISTIC=1, never by the bench.
#include "common.h"
#pragma clang fp contract(off)
#include "bilin.h"

#include <rocprim/device/device_radix_sort.hpp>

namespace vst {

static constexpr unsigned long long kSentinel = ~0ull;

__global__ void warp_det_emit_k(const float* __restrict__ flow, unsigned long long* __restrict__ keys, int N,
                                int H, int W, int align, int masked) {
  const long total = (long)N * H * W;
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= total) return;
  const int w = p % W, h = (p / W) % H, n = p / ((long)W * H);
  const long plane = (long)H * W;
  const long fo = (long)n * 2 * plane + (long)h * W + w;
  const Bilin b = bilin(h, w, flow[fo], flow[fo + plane], H, W, align);
  const bool ok = !masked || warp_valid(b, H, W);
  const long img = (long)n * plane;
  const int ys[4] = {b.y0, b.y0, b.y0 + 1, b.y0 + 1};
  const int xs[4] = {b.x0, b.x0 + 1, b.x0, b.x0 + 1};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const bool in = ok && inb(ys[k], xs[k], H, W);
    const unsigned long long t = (unsigned long long)(img + (long)ys[k] * W + xs[k]);
    keys[p * 4 + k] = in ? ((t << 32) | (unsigned long long)(p * 4 + k)) : kSentinel;
  }
}

// One key walk per run serves up to GC channels (the run's keys, flow and bilinear weights are read and
// recomputed once per GC channels, not once per channel); each channel's sum is still added in the
// run's key order, so the result is the same sequence of roundings as a channel-at-a-time walk.
constexpr int GC = 8;

__global__ void warp_det_gather_k(const unsigned long long* __restrict__ keys, long nkeys,
                                  const float* __restrict__ gout, const float* __restrict__ flow,
                                  float* __restrict__ gx, int N, int H, int W, int Cs, int Cl, int align,
                                  int negate) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nkeys) return;
  const unsigned long long key = keys[i];
  if (key == kSentinel) return;
  const unsigned long long t = key >> 32;
  if (i > 0 && (keys[i - 1] >> 32) == t) return;  // not the head of its target's run
  const long plane = (long)H * W;
  for (int c0 = 0; c0 < Cl; c0 += GC) {
    const int nc = Cl - c0 < GC ? Cl - c0 : GC;
    float s[GC];
#pragma unroll
    for (int c = 0; c < GC; ++c) s[c] = c < nc ? gx[(long)t * Cs + c0 + c] : 0.f;
    for (long j = i; j < nkeys; ++j) {
      const unsigned long long kj = keys[j];
      if (kj == kSentinel || (kj >> 32) != t) break;
      const long r = (long)(kj & 0xffffffffull);
      const long p = r >> 2;
      const int k = (int)(r & 3);
      const int w = p % W, h = (p / W) % H, n = p / ((long)W * H);
      const long fo = (long)n * 2 * plane + (long)h * W + w;
      const Bilin b = bilin(h, w, flow[fo], flow[fo + plane], H, W, align);
      const float wt = k == 0 ? b.nw : k == 1 ? b.ne : k == 2 ? b.sw : b.se;
#pragma unroll
      for (int c = 0; c < GC; ++c) {
        if (c >= nc) break;
        const float v = wt * gout[p * Cs + c0 + c];
        s[c] = s[c] + (negate ? -v : v);
      }
    }
#pragma unroll
    for (int c = 0; c < GC; ++c)
      if (c < nc) gx[(long)t * Cs + c0 + c] = s[c];
  }
}

static size_t sort_tmp_bytes(long nkeys) {
  size_t bytes = 0;
  (void)rocprim::radix_sort_keys(nullptr, bytes, (unsigned long long*)nullptr, (unsigned long long*)nullptr,
                           (size_t)nkeys, 0, 64, (hipStream_t)0);
  return bytes;
}

}  // namespace vst

using namespace vst;

extern "C" size_t vst_warp_bwd_det_ws_bytes(int N, int H, int W) {
  const long nkeys = 4L * N * H * W;
  return (size_t)nkeys * 8 * 2 + ((sort_tmp_bytes(nkeys) + 255) & ~(size_t)255) + 256;
}

extern "C" int vst_warp_bwd_input_det(const float* gout, const float* flow, float* gx, void* ws, size_t ws_bytes,
                                      int N, int H, int W, int Cs, int Cl, int align_corners, int masked,
                                      int negate, void* stream) {
  VST_REQUIRE(gout && flow && gx && ws && N > 0 && H > 0 && W > 0 && Cl > 0 && Cl <= Cs,
              "warp_bwd_input_det: bad args");
  const long total = (long)N * H * W, nkeys = 4 * total;
  VST_REQUIRE(nkeys < (1L << 32) && total < (1L << 31), "warp_bwd_input_det: frame too large (32-bit keys)");
  VST_REQUIRE(ws_bytes >= vst_warp_bwd_det_ws_bytes(N, H, W), "warp_bwd_input_det: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  char* base = reinterpret_cast<char*>(((uintptr_t)ws + 255) & ~(uintptr_t)255);
  unsigned long long* kin = reinterpret_cast<unsigned long long*>(base);
  unsigned long long* kout = kin + nkeys;
  void* tmp = reinterpret_cast<void*>(kout + nkeys);
  size_t tmp_bytes = sort_tmp_bytes(nkeys);
  hipLaunchKernelGGL(warp_det_emit_k, dim3(ceil_div(total, 256)), dim3(256), 0, s, flow, kin, N, H, W,
                     align_corners, masked);
  if (rocprim::radix_sort_keys(tmp, tmp_bytes, kin, kout, (size_t)nkeys, 0, 64, s) != hipSuccess) {
    set_error("warp_bwd_input_det: radix sort failed");
    return VST_EHIP;
  }
  hipLaunchKernelGGL(warp_det_gather_k, dim3(ceil_div(nkeys, 256)), dim3(256), 0, s, kout, nkeys, gout, flow, gx,
                     N, H, W, Cs, Cl, align_corners, negate);
  return check_launch("warp_bwd_input_det");
}
