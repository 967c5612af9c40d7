// RAFT inference glue kernels (the encoders and the update block run
// on the conv kernels; these are the element-wise / layout steps between them).  All activations
// are NHWC fp32; every kernel is one streaming pass (HBM / launch bound, no reuse to stage).
//
//   raft_prep          InputPadder(replicate) + 2*(x/255)-1 + NCHW -> NHWC4       (raft.py:89-90,
//                      utils/utils.py:7-20)
//   add_relu           relu(a + b)                              (extractor.py ResidualBlock tail)
//   copy_channels      channel-block copy between NHWC tensors  (torch.cat along C)
//   raft_ctx_split     net = tanh(c[:hdim]), inp = relu(c[hdim:]) into H and the GRU concat
//                      buffers                                   (raft.py:107-109)
//   raft_flow4         flow = coords1 - coords0 as NHWC4         (raft.py:121)
//   raft_motion        [out(126) | flow(2)] into both GRU concat buffers (update.py BasicMotionEncoder
//                      tail + the cat of BasicUpdateBlock)
//   gru_reset / gru_update   SepConvGRU element-wise half-steps  (update.py:41-58)
//   raft_coords_update coords1 += delta_flow                     (raft.py:127)
//   raft_upsample      convex 8x upsampling                      (raft.py:72-83)
#include "common.h"

namespace vst {

__global__ void raft_prep_k(const float* __restrict__ img, float4* __restrict__ out, int H, int W, int Hp, int Wp,
                            int pl, int pt, long total) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int wp = i % Wp;
  const long t = i / Wp;
  const int hp = t % Hp;
  const long n = t / Hp;
  const int h = min(max(hp - pt, 0), H - 1), w = min(max(wp - pl, 0), W - 1);
  const float* src = img + n * 3 * H * W + (long)h * W + w;
  float v[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) v[c] = __fsub_rn(__fmul_rn(2.f, __fdiv_rn(src[(long)c * H * W], 255.f)), 1.f);
  out[i] = make_float4(v[0], v[1], v[2], 0.f);
}

__global__ void raft_prep_nhwc_k(const float* __restrict__ img, int cs, float4* __restrict__ out, int H, int W,
                                 int Hp, int Wp, int pl, int pt, long total) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int wp = i % Wp;
  const long t = i / Wp;
  const int hp = t % Hp;
  const long n = t / Hp;
  const int h = min(max(hp - pt, 0), H - 1), w = min(max(wp - pl, 0), W - 1);
  const float* src = img + ((n * H + h) * (long)W + w) * cs;
  float v[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) v[c] = __fsub_rn(__fmul_rn(2.f, __fdiv_rn(src[c], 255.f)), 1.f);
  out[i] = make_float4(v[0], v[1], v[2], 0.f);
}

__global__ void add_relu_k(const float4* __restrict__ a, const float4* __restrict__ b, float4* __restrict__ y,
                           long n4) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const float4 u = a[i], v = b[i];
  y[i] = make_float4(fmaxf(u.x + v.x, 0.f), fmaxf(u.y + v.y, 0.f), fmaxf(u.z + v.z, 0.f), fmaxf(u.w + v.w, 0.f));
}

// dst[p][dc0 + c] = src[p][sc0 + c], c < nc (float4 granules when everything is 4-aligned)
__global__ void copy_channels_k(const float* __restrict__ src, int scs, int sc0, float* __restrict__ dst, int dcs,
                                int dc0, int nc, long total) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const long p = i / nc;
  const int c = i - p * nc;
  dst[p * dcs + dc0 + c] = src[p * scs + sc0 + c];
}

__global__ void copy_channels4_k(const float4* __restrict__ src, int scs4, int sc04, float4* __restrict__ dst,
                                 int dcs4, int dc04, int nc4, long total) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const long p = i / nc4;
  const int c = i - p * nc4;
  dst[p * dcs4 + dc04 + c] = src[p * scs4 + sc04 + c];
}

__device__ __forceinline__ float sigm(float x) { return __fdiv_rn(1.f, __fadd_rn(1.f, expf(-x))); }

// c: [P][cs] context features; net (hdim) -> tanh -> h [P][hdim] and hx[:, 0:hdim];
// inp (cdim) -> relu -> hx[:, hdim:hdim+cdim] and rhx[:, hdim:hdim+cdim]
__global__ void raft_ctx_split_k(const float* __restrict__ c, int cs, int hdim, int cdim, float* __restrict__ h,
                                 float* __restrict__ hx, float* __restrict__ rhx, int xcs, long total) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int nch = hdim + cdim;
  const long p = i / nch;
  const int k = i - p * nch;
  const float v = c[p * cs + k];
  if (k < hdim) {
    const float t = tanhf(v);
    h[p * hdim + k] = t;
    hx[p * xcs + k] = t;
  } else {
    const float r = fmaxf(v, 0.f);
    hx[p * xcs + k] = r;
    rhx[p * xcs + k] = r;
  }
}

// flow4[p] = (x1 - x0, y1 - y0, 0, 0) with coords0 = the pixel grid; coords1 NCHW [B][2][h][w]
__global__ void raft_flow4_k(const float* __restrict__ coords1, float4* __restrict__ flow4, int h, int w,
                             long P) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const long hw = (long)h * w;
  const long n = p / hw, q = p - n * hw;
  const int y = q / w, x = q - (long)y * w;
  const float fx = __fsub_rn(coords1[(n * 2) * hw + q], (float)x);
  const float fy = __fsub_rn(coords1[(n * 2 + 1) * hw + q], (float)y);
  flow4[p] = make_float4(fx, fy, 0.f, 0.f);
}

// motion features [out[:, :nout] | flow] -> hx / rhx channels [c0, c0 + nout + 2)
__global__ void raft_motion_k(const float* __restrict__ out, int ocs, int nout, const float4* __restrict__ flow4,
                              float* __restrict__ hx, float* __restrict__ rhx, int xcs, int c0, long total) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int nm = nout + 2;
  const long p = i / nm;
  const int k = i - p * nm;
  float v;
  if (k < nout) {
    v = out[p * ocs + k];
  } else {
    const float4 f = flow4[p];
    v = k == nout ? f.x : f.y;
  }
  hx[p * xcs + c0 + k] = v;
  rhx[p * xcs + c0 + k] = v;
}

// rhx[:, 0:hd] = sigmoid(r) * h, r = zr[:, hd:2hd]
__global__ void gru_reset_k(const float* __restrict__ zr, const float* __restrict__ h, float* __restrict__ rhx,
                            int hd, int xcs, long total) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const long p = i / hd;
  const int k = i - p * hd;
  rhx[p * xcs + k] = __fmul_rn(sigm(zr[p * 2 * hd + hd + k]), h[i]);
}

// h = (1 - z) * h + z * q, z = sigmoid(zr[:, 0:hd]); written to h and hx[:, 0:hd]
__global__ void gru_update_k(const float* __restrict__ zr, const float* __restrict__ q, float* __restrict__ h,
                             float* __restrict__ hx, int hd, int xcs, long total) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const long p = i / hd;
  const int k = i - p * hd;
  const float z = sigm(zr[p * 2 * hd + k]);
  const float hn = __fadd_rn(__fmul_rn(__fsub_rn(1.f, z), h[i]), __fmul_rn(z, q[i]));
  h[i] = hn;
  hx[p * xcs + k] = hn;
}

// coords1[n][c][q] += delta[p].c (delta NHWC with channel stride dcs)
__global__ void raft_coords_update_k(float* __restrict__ coords1, const float* __restrict__ delta, int dcs,
                                     long hw, long P) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const long n = p / hw, q = p - n * hw;
  coords1[(n * 2) * hw + q] = __fadd_rn(coords1[(n * 2) * hw + q], delta[p * dcs]);
  coords1[(n * 2 + 1) * hw + q] = __fadd_rn(coords1[(n * 2 + 1) * hw + q], delta[p * dcs + 1]);
}

// out[n][c][8y+i][8x+j] = sum_k softmax_k(mask[p][k*64 + i*8 + j]) * 8 * flow[n][c](y+ky-1, x+kx-1)
// (zero outside), flow = coords1 - grid.  One thread per fine pixel.
__global__ void raft_upsample_k(const float* __restrict__ coords1, const float* __restrict__ mask, int mcs,
                                float* __restrict__ out, int h, int w, long total) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int W8 = 8 * w, H8 = 8 * h;
  const int X = i % W8;
  const long t = i / W8;
  const int Y = t % H8;
  const long n = t / H8;
  const int x = X >> 3, j = X & 7, y = Y >> 3, ii = Y & 7;
  const long hw = (long)h * w;
  const float* m = mask + (n * hw + (long)y * w + x) * mcs + ii * 8 + j;
  float mk[9], mx = -INFINITY;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    mk[k] = m[k * 64];
    mx = fmaxf(mx, mk[k]);
  }
  float den = 0.f;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    mk[k] = expf(mk[k] - mx);
    den += mk[k];
  }
  float ax = 0.f, ay = 0.f;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int yy = y + k / 3 - 1, xx = x + k % 3 - 1;
    float fx = 0.f, fy = 0.f;
    if (yy >= 0 && yy < h && xx >= 0 && xx < w) {
      const long q = (long)yy * w + xx;
      fx = 8.f * __fsub_rn(coords1[(n * 2) * hw + q], (float)xx);
      fy = 8.f * __fsub_rn(coords1[(n * 2 + 1) * hw + q], (float)yy);
    }
    const float wk = mk[k] / den;
    ax += wk * fx;
    ay += wk * fy;
  }
  out[((n * 2) * H8 + Y) * (long)W8 + X] = ax;
  out[((n * 2 + 1) * H8 + Y) * (long)W8 + X] = ay;
}

}  // namespace vst

using namespace vst;

static inline dim3 g256(long n) { return dim3(ceil_div(n, 256)); }

extern "C" int vst_raft_prep(const float* img, float* out, int B, int H, int W, int pad_l, int pad_r, int pad_t,
                             int pad_b, void* stream) {
  VST_REQUIRE(img && out && B > 0 && H > 0 && W > 0 && pad_l >= 0 && pad_r >= 0 && pad_t >= 0 && pad_b >= 0,
              "raft_prep: bad args");
  const int Hp = H + pad_t + pad_b, Wp = W + pad_l + pad_r;
  const long total = (long)B * Hp * Wp;
  hipLaunchKernelGGL(raft_prep_k, g256(total), dim3(256), 0, (hipStream_t)stream, img,
                     reinterpret_cast<float4*>(out), H, W, Hp, Wp, pad_l, pad_t, total);
  return check_launch("raft_prep");
}

extern "C" int vst_raft_prep_nhwc(const float* img, int src_cs, float* out, int B, int H, int W, int pad_l,
                                  int pad_r, int pad_t, int pad_b, void* stream) {
  VST_REQUIRE(img && out && src_cs >= 3 && B > 0 && H > 0 && W > 0 && pad_l >= 0 && pad_r >= 0 && pad_t >= 0 &&
                  pad_b >= 0,
              "raft_prep_nhwc: bad args");
  const int Hp = H + pad_t + pad_b, Wp = W + pad_l + pad_r;
  const long total = (long)B * Hp * Wp;
  hipLaunchKernelGGL(raft_prep_nhwc_k, g256(total), dim3(256), 0, (hipStream_t)stream, img, src_cs,
                     reinterpret_cast<float4*>(out), H, W, Hp, Wp, pad_l, pad_t, total);
  return check_launch("raft_prep_nhwc");
}

extern "C" int vst_add_relu(const float* a, const float* b, float* y, long n, void* stream) {
  VST_REQUIRE(a && b && y && n > 0 && n % 4 == 0, "add_relu: bad args");
  hipLaunchKernelGGL(add_relu_k, g256(n / 4), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const float4*>(a), reinterpret_cast<const float4*>(b),
                     reinterpret_cast<float4*>(y), n / 4);
  return check_launch("add_relu");
}

extern "C" int vst_copy_channels(const float* src, int src_cs, int src_c0, float* dst, int dst_cs, int dst_c0,
                                 int nc, long npix, void* stream) {
  VST_REQUIRE(src && dst && nc > 0 && npix > 0 && src_c0 >= 0 && dst_c0 >= 0 && src_c0 + nc <= src_cs &&
                  dst_c0 + nc <= dst_cs,
              "copy_channels: bad args");
  hipStream_t s = (hipStream_t)stream;
  if (src_cs % 4 == 0 && src_c0 % 4 == 0 && dst_cs % 4 == 0 && dst_c0 % 4 == 0 && nc % 4 == 0) {
    const long total = npix * (nc / 4);
    hipLaunchKernelGGL(copy_channels4_k, g256(total), dim3(256), 0, s, reinterpret_cast<const float4*>(src),
                       src_cs / 4, src_c0 / 4, reinterpret_cast<float4*>(dst), dst_cs / 4, dst_c0 / 4, nc / 4,
                       total);
  } else {
    const long total = npix * nc;
    hipLaunchKernelGGL(copy_channels_k, g256(total), dim3(256), 0, s, src, src_cs, src_c0, dst, dst_cs, dst_c0, nc,
                       total);
  }
  return check_launch("copy_channels");
}

extern "C" int vst_raft_ctx_split(const float* c, int cs, int hdim, int cdim, float* h, float* hx, float* rhx,
                                  int xcs, long npix, void* stream) {
  VST_REQUIRE(c && h && hx && rhx && hdim + cdim <= cs && hdim + cdim <= xcs && npix > 0, "raft_ctx_split: bad args");
  const long total = npix * (hdim + cdim);
  hipLaunchKernelGGL(raft_ctx_split_k, g256(total), dim3(256), 0, (hipStream_t)stream, c, cs, hdim, cdim, h, hx,
                     rhx, xcs, total);
  return check_launch("raft_ctx_split");
}

extern "C" int vst_raft_flow4(const float* coords1, float* flow4, int B, int h, int w, void* stream) {
  VST_REQUIRE(coords1 && flow4 && B > 0 && h > 0 && w > 0, "raft_flow4: bad args");
  const long P = (long)B * h * w;
  hipLaunchKernelGGL(raft_flow4_k, g256(P), dim3(256), 0, (hipStream_t)stream, coords1,
                     reinterpret_cast<float4*>(flow4), h, w, P);
  return check_launch("raft_flow4");
}

extern "C" int vst_raft_motion(const float* out, int ocs, int nout, const float* flow4, float* hx, float* rhx,
                               int xcs, int c0, long npix, void* stream) {
  VST_REQUIRE(out && flow4 && hx && rhx && nout <= ocs && c0 + nout + 2 <= xcs && npix > 0, "raft_motion: bad args");
  const long total = npix * (nout + 2);
  hipLaunchKernelGGL(raft_motion_k, g256(total), dim3(256), 0, (hipStream_t)stream, out, ocs, nout,
                     reinterpret_cast<const float4*>(flow4), hx, rhx, xcs, c0, total);
  return check_launch("raft_motion");
}

extern "C" int vst_gru_reset(const float* zr, const float* h, float* rhx, int hd, int xcs, long npix, void* stream) {
  VST_REQUIRE(zr && h && rhx && hd > 0 && hd <= xcs && npix > 0, "gru_reset: bad args");
  const long total = npix * hd;
  hipLaunchKernelGGL(gru_reset_k, g256(total), dim3(256), 0, (hipStream_t)stream, zr, h, rhx, hd, xcs, total);
  return check_launch("gru_reset");
}

extern "C" int vst_gru_update(const float* zr, const float* q, float* h, float* hx, int hd, int xcs, long npix,
                              void* stream) {
  VST_REQUIRE(zr && q && h && hx && hd > 0 && hd <= xcs && npix > 0, "gru_update: bad args");
  const long total = npix * hd;
  hipLaunchKernelGGL(gru_update_k, g256(total), dim3(256), 0, (hipStream_t)stream, zr, q, h, hx, hd, xcs, total);
  return check_launch("gru_update");
}

extern "C" int vst_raft_coords_update(float* coords1, const float* delta, int dcs, int B, int h, int w,
                                      void* stream) {
  VST_REQUIRE(coords1 && delta && dcs >= 2 && B > 0 && h > 0 && w > 0, "raft_coords_update: bad args");
  const long P = (long)B * h * w;
  hipLaunchKernelGGL(raft_coords_update_k, g256(P), dim3(256), 0, (hipStream_t)stream, coords1, delta, dcs,
                     (long)h * w, P);
  return check_launch("raft_coords_update");
}

extern "C" int vst_raft_upsample(const float* coords1, const float* mask, int mcs, float* out, int B, int h, int w,
                                 void* stream) {
  VST_REQUIRE(coords1 && mask && out && mcs >= 576 && B > 0 && h > 0 && w > 0, "raft_upsample: bad args");
  const long total = (long)B * 64 * h * w;
  hipLaunchKernelGGL(raft_upsample_k, g256(total), dim3(256), 0, (hipStream_t)stream, coords1, mask, mcs, out, h,
                     w, total);
  return check_launch("raft_upsample");
}
