// Shared helpers for the gfx950 kernels of libvst_hip.so (see include/vst_hip.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/vst_hip.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4v __attribute__((ext_vector_type(4)));

namespace vst {

// per-thread last error message (host side)
void set_error(const char* fmt, ...);

inline int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return VST_EHIP;
  }
  return VST_OK;
}

// Compute units of one MI355X (8 XCDs x 32 CUs): the unit of a launch's block rounds.
#define VST_NUM_CUS 256

#define VST_REQUIRE(cond, ...)            \
  do {                                    \
    if (!(cond)) {                        \
      ::vst::set_error(__VA_ARGS__);      \
      return VST_EINVAL;                  \
    }                                     \
  } while (0)

// XCD-aware tile order for a 1-D grid of T tiles.  Workgroups are dealt round-robin over the 8
// XCDs (block L runs on XCD L % 8, MI355X_MICROARCH.md), so XCD x is given the contiguous tile range
// [x*(T/8) + min(x, T%8), +T/8 + (x < T%8)): neighbouring tiles — the ones sharing operand rows —
// run on one XCD and share its L2, for any T (a bijection on [0, T)).
__device__ __forceinline__ int xcd_tile(int L, int T) {
  const int x = L & 7, k = L >> 3, q = T >> 3, r = T & 7;
  return x * q + (x < r ? x : r) + k;
}

__device__ __forceinline__ int reflect_idx(int i, int n) {
  // ReflectionPad2d index map: mirror without repeating the edge.
  i = i < 0 ? -i : i;
  return i >= n ? 2 * n - 2 - i : i;
}

// The border rows of a ReflectionPad2d(1) + 3x3 data gradient (conv_bf.hip dgrad_border_pos: per
// image NB = dgrad_border_rows rows of padded positions) that add into pixel (h, w): 0 for a pixel no
// padded position mirrors onto, 1 for the single-target rows / columns, 3 for the four corner targets
// (1 | H-2, 1 | W-2).  *b0 = the first such row.
__host__ __device__ __forceinline__ int dgrad_border_rows_of(int h, int w, int H, int W, int* b0) {
  const int sw = W - 2, sh = H - 2, S4 = ((2 * sw + 2 * sh + 3) / 4) * 4;
  const bool rh = h == 1 || h == H - 2, rw = w == 1 || w == W - 2;
  if (rh && rw) {
    *b0 = S4 + 4 * ((h == 1 ? 0 : 2) + (w == 1 ? 0 : 1));
    return 3;
  }
  const int kw = w == 0 ? 0 : (w == W - 1 ? sw - 1 : w - 1);
  const int kh = h == 0 ? 0 : (h == H - 1 ? sh - 1 : h - 1);
  if (h == 1) { *b0 = kw; return 1; }
  if (h == H - 2) { *b0 = sw + kw; return 1; }
  if (w == 1) { *b0 = 2 * sw + kh; return 1; }
  if (w == W - 2) { *b0 = 2 * sw + sh + kh; return 1; }
  return 0;
}

// The border slabs' layout (conv_bf.hip bf_dgrad_refl1_slabs): ks split-K slabs of Mb rows; Ll == 0:
// the full-K border rows, Lt = NB rows per image (dgrad_border_pos); else the K-restricted segments
// top [0, Lt), bottom [Lt, 2Lt) (image n, column k: q = (-1 | H, k-1)), left [2Lt, 2Lt+Ll), right
// [2Lt+Ll, 2Lt+2Ll) (image n, row k: q = (k, -1 | W)).
struct BorderSlabs {
  int ks, Mb, Lt, Ll;
};

// The slab rows that add into pixel (h, w) of image n, in summation order (<= 3; 0: none)
__host__ __device__ __forceinline__ int dgrad_border_slab_rows(int n, int h, int w, int H, int W, int Lt, int Ll,
                                                               int* rows) {
  if (Ll == 0) {
    int b0;
    const int nr = dgrad_border_rows_of(h, w, H, W, &b0);
    for (int r = 0; r < nr; ++r) rows[r] = n * Lt + b0 + r;
    return nr;
  }
  int nr = 0;
  if (h == 1 || h == H - 2) {
    const int base = (h == 1 ? 0 : Lt) + n * (W + 2);
    rows[nr++] = base + w + 1;                  // q = (-1 | H, w)
    if (w == 1) rows[nr++] = base;              // q = (-1 | H, -1)
    if (w == W - 2) rows[nr++] = base + W + 1;  // q = (-1 | H, W)
  }
  if (w == 1) rows[nr++] = 2 * Lt + n * H + h;           // q = (h, -1)
  if (w == W - 2) rows[nr++] = 2 * Lt + Ll + n * H + h;  // q = (h, W)
  return nr;
}

__device__ __forceinline__ float apply_act(float v, int act, float slope) {
  if (act == VST_ACT_RELU) return v > 0.f ? v : 0.f;
  if (act == VST_ACT_LRELU) return v > 0.f ? v : v * slope;
  if (act == VST_ACT_TANH) return tanhf(v);
  return v;
}

// derivative of the activation expressed through its OUTPUT y (valid for relu/lrelu/tanh)
__device__ __forceinline__ float act_grad_from_out(float y, int act, float slope) {
  if (act == VST_ACT_RELU) return y > 0.f ? 1.f : 0.f;
  if (act == VST_ACT_LRELU) return y > 0.f ? 1.f : slope;
  if (act == VST_ACT_TANH) return 1.f - y * y;
  return 1.f;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ void add_f4(float4& a, const float4& b) {
  a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
}

inline int ceil_div(long a, long b) { return (int)((a + b - 1) / b); }

// VALU kernels for convolutions with <= 4 output channels (skinny.hip)
int skinny_out_launch(int mode, const float* in, const float* wp, const float* bias,
                      const float* addend, float* out, int N, int Hi, int Wi, int Cin, int Ho,
                      int Wo, int R, int S, int st, int pad, int reflect, int act, float slope,
                      hipStream_t s, int co_real = 4);
// [row][k]-LDS implicit-GEMM fprop / transposed conv (conv_rk.hip); kind = tile override or -1
// (padh, padw: zero/reflect padding rows / columns — the forward kernels take them separately)
void rk_fprop_launch(const float* x, const float* wp, const float* bias, float* y, int N, int H, int W,
                     int C, int Ho, int Wo, int Cop, int R, int S, int st, int padh, int padw, int reflect,
                     int act, float slope, int kind, int math, hipStream_t s);
long rk_cp_ld(long P);
// split-operand bf16 implicit GEMM (conv_bf.hip); wsplit = vst_weight_split planes, stride wps
bool bf_convT_phases_ok(int C, int Cop, int math);
int bf_convT_phases_launch(const float* x, const void* const ws[4], const float* bias, float* y, int N, int H, int W,
                           int C, int Cop, int act, float slope, int math, hipStream_t s, int full = 0);
int bf_fprop_launch(const float* x, const void* wsplit, long wps, const float* bias, float* y, int N,
                    int H, int W, int C, int Ho, int Wo, int Cop, int R, int S, int st, int padh, int padw,
                    int reflect, int act, float slope, int math, int kind, hipStream_t s,
                    double* part = nullptr, float* tws = nullptr, size_t tws_floats = 0, const float* addend = nullptr,
                    int oph = 0);
// direct patch-staged 4-channel-input convs (conv_c4.hip)
// the 64 -> 4-output 7 x 7 tap conv as one direct kernel (conv_tap64.hip)
bool tap64_ok(int Cx, int R, int W, int math);
int tap64_launch(const float* x, const void* wsplit, long wps, const float* bias, float* y, int N, int H, int W,
                 int pad, int reflect, int act, float slope, int math, hipStream_t s);
bool c4_direct_ok(int C, int Cop, int R, int S, int st, int Ho, int Wo, int math);
int c4_direct_launch(const float* x, const void* wsplit, long wps, const float* bias, float* y, int N, int H, int W,
                     int Ho, int Wo, int R, int S, int pad, int reflect, int act, float slope, int math, double* part,
                     hipStream_t s);
// ReflectionPad2d(1) + 3x3 data gradient: interior GEMM + border-GEMM slabs (+ their add unless the
// caller takes them: add_border = false)
bool bf_dgrad_refl1_ok(int N, int H, int W, int Cy, int Cx, int math);
size_t bf_dgrad_refl1_ws_floats(int N, int H, int W, int Cy, int Cx, int math);
size_t bf_dgrad_refl1_slabs(int N, int H, int W, int Cy, int Cx, int math, BorderSlabs* b);
int bf_dgrad_refl1_launch(const float* dy, const void* wsplit, long wps, const float* addend, float* dx, int N, int H,
                          int W, int Cy, int Cx, int math, hipStream_t s, float* ws, size_t ws_floats, bool add_border);
// ... with the IN-backward partials of the layer below taken by the interior GEMM's epilogue and the border
// add (vst_conv2d_dgrad_refl_in_epi): part [N][bf_dgrad_refl1_inb_slices][Cx][3] fp64
bool bf_dgrad_refl1_inb_ok(int N, int H, int W, int Cy, int Cx, int math);
int bf_dgrad_refl1_inb_slices(int H, int W);
int bf_dgrad_refl1_inb_launch(const float* dy, const void* wsplit, long wps, const float* addend, float* dx, int N,
                              int H, int W, int Cy, int Cx, int math, hipStream_t s, float* ws, size_t ws_floats,
                              const float* z, const float* st, double* part, int act, float slope,
                              const __bf16* apl = nullptr, long pps = 0);
size_t bf_fprop_ws_floats(long M, int Cop, int C, int R, int S, int math);
int bf_tail_ks(long M, int Cop, int m_split, int nk);
void bf_split_plan(long M, int Cop, int C, int R, int S, int math, int kind, int* m_first, int* ks_out);
void bf_plan(long M, int Cop, int math, int kind, int* kind_out, int* m_split_out, int* tail_out);
// split-arithmetic weight gradient (conv_bf.hip): dy as pre-split bf16 planes, x as the padded fp32 copy
void bf_nhwc_to_planes(const float* x, void* y, long P, int Cs, int np, hipStream_t s, int row_in = 0,
                       int row_out = 0);
void bf_wgrad_launch(const float* xt, const void* dyp, float* slab, int N, int H, int W, int Cx, int Ho,
                     int Wo, int Cyp, int S, int pad, int st, int Mw, int chunk, int nsplit, int kind, int math,
                     hipStream_t s);
void bf_wgrad_geom(int kind, int math, int* bm, int* bn, int* bk, int* slots);
// ... over the NHWC operands (x fp32 NHWC, dy as NHWC bf16 planes [3][P][Cyp], plane stride pps): conv_wgrad_nhwc_k
bool bf_wgrad_nhwc_ok(int kind, int Wo, int Cx, int Cyp);
void bf_wgrad_nhwc_launch(const float* x, const void* dy, long pps, bool bf32, float* slab, int N, int H, int W,
                          int Cx, int Ho, int Wo, int Cyp, int S, int pad, int st, int reflect, int Mw, int chunk,
                          int nsplit, int kind, hipStream_t s, float* dwd = nullptr, int dco = 0, int dacc = 0);

void rk_tile_geom(int kind, int math, int* bm, int* bn, int* bk, int* slots);
void rk_nhwc_to_cp(const float* x, float* y, long P, int Cs, int pack, hipStream_t s);
void rk_nhwc_to_cp_pad(const float* x, float* y, int N, int H, int W, int Cs, int pad, int reflect,
                       int phase, int pack, hipStream_t s, int extra = 0);
void rk_wgrad_launch(const float* xt, const float* dyt, float* slab, int N, int H, int W, int Cx,
                     int Ho, int Wo, int Cyp, int S, int pad, int st, int Mw, int chunk,
                     int nsplit, int kind, int math, hipStream_t s);
void rk_tconv_launch(const float* in, const float* wp, const float* bias, const float* addend,
                     float* out, int N, int Hi, int Wi, int Cy, int Ho, int Wo, int Cx, int R, int S,
                     int st, int pad, int reflect, int act, float slope, int kind, int math,
                     hipStream_t s);
// g_head = false turns the head kernels below off (skinny.hip; a constant: developer A/Bs recompile)
extern const bool g_head;
// the PatchGAN head (one real output channel, stride 1, zero pad, <= 4x4 taps): patch.hip
bool head_ok(int Cin, int R, int S, int st, int reflect, int Wo);
int head_fwd_launch(const float* x, const float* wp, const float* bias, float* out, int N, int Hi, int Wi, int Cin,
                    int Ho, int Wo, int R, int S, int pad, int act, float slope, hipStream_t s);
size_t head_wgrad_ws_floats(int N, int Hi, int Cin, int R, int S);
// the forward as a per-row tap GEMM (z = N*Hi*Wi*16 floats of workspace) + a tap sum
bool head_tap_ok(int Cin);
size_t head_tap_ws_floats(int N, int Hi, int Wi);
int head_tap_fwd_launch(const float* x, const float* wp, const float* bias, float* out, float* ws, int N, int Hi,
                        int Wi, int Cin, int Ho, int Wo, int R, int S, int pad, int act, float slope, hipStream_t s);
int head_wgrad_launch(const float* x, const float* dy, float* dw, float* ws, int N, int Hi, int Wi, int Cin, int Ci,
                      int Ho, int Wo, int R, int S, int pad, long si, int accumulate, hipStream_t s,
                      float* db = nullptr);
extern const bool g_img_wgrad;
// image-input (4-channel x, <= 3 real) weight gradient with the bias gradient folded in (patch.hip)
bool img_wgrad_ok(int Cx, int Cyp, int R, int S, int st, int reflect, int Ci, int Wo);
size_t img_wgrad_ws_floats(int N, int Ho, int Wo);
int img_wgrad_launch(const float* x, const float* dy, float* dw, float* db, float* ws, int N, int H, int W, int Ho,
                     int Wo, int Cyp, int R, int S, int st, int pad, int Co, int Ci, long so, long si, int accumulate,
                     hipStream_t s);
int head_dgrad_launch(const float* dy, const float* wp, const float* addend, float* dx, int N, int Hd, int Wd, int Cx,
                      int H, int W, int R, int S, int pad, hipStream_t s);
int skinny_wgrad_launch(const float* x, const float* dy, float* slab, int H, int W, int Cx, int Ho,
                        int Wo, int S, int st, int pad, int reflect, int Mw, int P, int chunk,
                        int nsplit, hipStream_t s);

}  // namespace vst
