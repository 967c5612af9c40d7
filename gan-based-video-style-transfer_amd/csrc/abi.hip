// The SURVEY §8b spelling of the C ABI: a conv descriptor (vst_conv_desc), one workspace query
// (vst_workspace_size) and the entry-point names a binder written from that contract expects
// (vst_conv2d_{fwd,dgrad,wgrad}_desc, vst_adam_multi_tensor, vst_gram, vst_corr_volume,
// vst_warp_bilinear_*, vst_masked_sqdiff_mean_*, vst_l1_mean_*, vst_mse_const_*).  Each is a host-side
// wrapper that validates the descriptor and forwards to the kernels behind the shape-argument entry
// points (conv.hip, loss.hip, flow.hip, style.hip, misc.hip); no kernel lives here.
#include "common.h"

namespace {

int desc_ok(const vst_conv_desc* d, const char* what) {
  VST_REQUIRE(d, "%s: null descriptor", what);
  VST_REQUIRE(d->N > 0 && d->H > 0 && d->W > 0 && d->C > 0 && d->K > 0 && d->R > 0 && d->S > 0 &&
                  d->stride > 0 && d->pad >= 0,
              "%s: bad shape", what);
  VST_REQUIRE(d->dilation == 1 || d->dilation == 0, "%s: dilation %d unsupported (the reference uses 1)", what,
              d->dilation);
  VST_REQUIRE(d->layout == VST_LAYOUT_NHWC, "%s: only NHWC is supported", what);
  VST_REQUIRE(d->dtype == VST_DTYPE_F32, "%s: only fp32 tensors are supported", what);
  VST_REQUIRE(d->C % 4 == 0 && d->K % 4 == 0, "%s: channel strides must be multiples of 4", what);
  VST_REQUIRE(d->pad_mode == VST_PAD_ZERO || d->pad_mode == VST_PAD_REFLECT, "%s: bad pad_mode", what);
  VST_REQUIRE(d->math >= VST_MATH_F32 && d->math <= VST_MATH_BF16X6, "%s: bad math %d", what, d->math);
  VST_REQUIRE(!d->transposed || (d->pad_mode == VST_PAD_ZERO && d->output_padding >= 0 &&
                                 d->output_padding < d->stride),
              "%s: a transposed conv takes zero padding and 0 <= output_padding < stride", what);
  return VST_OK;
}

// output spatial size of the descriptor's op (conv or transposed conv)
void out_hw(const vst_conv_desc* d, int* Ho, int* Wo) {
  if (d->transposed) {
    *Ho = (d->H - 1) * d->stride - 2 * d->pad + d->R + d->output_padding;
    *Wo = (d->W - 1) * d->stride - 2 * d->pad + d->S + d->output_padding;
  } else {
    *Ho = (d->H + 2 * d->pad - d->R) / d->stride + 1;
    *Wo = (d->W + 2 * d->pad - d->S) / d->stride + 1;
  }
}

}  // namespace

extern "C" int vst_conv_desc_out_hw(const vst_conv_desc* d, int* Ho, int* Wo) {
  if (int e = desc_ok(d, "conv_desc_out_hw")) return e;
  VST_REQUIRE(Ho && Wo, "conv_desc_out_hw: null output");
  out_hw(d, Ho, Wo);
  return VST_OK;
}

extern "C" size_t vst_workspace_size(const vst_conv_desc* d, int op) {
  if (desc_ok(d, "workspace_size") != VST_OK) return 0;
  int Ho, Wo;
  out_hw(d, &Ho, &Wo);
  switch (op) {
    case VST_OP_FWD:
      return d->transposed ? 0
                           : vst_conv2d_fwd_ws_bytes(d->N, d->H, d->W, d->C, d->K, d->R, d->S, d->stride, d->pad,
                                                     d->math);
    case VST_OP_DGRAD:
      // a conv's data gradient runs the gather-form transposed kernel (no workspace); a transposed
      // conv's data gradient is a forward conv over its output gradient
      return d->transposed ? vst_conv2d_fwd_ws_bytes(d->N, Ho, Wo, d->K, d->C, d->R, d->S, d->stride, d->pad, d->math)
                           : 0;
    case VST_OP_WGRAD:
      return d->transposed ? vst_conv2d_wgrad_ws_bytes(d->N, Ho, Wo, d->K, d->H, d->W, d->C, d->R, d->S, d->stride)
                           : vst_conv2d_wgrad_ws_bytes(d->N, d->H, d->W, d->C, Ho, Wo, d->K, d->R, d->S, d->stride);
    default:
      return 0;
  }
}

extern "C" int vst_conv2d_fwd_desc(const vst_conv_desc* d, const float* x, const float* wp, const void* wsplit,
                                   const float* bias, float* y, double* in_part, int* in_nsplit, float* ws,
                                   size_t ws_bytes, void* stream) {
  if (int e = desc_ok(d, "conv2d_fwd_desc")) return e;
  if (d->transposed) {
    int Ho, Wo;
    out_hw(d, &Ho, &Wo);
    VST_REQUIRE(!in_part, "conv2d_fwd_desc: IN partials come from a direct conv only");
    return vst_conv2d_tfwd(x, wp, bias, nullptr, y, d->N, d->H, d->W, d->C, Ho, Wo, d->K, d->R, d->S, d->stride,
                           d->pad, VST_PAD_ZERO, d->epilogue, d->slope, d->math, stream);
  }
  return vst_conv2d_fwd_ws(x, wp, wsplit, bias, y, d->N, d->H, d->W, d->C, d->K, d->R, d->S, d->stride, d->pad,
                           d->pad_mode, d->epilogue, d->slope, d->math, in_part, in_nsplit, ws, ws_bytes, stream);
}

extern "C" int vst_conv2d_dgrad_desc(const vst_conv_desc* d, const float* dy, const float* wp, const void* wsplit,
                                     float* dx, float* ws, size_t ws_bytes, void* stream) {
  if (int e = desc_ok(d, "conv2d_dgrad_desc")) return e;
  int Ho, Wo;
  out_hw(d, &Ho, &Wo);
  if (d->transposed)  // dx = conv(dy, W seen as a Conv2d weight [Ci_T][Co_T]): wp = its VST_PACK_OK pack
    return vst_conv2d_fwd_ws(dy, wp, wsplit, nullptr, dx, d->N, Ho, Wo, d->K, d->C, d->R, d->S, d->stride, d->pad,
                             VST_PAD_ZERO, VST_ACT_NONE, 0.f, d->math, nullptr, nullptr, ws, ws_bytes, stream);
  // dx = transposed gather of dy with the VST_PACK_IK pack (reflect padding folded in-kernel)
  return vst_conv2d_tfwd(dy, wp, nullptr, nullptr, dx, d->N, Ho, Wo, d->K, d->H, d->W, d->C, d->R, d->S, d->stride,
                         d->pad, d->pad_mode, VST_ACT_NONE, 0.f, d->math, stream);
}

extern "C" int vst_conv2d_wgrad_desc(const vst_conv_desc* d, const float* x, const float* dy, float* dw, int Co,
                                     int Ci, int accumulate, float* ws, size_t ws_bytes, void* stream) {
  if (int e = desc_ok(d, "conv2d_wgrad_desc")) return e;
  int Ho, Wo;
  out_hw(d, &Ho, &Wo);
  const long RS = (long)d->R * d->S;
  if (d->transposed)  // Wt[Ci_T][Co_T] is the weight gradient of x_T = conv(dy_T, .): roles swapped
    return vst_conv2d_wgrad(dy, x, dw, ws, ws_bytes, d->N, Ho, Wo, d->K, d->H, d->W, d->C, d->R, d->S, d->stride,
                            d->pad, VST_PAD_ZERO, Ci, Co, Co * RS, RS, accumulate, d->math, stream);
  return vst_conv2d_wgrad(x, dy, dw, ws, ws_bytes, d->N, d->H, d->W, d->C, Ho, Wo, d->K, d->R, d->S, d->stride,
                          d->pad, d->pad_mode, Co, Ci, Ci * RS, RS, accumulate, d->math, stream);
}

extern "C" int vst_adam_multi_tensor(float* const* p, const float* const* g, float* const* m, float* const* v,
                                     const long* n, int ntensors, float lr, float beta1, float beta2, float eps,
                                     int step, void* stream) {
  VST_REQUIRE(p && g && m && v && n && ntensors >= 0, "adam_multi_tensor: null argument");
  for (int i = 0; i < ntensors; ++i)
    if (int e = vst_adam_step(p[i], g[i], m[i], v[i], n[i], lr, beta1, beta2, eps, step, stream)) return e;
  return VST_OK;
}

extern "C" size_t vst_gram_ws_bytes(int HW, int C) {
  return vst_conv2d_wgrad_ws_bytes(1, 1, HW, C, 1, HW, C, 1, 1, 1);
}

extern "C" int vst_gram(const float* f, float* G, int B, int HW, int C, float* ws, size_t ws_bytes, int math,
                        void* stream) {
  VST_REQUIRE(f && G && B > 0 && HW > 0 && C > 0 && C % 4 == 0, "gram: bad arguments");
  for (int b = 0; b < B; ++b) {
    const float* fb = f + (long)b * HW * C;
    // the feature map seen as a 1 x HW image: G_b = F_b^T F_b is its 1x1 weight gradient with dy = x = F_b
    if (int e = vst_conv2d_wgrad(fb, fb, G + (long)b * C * C, ws, ws_bytes, 1, 1, HW, C, 1, HW, C, 1, 1, 1, 0,
                                 VST_PAD_ZERO, C, C, C, 1, 0, math, stream))
      return e;
  }
  return vst_axpby(G, G, (long)B * C * C, 1.0f / (float)HW, 0.0f, stream);
}

// level-0 plane stride of the pyramid: H*W rounded up to a multiple of 4 (raft_corr.CorrBlock's cpad)
static long corr_ld0(long HW) { return (HW + 3) / 4 * 4; }

extern "C" size_t vst_corr_volume_ws_bytes(int B, int H, int W, int Dp) {
  const long HW = (long)H * W, ld0 = corr_ld0(HW);
  (void)B;
  // fmap1 / sqrt(D) (one image), fmap2 rows padded to ld0, its three bf16 planes
  return (size_t)(HW * Dp + ld0 * Dp) * sizeof(float) + (size_t)3 * ld0 * Dp * 2;
}

extern "C" int vst_corr_volume(const float* f1, const float* f2, float* pyr, int B, int H, int W, int Dp, int D,
                               const float* sqrt_d, int levels, float* ws, size_t ws_bytes, int math, void* stream) {
  VST_REQUIRE(f1 && f2 && pyr && ws && sqrt_d && B > 0 && H > 0 && W > 0 && D > 0 && Dp >= D && Dp % 8 == 0 &&
                  levels >= 1 && (H >> (levels - 1)) >= 1 && (W >> (levels - 1)) >= 1,
              "corr_volume: bad arguments");
  VST_REQUIRE(ws_bytes >= vst_corr_volume_ws_bytes(B, H, W, Dp), "corr_volume: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const long HW = (long)H * W, ld0 = corr_ld0(HW);
  float* f1s = ws;
  float* wp = ws + HW * Dp;
  void* planes = wp + ld0 * Dp;
  if (ld0 > HW && hipMemsetAsync(wp + HW * Dp, 0, (ld0 - HW) * Dp * sizeof(float), s) != hipSuccess)
    return vst::check_launch("corr_volume memset");
  for (int b = 0; b < B; ++b) {
    // corr.py:58-59 divides the product by sqrt(D); applied to fmap1 (exact for power-of-two D)
    if (int e = vst_channel_normalize(f1 + (long)b * HW * Dp, f1s, nullptr, sqrt_d, 1.0f, HW, Dp, D, 0, stream))
      return e;
    if (hipMemcpyAsync(wp, f2 + (long)b * HW * Dp, HW * Dp * sizeof(float), hipMemcpyDeviceToDevice, s) != hipSuccess)
      return vst::check_launch("corr_volume copy");
    if (int e = vst_weight_split(wp, planes, ld0 * Dp, stream)) return e;
    // level 0 planes: a 1x1 conv whose weight rows are fmap2's pixels, ld0 output channels
    if (int e = vst_conv2d_fwd(f1s, wp, planes, nullptr, pyr + (long)b * HW * ld0, 1, H, W, Dp, (int)ld0, 1, 1, 1, 0,
                               VST_PAD_ZERO, VST_ACT_NONE, 0.f, math, stream))
      return e;
  }
  return vst_corr_pyramid(pyr, (long)B * HW, H, W, ld0, levels, stream);
}

extern "C" int vst_warp_bilinear_fwd(const float* x, const float* flow, float* out, int N, int H, int W, int Cs,
                                     int align_corners, int validity_mask, void* stream) {
  return validity_mask ? vst_warp_masked_fwd(x, flow, out, N, H, W, Cs, align_corners, stream)
                       : vst_warp_fwd(x, flow, out, N, H, W, Cs, align_corners, stream);
}

extern "C" int vst_warp_bilinear_bwd_input(const float* gout, const float* flow, float* gx, int N, int H, int W,
                                           int Cs, int align_corners, int validity_mask, void* stream) {
  return validity_mask ? vst_warp_masked_bwd_input(gout, flow, gx, N, H, W, Cs, align_corners, stream)
                       : vst_warp_bwd_input(gout, flow, gx, N, H, W, Cs, align_corners, stream);
}

extern "C" int vst_masked_sqdiff_mean_fwd(const float* a, const float* b, const float* flow, const float* mask,
                                          float* loss, float* part, int N, int H, int W, int Cs, int Cl, float lambda,
                                          void* stream) {
  return vst_loss_temporal(a, b, flow, mask, loss, part, N, H, W, Cs, Cl, lambda, stream);
}

extern "C" int vst_masked_sqdiff_mean_bwd(const float* a, const float* b, const float* flow, const float* mask,
                                          const float* gout, float* ga, float* gb, int N, int H, int W, int Cs, int Cl,
                                          float lambda, void* stream) {
  return vst_loss_temporal_bwd(a, b, flow, mask, gout, ga, gb, N, H, W, Cs, Cl, lambda, stream);
}

extern "C" int vst_l1_mean_fwd(const float* a, const float* b, float* loss, float* part, long npix, int Cs, int Cl,
                               float scale, void* stream) {
  return vst_loss_l1(a, b, loss, part, npix, Cs, Cl, scale, stream);
}

extern "C" int vst_l1_mean_bwd(const float* a, const float* b, const float* gout, float* grad, long npix, int Cs,
                               int Cl, float scale, void* stream) {
  return vst_loss_l1_bwd(a, b, gout, grad, npix, Cs, Cl, scale, stream);
}

extern "C" int vst_mse_const_fwd(const float* a, float target, float* loss, float* part, long npix, int Cs, int Cl,
                                 float scale, void* stream) {
  return vst_loss_mse_const(a, target, loss, part, npix, Cs, Cl, scale, stream);
}

extern "C" int vst_mse_const_bwd(const float* a, float target, const float* gout, float* grad, long npix, int Cs,
                                 int Cl, float scale, void* stream) {
  return vst_loss_mse_const_bwd(a, target, gout, grad, npix, Cs, Cl, scale, stream);
}
