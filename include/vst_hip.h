/*
 * vst_hip.h — C ABI of libvst_hip.so, the MI355X (gfx950) HIP implementation of the
 * GAN-based video style transfer hot path (CycleGAN video train step + generator inference).
 *
 * Every entry point takes DEVICE pointers owned by the caller, plain int shapes, and a
 * hipStream_t passed as void* (0 = null stream).  Nothing here allocates device memory, frees
 * caller memory or synchronises the host; every call is stream-ordered and graph-capturable.
 * Returns VST_OK (0) or an error code; vst_last_error() returns a message for the calling thread.
 *
 * Tensor conventions
 *   activations   NHWC fp32, channel stride C a multiple of 4 (padding channels are zero);
 *                 image tensors are NHWC4 (3 logical channels + a zero channel).
 *   conv weights  as PyTorch stores them: Conv2d [Co][Ci][R][S], ConvTranspose2d [Ci][Co][R][S];
 *                 the kernels read a packed copy made by vst_weight_pack (cached by the caller).
 *
 * Reference interfaces replaced (paths relative to the reference root):
 *   vst_conv2d_fwd / vst_conv2d_tfwd / vst_conv2d_wgrad / vst_reflect_fold
 *       nn.Conv2d, nn.ConvTranspose2d, nn.ReflectionPad2d forward+autograd as used by
 *       methods/GAN-based/CycleGAN/models/networks.py:340-367 (ResnetGenerator), 404-426
 *       (ResnetBlock), 556-578 (NLayerDiscriminator)
 *   vst_instnorm_stats / vst_instnorm_act_fwd / vst_instnorm_act_bwd(_reduce)
 *       nn.InstanceNorm2d(affine=False) + nn.ReLU / nn.LeakyReLU(0.2), networks.py:30, 343-372, 564-576
 *   vst_warp_fwd / vst_warp_bwd_input
 *       utils/flowtools.py:18-32 warp (F.grid_sample, bilinear, zeros, align_corners=False)
 *       and methods/GAN-based/CycleGANCon/models/cycle_gan_model.py:191-203
 *   vst_fbcheck                 utils/flowtools.py:34-58 fbcCheckTorch (+ gradient 12-16)
 *   vst_loss_*                  networks.py:209-275 GANLoss('lsgan'), torch.nn.L1Loss
 *                               (cycle_gan_model.py:94-95), temporal loss cycle_gan_model.py:204
 *   vst_adam_step               torch.optim.Adam as constructed at cycle_gan_model.py:97-98
 *   vst_warp_masked_*           methods/learning-based/fs_lib.py:5-39 warp (grid_sample * validity mask)
 *   vst_instnorm_affine_*       nn.InstanceNorm2d(affine=True) (+ReLU, + ResidualBlock layer_strength
 *                               gate) of methods/learning-based/network.py:147-298 (FastStyleNet)
 *   vst_upsample2x_*            F.interpolate(scale_factor=2) in network.py:206-207
 *   vst_scaled_tanh_*           ConvTanh network.py:111-118
 *   vst_channel_normalize       fast_style_transfer.py:819-822 normalize (+ the fs_johnson.py:31 /255)
 *   vst_maxpool2_*              torchvision VGG MaxPool2d(2,2) used by network.py:10-78 (Vgg16/Vgg19)
 *   vst_loss_mse / _tv, vst_gram_sym
 *                               fs_johnson.py:35-47 content / style / TV losses and the backward of
 *                               fast_style_transfer.py:813-817 gram_matrix (Gram itself = 1x1 wgrad)
 *   vst_corr_pyramid / vst_corr_lookup
 *                               utils/raft/raft/corr.py:12-60 CorrBlock (all-pairs volume = 1x1 conv
 *                               GEMM on vst_conv2d_fwd) + utils/raft/raft/utils/utils.py:57-71
 */
#ifndef VST_HIP_H
#define VST_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { VST_OK = 0, VST_EINVAL = 1, VST_EUNSUPPORTED = 2, VST_EHIP = 3 };
enum { VST_PAD_ZERO = 0, VST_PAD_REFLECT = 1 };
enum { VST_ACT_NONE = 0, VST_ACT_RELU = 1, VST_ACT_LRELU = 2, VST_ACT_TANH = 3 };
enum { VST_PACK_KC = 0,   /* [R][S][Ci][Co]  (rows k=(r,s,ci), cols co) */
       VST_PACK_CK = 1,   /* [R][S][Co][Ci]  (rows k=(r,s,co), cols ci) */
       VST_PACK_OK = 2,   /* [Co][R][S][Ci]  conv forward B operand, k=(r,s,ci) contiguous per co */
       VST_PACK_IK = 3,   /* [Ci][R][S][Co]  dgrad / transposed-conv B operand, k=(r,s,co) per ci */
       VST_PACK_IKF = 4,  /* IK with the taps rotated 180 deg: w[co][ci][R-1-r][S-1-s] — the
                           * VST_PACK_OK pack of the conv whose forward is this conv's stride-1
                           * data gradient (dx = conv(dy, IKF, pad R-1-pad), then reflect fold) */
       VST_PACK_SOK = 5 };/* [S][Co][R][Ci]: the VST_PACK_OK pack of the R x 1 conv with S*Op outputs
                           * (s, co) — out[(s*Op + co)][r][ci] = w[co][ci][r][s] (vst_tapconv_h_fwd) */

const char* vst_last_error(void);
int vst_version(void);
/* Build configuration of the conv kernels, e.g. "x6_mfma=16x16x32 x3_mfma=32x32x16 kslice=1 x6_256=1":
 * which MFMA instruction the split-bf16 GEMMs issue (recorded with every roofline / PMC record). */
const char* vst_build_info(void);

/* ---- layout ------------------------------------------------------------------------------ */
/* NCHW (C logical channels) <-> NHWC with channel stride Cs >= C (pad channels written 0). */
int vst_nchw_to_nhwc(const float* x, float* y, int N, int C, int H, int W, int Cs, void* stream);
int vst_nhwc_to_nchw(const float* x, float* y, int N, int C, int H, int W, int Cs, void* stream);
/* Pack a PyTorch conv weight w[O][I][R][S] (ConvTranspose: pass Ci as O) for the GEMM kernels.
 * mode VST_PACK_KC -> out[R][S][Ip][Op]; VST_PACK_CK -> out[R][S][Op][Ip];
 * VST_PACK_OK -> out[Op][R][S][Ip] (consumed by vst_conv2d_fwd);
 * VST_PACK_IK -> out[Ip][R][S][Op] (consumed by vst_conv2d_tfwd);
 * VST_PACK_IKF -> out[Ip][R][S][Op] with rotated taps (consumed by vst_conv2d_fwd as a dgrad).
 * Ip/Op are the padded channel strides (multiples of 4, zero filled). */
int vst_weight_pack(const float* w, float* out, int O, int I, int R, int S, int Op, int Ip,
                    int mode, void* stream);
/* Split n fp32 values (a weight pack) into three bf16 planes out[0..n) = hi = bf16(v),
 * out[n..2n) = mid = bf16(v - hi), out[2n..3n) = lo = bf16(v - hi - mid) (2-byte elements).
 * The split-arithmetic conv paths read these planes as their B operand (`wsplit`). */
int vst_weight_split(const float* w, void* out, long n, void* stream);
/* vst_weight_pack + vst_weight_split of the pack in one pass (split: 3 * R*S*Op*Ip bf16). */
int vst_weight_pack_split(const float* w, float* out, void* split, int O, int I, int R, int S, int Op, int Ip,
                          int mode, void* stream);
/* Many packs in one launch (a network's whole pack set after each optimizer step).  `jobs` is a
 * DEVICE array of njobs 168-byte records, little-endian, natural alignment:
 *   {const float* w; float* out; void* split (3 bf16 planes or NULL);
 *    int O, I, R, S, Op, Ip, mode, pad; long total (= R*S*Op*Ip), block0 (first 256-thread block);
 *    long so, si, sr, ss; int tr[8], ts[8];}
 * sorted by block0 (job 0 at block 0, nblocks = the last job's block0 + its blocks).  Element
 * (o, i, r, s) of job j's logical weight is read at w[o*so + i*si + tr[r]*sr + ts[s]*ss] (tap maps
 * need R, S <= 8; tr[0] = -1 / ts[0] = -1 means the identity map, any R / S),
 * so a tap subset / transposed view (ConvTranspose phase packs) packs without a copy.  Replaces one
 * vst_weight_pack_split launch per pack (networks.py re-packs every layer after every Adam step). */
int vst_weight_pack_batch(const void* jobs, int njobs, long nblocks, void* stream);

/* ---- convolution (implicit GEMM on MFMA) -------------------------------------------------- */
/* `math` argument of vst_conv2d_fwd / _tfwd / _wgrad: the GEMM arithmetic of that call.
 *   VST_MATH_F32     v_mfma_f32_32x32x2_f32: exact fp32 products, fp32 accumulate (1x rate).
 *   VST_MATH_BF16X3  every fp32 operand split into bf16 hi + lo; acc += lo*hi + hi*lo + hi*hi on
 *                    v_mfma_f32_32x32x16_bf16 (fp32 accumulate, 5.3x rate): product error
 *                    <= ~2^-16 relative (finer than the TF32 convs cuDNN runs by default).
 *   VST_MATH_BF16X6  three-plane split (hi, mid, lo), six products: error <= ~2^-24 relative,
 *                    i.e. fp32-equivalent (2.7x rate).
 * The Python mirror uses BF16X6 for every forward conv (forward rounding decides ReLU masks and
 * hence which gradients exist, so it must stay at fp32 accuracy) and BF16X3 for the data and
 * weight gradients (linear in their inputs: errors stay ~1e-5 relative).  Layers routed to the
 * VALU skinny / legacy kernels (<= 4 output channels, strided weight gradients) always compute in
 * exact fp32, whatever `math` asks. */
enum { VST_MATH_F32 = 0, VST_MATH_BF16X3 = 1, VST_MATH_BF16X6 = 2 };
/* y[N][Ho][Wo][Cop] = act(conv(x[N][H][W][Cx], w) + bias).  wp = VST_PACK_OK pack
 * ([Cop][R][S][Cx]); bias has Cop entries or is NULL.  pad_mode VST_PAD_ZERO / VST_PAD_REFLECT.
 * Ho = (H + 2*pad - R)/stride + 1. */
int vst_conv2d_fwd(const float* x, const float* wp, const void* wsplit, const float* bias, float* y,
                   int N, int H, int W, int Cx, int Cop, int R, int S, int stride, int pad,
                   int pad_mode, int act, float slope, int math, void* stream);
/* Workspace of vst_conv2d_fwd_ws for this shape and arithmetic (0: the launch needs none).  Under
 * bf16x6 a grid that is not a whole number of 256x128-tile rounds runs its whole rounds as one
 * launch and the remaining pixel rows as a split-K launch (ks K ranges of the same 256x128 tiles)
 * whose partial tiles go to the workspace and are summed in split order by a reduction that applies
 * bias / act / the IN partials — instead of a launch of smaller tiles that leaves CUs idle. */
size_t vst_conv2d_fwd_ws_bytes(int N, int H, int W, int Cx, int Cop, int R, int S, int stride, int pad,
                               int math);
/* vst_conv2d_fwd (part == NULL) / vst_conv2d_fwd_in (part, nsplit) with a caller workspace ws of
 * ws_bytes >= vst_conv2d_fwd_ws_bytes (ws may be NULL when that is 0). */
int vst_conv2d_fwd_ws(const float* x, const float* wp, const void* wsplit, const float* bias, float* y, int N,
                      int H, int W, int Cx, int Cop, int R, int S, int stride, int pad, int pad_mode, int act,
                      float slope, int math, double* part, int* nsplit, float* ws, size_t ws_bytes, void* stream);
/* The data gradient of ReflectionPad2d(pad) + Conv2d(C -> 4, R x R) (the generator's last layer,
 * networks.py:365-366) without the padded frame: dx = vst_conv2d_fwd(dy, the VST_PACK_IKF pack, zero
 * padding pad) — the interior of the full correlation — then this pass adds, in a fixed order, the
 * frame positions that the reflect fold maps onto rows / columns 1..pad and H-1-pad..H-2 (fp32, from dy;
 * one writer per element).  dy NHWC4, w the fp32 IKF pack [C][R][R][4], dx NHWC C; R = 2 pad + 1,
 * C % 16 == 0.  Replaces the conv over the (H+2pad) x (W+2pad) frame + vst_reflect_fold. */
int vst_c4_dgrad_frame(const float* dy, const float* w, float* dx, int N, int H, int W, int C, int R, int pad,
                       void* stream);
/* Host-only: the split-K count (0 = none) vst_conv2d_fwd_ws uses for this shape and arithmetic: of
 * the tail launch, or — for grids of at most 128 256x128 tiles (PatchGAN layers, half batches) — of
 * the whole conv, run as one split-K launch + the reduction. */
int vst_conv_plan_fwd_tail(int N, int H, int W, int Cx, int Cop, int R, int S, int stride, int pad, int math,
                           int* ksplit);
/* vst_conv2d_fwd for a weight whose output channels co_real..Cop-1 are padding (zero weight rows,
 * zero bias): the 4-output-channel path (Cop == 4) then computes only the real ones (PatchGAN head:
 * co_real = 1); the padded channels come out as act(0), as from vst_conv2d_fwd. */
int vst_conv2d_fwd_co(const float* x, const float* wp, const void* wsplit, const float* bias, float* y, int N, int H,
                      int W, int Cx, int Cop, int R, int S, int stride, int pad, int pad_mode, int act, float slope,
                      int math, int co_real, void* stream);
/* vst_conv2d_fwd_co with a caller workspace of vst_conv2d_fwd_co_ws_bytes bytes (0: the shape takes no
 * workspace route, ws may be NULL): with co_real = 1 the PatchGAN head (networks.py:578; stride 1, zero
 * padding, R, S <= 4, Cx a power of two in 32..1024) runs as a per-input-row tap GEMM that reads x once
 * (z[n][h][w][tap] in ws) plus a fixed-order tap sum (patch.hip). */
size_t vst_conv2d_fwd_co_ws_bytes(int N, int H, int W, int Cx, int Cop, int R, int S, int stride, int pad,
                                  int pad_mode, int co_real);
int vst_conv2d_fwd_co_ws(const float* x, const float* wp, const void* wsplit, const float* bias, float* y, int N,
                         int H, int W, int Cx, int Cop, int R, int S, int stride, int pad, int pad_mode, int act,
                         float slope, int math, int co_real, float* ws, size_t ws_bytes, void* stream);
/* vst_conv2d_fwd plus the InstanceNorm statistics partials of its output, from the GEMM epilogue
 * (the conv that feeds an InstanceNorm): when the split-bf16 kernels run the conv and Ho*Wo % 32 == 0,
 * part (fp64, N * (Ho*Wo/32) * Cop * 2) receives {sum y, sum y^2} per (image, 32-pixel group,
 * channel) and *nsplit = Ho*Wo/32; otherwise *nsplit = 0 and the caller runs vst_instnorm_stats.
 * Replaces the statistics pass's full read of y (networks.py InstanceNorm after each conv). */
int vst_conv2d_fwd_in(const float* x, const float* wp, const void* wsplit, const float* bias, float* y, int N,
                      int H, int W, int Cx, int Cop, int R, int S, int stride, int pad, int pad_mode, int act,
                      float slope, int math, double* part, int* nsplit, void* stream);
/* Transposed convolution / conv data-gradient (gather form, split by output parity class):
 *   out[n][h][w][cx] = sum_{r,s,cy : h = ho*stride - pad + r, w = wo*stride - pad + s}
 *                        in[n][ho][wo][cy] * w[cy][cx][r][s]        (+ bias[cx], act)
 * in is [N][Hi][Wi][Cy]; out is [N][Ho][Wo][Cx] (Ho/Wo given: (Hi-1)*stride - 2*pad + R + output_padding).
 * wp = VST_PACK_IK pack ([Cx][R][S][Cy]): for ConvTranspose2d forward pack Wt seen as O=Ci, I=Co;
 * for the dgrad of a Conv2d pass the IK pack of its weight. */
/* pad_mode VST_PAD_REFLECT (stride 1 only) gives the data-gradient of a ReflectionPad2d(pad) +
 * valid conv directly: the mirrored contributions are gathered in-kernel (no padded buffer/fold).
 * addend (NULL or [N][Ho][Wo][Cx]) is added after bias/act (fused residual gradient). */
int vst_conv2d_tfwd(const float* in, const float* wp, const float* bias, const float* addend,
                    float* out, int N, int Hi, int Wi, int Cy, int Ho, int Wo, int Cx, int R,
                    int S, int stride, int pad, int pad_mode, int act, float slope, int math,
                    void* stream);
/* vst_conv2d_tfwd when only the first co_real of the Cy dy channels are real (the rest and their weight
 * rows zero): with co_real = 1, Cy = 4, stride 1, zero padding, R, S <= 4, no bias / activation — the
 * data gradient of the PatchGAN head Conv2d(8*ndf, 1, 4, 1, 1) (networks.py:578) — a row kernel writes
 * dx once (patch.hip); any other shape runs vst_conv2d_tfwd. */
int vst_conv2d_tfwd_co(const float* in, const float* wp, const float* bias, const float* addend, float* out, int N,
                       int Hi, int Wi, int Cy, int Ho, int Wo, int Cx, int R, int S, int stride, int pad, int pad_mode,
                       int act, float slope, int math, int co_real, void* stream);
/* Weight gradient of y = conv(x, w):  dw[co][ci][r][s] (+)= sum_pix x_gather * dy (bias gradient:
 * vst_channel_sum of dy).  x: [N][H][W][Cx], dy: [N][Ho][Wo][Cyp].  dw is written
 * with strides (so, si) for (co, ci) and r*S+s contiguous, for co < Co, ci < Ci (logical); pass
 * so = Ci*R*S, si = R*S for a Conv2d weight.  A ConvTranspose2d weight Wt[Ci][Co][R][S] is the
 * weight gradient of the equivalent conv x_T = conv(dy_T, .): call with x := grad of the convT
 * output, dy := convT input, (Co, Ci) := (Ci_T, Co_T), db := NULL (use vst_channel_sum).  accumulate != 0 adds into dw/db.  Split-K partial slabs go to
 * ws (vst_conv2d_wgrad_ws_bytes bytes) and are reduced in a fixed order (deterministic).
 * Stride 1 and 2 with W_out % 4 == 0 (stride 2: W even) stage padded channel-major copies of x and
 * dy in ws; for stride 2 that copy is sized for pad <= min(R, S) - 1 (VST_EINVAL beyond). */
size_t vst_conv2d_wgrad_ws_bytes(int N, int H, int W, int Cx, int Ho, int Wo, int Cyp, int R, int S,
                                 int stride);
int vst_conv2d_wgrad(const float* x, const float* dy, float* dw, float* ws, size_t ws_bytes, int N,
                     int H, int W, int Cx, int Ho, int Wo, int Cyp, int R, int S, int stride,
                     int pad, int pad_mode, int Co, int Ci, long so, long si, int accumulate,
                     int math, void* stream);
/* Weight AND bias gradient of y = conv(x, w) + b in one pass, for the shapes a fused route takes:
 *   - image-input layers (Cx == 4 with Ci <= 3 real channels, R*S <= 16, zero padding, Cyp <= 64 even:
 *     the PatchGAN first layer Conv2d(3, ndf, 4, 2, 1), networks.py:556) — fp32 MFMA over the fp32 dy
 *     stream, db from a constant-1 operand column;
 *   - the one-channel PatchGAN head (Cyp == 4, Co == 1, stride 1, zero pad, R, S <= 4, networks.py:578).
 * Arguments as vst_conv2d_wgrad; db[co] (+)= sum_pix dy[pix][co] for co < Co.  Any other shape returns
 * VST_EUNSUPPORTED without launching anything: use vst_conv2d_wgrad + vst_channel_sum. */
int vst_conv2d_wgrad_bias(const float* x, const float* dy, float* dw, float* db, float* ws, size_t ws_bytes, int N,
                          int H, int W, int Cx, int Ho, int Wo, int Cyp, int R, int S, int stride, int pad,
                          int pad_mode, int Co, int Ci, long so, long si, int accumulate, int math, void* stream);
/* Data gradient of ReflectionPad2d(1) + 3x3 conv, stride 1 (the ResnetBlock convs, networks.py:404-426):
 * dx[N][H][W][Cx] (+= addend, or NULL) from dy[N][H][W][Cy], wsplit = the bf16 planes of the
 * VST_PACK_IKF pack of the conv weight.  The interior term runs as the zero-pad-1 forward conv of dy
 * (addend in its epilogue); the 2(H+W)+4 positions of the padded border, whose contributions the
 * reflection folds into rows / columns 1 and H-2 / W-2, run as one small split-K GEMM whose slabs are
 * added there (no (H+2) x (W+2) frame, no fold pass).  Needs math BF16X3/X6, Cy % 32 == 0,
 * Cx % 4 == 0, H, W >= 4 (else VST_EUNSUPPORTED; ws_bytes query returns 0).  ws: ws_bytes bytes. */
size_t vst_conv2d_dgrad_refl_ws_bytes(int N, int H, int W, int Cy, int Cx, int math);
int vst_conv2d_dgrad_refl(const float* dy, const void* wsplit, const float* addend, float* dx, float* ws,
                          size_t ws_bytes, int N, int H, int W, int Cy, int Cx, int math, void* stream);
/* vst_conv2d_wgrad with operand images made by the producers of x and dy: x_t (or NULL) = the
 * padded channel-major image of x that vst_instnorm_act_fwd_cp writes (same pad / mode / stride);
 * dy_planes (or NULL) = the three bf16 planes [3][Cyp][vst_cp_ld(N*Ho*Wo)] of dy that
 * vst_instnorm_act_bwd_planes writes.  Used only when vst_conv_plan_wgrad reports VST_WPLAN_BF (the
 * x6 split-bf16 kernel); on other paths both are ignored and x / dy are read as in vst_conv2d_wgrad.
 * With x_t on that path Cx need not be a multiple of 4 (x itself is not read). */
int vst_conv2d_wgrad_pre(const float* x, const float* x_t, const float* dy, const void* dy_planes, float* dw,
                         float* ws, size_t ws_bytes, int N, int H, int W, int Cx, int Ho, int Wo, int Cyp, int R,
                         int S, int stride, int pad, int pad_mode, int Co, int Ci, long so, long si, int accumulate,
                         int math, void* stream);
/* The weight gradient over the NHWC operands the convs themselves use (round 6): x fp32 NHWC [N][H][W][Cx] (the
 * conv's input, padding applied per gathered pixel) and dy as its NHWC bf16 planes dy_apl [3][N*Ho*Wo*Cyp] (hi, mid,
 * lo: the RNE split that vst_instnorm_act_bwd_planes_apre / the epi tail's apl write), so the producing IN passes
 * need not write the padded channel-major x image or dy's channel-major planes.  The x6 256x128 plans of
 * vst_conv2d_wgrad_pre (same split plan and reduction: bit-identical results); vst_conv2d_wgrad_nhwc_ok (host-only)
 * says whether a shape takes it (bf16x6, R == S, Wo % 32 == 0, Cx, Cyp % 8 == 0, a 256x128 / 128x128 wgrad tile), ws:
 * vst_conv2d_wgrad_nhwc_ws_bytes bytes (the split-K slabs).  Other arguments as vst_conv2d_wgrad. */
int vst_conv2d_wgrad_nhwc_ok(int N, int H, int W, int Cx, int Ho, int Wo, int Cyp, int R, int S, int stride, int pad,
                             int math);
size_t vst_conv2d_wgrad_nhwc_ws_bytes(int N, int H, int W, int Cx, int Ho, int Wo, int Cyp, int R, int S, int stride,
                                      int pad, int math);
int vst_conv2d_wgrad_nhwc(const float* x, const void* dy_apl, float* dw, float* ws, size_t ws_bytes, int N, int H,
                          int W, int Cx, int Ho, int Wo, int Cyp, int R, int S, int stride, int pad, int pad_mode,
                          int Co, int Ci, long so, long si, int accumulate, int math, void* stream);
/* ... with dy fp32 NHWC [N][Ho][Wo][Cyp] itself, split in the kernel like x (the layers whose dy has no planes:
 * the stride-2 convs and the ConvTranspose weight gradients); also the 128x128 wgrad plans.  Shapes with
 * Wo % 32 != 0 over few pixels (N Ho Wo % 32 == 0, the Cx R S patches <= 64 MB: the StarGAN discriminator's small
 * layers) run as a GEMM over an im2col copy of x's patches, with one split straight into dw (replaces the
 * fp32-operand kernel + slab + transposing reduction).  vst_conv2d_wgrad_nhwc_f32_ok / _f32_ws_bytes (host-only):
 * the shapes this entry takes and its workspace.  Reference: StarGAN/model.py:65-88 (the discriminator's convs). */
int vst_conv2d_wgrad_nhwc_f32_ok(int N, int H, int W, int Cx, int Ho, int Wo, int Cyp, int R, int S, int stride,
                                 int pad, int math);
size_t vst_conv2d_wgrad_nhwc_f32_ws_bytes(int N, int H, int W, int Cx, int Ho, int Wo, int Cyp, int R, int S,
                                          int stride, int pad, int math);
int vst_conv2d_wgrad_nhwc_f32(const float* x, const float* dy, float* dw, float* ws, size_t ws_bytes, int N, int H,
                              int W, int Cx, int Ho, int Wo, int Cyp, int R, int S, int stride, int pad, int pad_mode,
                              int Co, int Ci, long so, long si, int accumulate, int math, void* stream);
/* vst_instnorm_act_fwd that also writes x_t = the padded channel-major image [C][vst_cp_ld(N (H+2 pad)
 * (W+2 pad))] of its output (reflect / zero border by pad_mode; stride 2: column-phase rows) — the
 * A operand vst_conv2d_wgrad_pre takes for the conv that consumes y (its pad, pad_mode, stride). */
int vst_instnorm_act_fwd_cp(const float* x, const float* stats, const float* residual, float* y, float* x_t,
                            int N, int H, int W, int C, int act, float slope, int pad, int pad_mode, int stride,
                            void* stream);
/* vst_instnorm_act_fwd that also writes the padded image of its output as three bf16 planes
 * [3][C][vst_cp_ld(N (H+2 pad) (W+2 pad+wx))] (the RNE hi / mid / lo split), each padded row followed
 * by wx zero columns: the B operand of vst_tap_wgrad_swap (pad = (R-1)/2, wx from
 * vst_tap_wgrad_swap_ld's geometry). */
int vst_instnorm_act_fwd_planes(const float* x, const float* stats, const float* residual, float* y, void* planes,
                                int N, int H, int W, int C, int act, float slope, int pad, int pad_mode, int wx,
                                void* stream);
/* Plane stride (elements) of the channel-major operand images over P pixels. */
long vst_cp_ld(long P);
/* Debug/benchmark only: force the GEMM tile of fprop / tconv / wgrad (-1 = automatic) for calls
 * made from the CALLING host thread (thread-local; other threads keep automatic selection).
 * fprop/tconv: 0 = 128x128 (8 waves), 1 = 64x128, 2 = 128x64, 3 = 64x64, 4 = 128x128 64-deep K,
 * (split-arithmetic fprop only) 7 = 256x128.
 * wgrad: the same kinds 0..4 on the channel-major (stride-1) path; 8 + k forces the k-major
 * legacy wgrad kernel with tile k (0..3, 4 = 256x32). */
void vst_debug_set_tiles(int fprop, int tconv, int wgrad);
/* Host-only planning query (no launch, no device needed): the kernel vst_conv2d_fwd would run for
 * this shape and `math` on this thread.  *kind = split-arithmetic tile kind (0..8, see
 * vst_debug_set_tiles; 7 = 256x128), VST_PLAN_RK (fp32 [row][k] kernel), VST_PLAN_SKINNY
 * (<= 4 output channels, VALU) or VST_PLAN_C4_DIRECT (4 input channels, 64 outputs, stride 1,
 * R == 7, S <= 8, split-bf16 math (bf16x6 / bf16x3), Wo <= 256 or a multiple of 256, and Wo a multiple
 * of 32 unless Ho*Wo is not: the patch-staged direct kernel, conv_c4.hip); *m_split = first output-pixel row of the wave-quantisation tail
 * launch, 0 when the grid runs as one launch; *tail_kind = that tail launch's tile kind (-1: none). */
enum { VST_PLAN_RK = -1, VST_PLAN_SKINNY = -2, VST_PLAN_C4_DIRECT = -3 };
int vst_conv_plan_fwd(int N, int H, int W, int Cx, int Cop, int R, int S, int stride, int pad_h,
                      int pad_w, int math, int* kind, int* m_split, int* tail_kind);
/* Host-only planning query for vst_conv2d_wgrad: *path = VST_WPLAN_BF (channel-major copies + the
 * split-bf16 kernel conv_wgrad_bf_k), _RK (copies + conv_wgrad_rk_k), _GENERIC (conv_wgrad_k on the
 * NHWC operands) or _SKINNY (<= 4 output channels, VALU); *kind = its tile kind; *nsplit = split-K
 * slabs (reduced by slab_group_sum_k + wgrad_reduce_store_k). */
enum { VST_WPLAN_GENERIC = 0, VST_WPLAN_RK = 1, VST_WPLAN_BF = 2, VST_WPLAN_SKINNY = 3, VST_WPLAN_BF_PADW = 4 };
int vst_conv_plan_wgrad(int N, int H, int W, int Cx, int Ho, int Wo, int Cyp, int R, int S, int stride,
                        int math, int* path, int* kind, int* nsplit);
/* db[c] (+)= sum over NHW pixels of x[p][c] for c < Cl (channel stride Cs); bias gradient of a layer
 * whose output gradient is x.  ws: vst_channel_sum_ws_bytes bytes; fixed-order (deterministic). */
size_t vst_channel_sum_ws_bytes(long NHW, int Cs);
int vst_channel_sum(const float* x, float* db, float* ws, long NHW, int Cs, int Cl, int accumulate,
                    void* stream);
/* Fold the gradient of a ReflectionPad2d(p): dx[n][h][w][c] = sum of dxp over padded positions
 * mapping to (h,w) (+ addend if non-NULL).  dxp: [N][H+2p][W+2p][C], dx/addend: [N][H][W][C]. */
int vst_reflect_fold(const float* dxp, const float* addend, float* dx, int N, int H, int W, int C,
                     int p, void* stream);

/* ---- instance norm + activation ---------------------------------------------------------- */
/* stats[n*C + c] = {mean, rstd} (2 floats interleaved: mean at 2*(n*C+c), rstd at +1), biased
 * variance, eps.  ws: vst_instnorm_ws_bytes(N, HW, C) bytes. */
size_t vst_instnorm_ws_bytes(int N, int HW, int C);
int vst_instnorm_stats(const float* x, float* stats, float* ws, int N, int HW, int C, float eps,
                       void* stream);
/* stats[n][c] = {mean, 1/sqrt(var + eps)} from fp64 partials part[n][z][c][2] = {sum, sum of squares}
 * over z < nsplit groups (vst_conv2d_fwd_in's epilogue partials); fixed-order fold. */
int vst_instnorm_finalize(const double* part, float* stats, int N, int HW, int C, int nsplit, float eps,
                          void* stream);
/* y = act((x - mean) * rstd) (+ residual).  residual may be NULL. */
int vst_instnorm_act_fwd(const float* x, const float* stats, const float* residual, float* y,
                         int N, int HW, int C, int act, float slope, void* stream);
/* Backward of y = act(IN(x)):  dx = rstd * (g - mean(g) - xhat * mean(g*xhat)),
 * g = gy * act'(xhat).  db (NULL or C floats) receives (accumulate_db: adds) sum_{n,p} dx — the
 * gradient of a conv bias feeding this IN — from the same fp64 reduction (no extra pass).
 * ws: vst_instnorm_ws_bytes bytes.  C must be 4*2^k <= 1024. */
int vst_instnorm_act_bwd(const float* gy, const float* x, const float* stats, float* dx, float* db,
                         float* ws, int N, int HW, int C, int act, float slope, int accumulate_db,
                         void* stream);
/* vst_conv2d_dgrad_refl fused with the InstanceNorm(+act) backward of the layer below it (the ResnetBlock data
 * gradients, networks.py:404-426, each followed by the IN backward of the block's previous layer): gout = the data
 * gradient (+ addend), x / stats = that IN's input and statistics, dx = its input gradient (db, planes as
 * vst_instnorm_act_bwd_planes).  The IN backward partials are taken by the data gradient itself: the interior
 * GEMM's epilogue sums {g', g' xhat, xhat} per 32-pixel group of its output tile and the border add adds the
 * correction of the pixels it changes, so no separate partial pass (a read of gout and x and a launch) runs.
 * gout is bit-identical to vst_conv2d_dgrad_refl; dx / planes / db to the separate passes up to the fp64
 * summation order of the partials.  x6 arithmetic only, H*W % 32 == 0 (ws_bytes query 0 = unsupported). */
size_t vst_conv2d_dgrad_refl_in_epi_ws_bytes(int N, int H, int W, int Cy, int Cx, int math);
int vst_conv2d_dgrad_refl_in_epi(const float* dy, const void* wsplit, const float* addend, float* gout,
                                 const float* x, const float* stats, float* dx, float* db, float* ws, size_t ws_bytes,
                                 int N, int H, int W, int Cy, int Cx, int act, float slope, int accumulate_db,
                                 void* planes, long ldp, int math, void* stream);
/* its halves: the data gradient + the partials (into the front of ws), then finalize + apply from them */
int vst_conv2d_dgrad_refl_epi_part(const float* dy, const void* dy_apl, const void* wsplit, const float* addend,
                                   float* gout, const float* x, const float* stats, float* ws, size_t ws_bytes, int N,
                                   int H, int W, int Cy, int Cx, int act, float slope, int math, void* stream);
int vst_instnorm_act_bwd_epi_tail(const float* gout, const float* x, const float* stats, float* dx, float* db,
                                  float* ws, int N, int H, int W, int Cx, int act, float slope, int accumulate_db,
                                  void* planes, long ldp, void* apl, void* stream);
/* (dy_apl: dy's NHWC bf16 planes [3][N*H*W*Cy] or NULL — the interior GEMM then takes its A operand pre-split by
 * LDS-DMA, the border GEMM from the planes too, and dy's fp32 image is not read; apl: the tail writes dx as its
 * NHWC planes INSTEAD of fp32 (the next data gradient's dy_apl; dx is left unwritten), or NULL) */
/* vst_instnorm_act_bwd_planes whose dx is written ONLY as its NHWC bf16 planes apl [3][N*HW*C] (hi, mid, lo: each
 * value's RNE split) — the pre-split A operand of the ResnetBlock data gradient that consumes it (dy_apl above). */
int vst_instnorm_act_bwd_planes_apre(const float* gy, const float* x, const float* stats, float* dx, float* db,
                                     float* ws, int N, int HW, int C, int act, float slope, int accumulate_db,
                                     void* planes, long ldp, void* apl, void* stream);
/* vst_instnorm_act_bwd whose apply pass also writes dx as the three bf16 planes [3][C][ldp] (hi, mid,
 * lo; ldp >= N*HW, vst_cp_ld(N*HW)) the x6 weight gradient of the conv below consumes
 * (vst_conv2d_wgrad_pre).  planes == NULL: identical to vst_instnorm_act_bwd. */
int vst_instnorm_act_bwd_planes(const float* gy, const float* x, const float* stats, float* dx, float* db,
                                float* ws, int N, int HW, int C, int act, float slope, int accumulate_db,
                                void* planes, long ldp, void* stream);
/* Elementwise activation backward in place-safe form: dx = gy * act'(y) given the OUTPUT y. */
int vst_act_bwd(const float* gy, const float* y, float* dx, long n, int act, float slope, void* stream);

/* ---- flow warp, consistency mask, losses --------------------------------------------------- */
/* out[n][h][w][c] = bilinear sample of x at (w + flow_x, h + flow_y) with the reference's
 * normalisation (grid/max(W-1,1)) and align_corners flag; zeros padding.  x, out: NHWC (C stride Cs);
 * flow: [N][2][H][W] (NCHW, as the reference stores it). */
int vst_warp_fwd(const float* x, const float* flow, float* out, int N, int H, int W, int Cs,
                 int align_corners, void* stream);
/* gx[...] += bilinear-transpose scatter of gout (gx must be zero-initialised by the caller). */
int vst_warp_bwd_input(const float* gout, const float* flow, float* gx, int N, int H, int W, int Cs,
                       int align_corners, void* stream);
/* Deterministic (atomic-free) warp input gradient — the debug switch of SURVEY §7 item 4, replacing
 * the atomic scatter of vst_warp_bwd_input / vst_warp_masked_bwd_input (masked = 1: fs_lib.warp's
 * validity mask) / vst_loss_temporal_bwd's ga (negate = 1, gout = that call's gb): gx[t][c] (c < Cl) +=
 * sum over the output pixels p and corners k (nw, ne, sw, se) landing on t, in ascending (p, k) order,
 * of (+-) w_k(p) * gout[p][c] — one fp32 rounding per add, identical from run to run.  ws: caller-owned,
 * vst_warp_bwd_det_ws_bytes(N, H, W) bytes.  Reference: utils/flowtools.py:18-32 (F.grid_sample). */
size_t vst_warp_bwd_det_ws_bytes(int N, int H, int W);
int vst_warp_bwd_input_det(const float* gout, const float* flow, float* gx, void* ws, size_t ws_bytes, int N,
                           int H, int W, int Cs, int Cl, int align_corners, int masked, int negate, void* stream);
/* mask[n][0][h][w] in {0,1} from forward/backward flows ff, bf ([N][2][H][W]). */
int vst_fbcheck(const float* ff, const float* bf, float* mask, int N, int H, int W, void* stream);

/* Losses.  Forward writes the scalar loss to loss[0] (device) using a per-block partial buffer
 * `part` of vst_loss_part_floats(npix) floats and a fixed-order final sum (deterministic).
 * Backward reads the upstream scalar gradient from device memory gout[0] (no host sync) and
 * WRITES the full gradient tensor (padding channels zero), except where noted.
 * Means run over npix * Cl elements (Cl logical channels of a channel stride Cs). */
int vst_loss_part_floats(long npix);
/* temporal (CycleGANCon cycle_gan_model.py:191-204):
 *   loss = lambda * mean((mask * (b - warp(a, flow)))^2),  a, b: NHWC, flow [N][2][H][W], mask [N][H][W].
 * bwd: gb written; ga ACCUMULATED (scatter through the warp) — either may be NULL. */
int vst_loss_temporal(const float* a, const float* b, const float* flow, const float* mask,
                      float* loss, float* part, int N, int H, int W, int Cs, int Cl, float lambda,
                      void* stream);
int vst_loss_temporal_bwd(const float* a, const float* b, const float* flow, const float* mask,
                          const float* gout, float* ga, float* gb, int N, int H, int W, int Cs,
                          int Cl, float lambda, void* stream);
/* L1: loss = scale * mean|a - b|; grad = gout*scale*sign(a-b)/count (sign(0)=0, as torch). */
int vst_loss_l1(const float* a, const float* b, float* loss, float* part, long npix, int Cs, int Cl,
                float scale, void* stream);
int vst_loss_l1_bwd(const float* a, const float* b, const float* gout, float* grad, long npix,
                    int Cs, int Cl, float scale, void* stream);
/* LSGAN: loss = scale * mean((a - target)^2); grad = gout*scale*2*(a-target)/count. */
int vst_loss_mse_const(const float* a, float target, float* loss, float* part, long npix, int Cs,
                       int Cl, float scale, void* stream);
int vst_loss_mse_const_bwd(const float* a, float target, const float* gout, float* grad, long npix,
                           int Cs, int Cl, float scale, void* stream);
/* out[0] = scale * sum(part[0..n)) in a fixed order. */
int vst_finish_sum(const float* part, int n, float* out, double scale, void* stream);

/* ---- optimizer ------------------------------------------------------------------------------ */
/* torch.optim.Adam (no weight decay, no amsgrad) over a flat parameter buffer:
 *   m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2;
 *   p -= lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps)                                    */
int vst_adam_step(float* p, const float* g, float* m, float* v, long n, float lr, float beta1,
                  float beta2, float eps, int step, void* stream);
/* y = a*x + b*y over n floats (gradient scaling / DP averaging helper). */
int vst_axpby(const float* x, float* y, long n, float a, float b, void* stream);

/* ---- learning-based style path -------------------------------------- */
/* fs_lib.warp: warp(x, flow) * (grid_sample(ones) >= 0.9999).  Same layouts as vst_warp_fwd; the
 * backward scatters only through kept samples (gx accumulated, must be zero-initialised). */
int vst_warp_masked_fwd(const float* x, const float* flow, float* out, int N, int H, int W, int Cs,
                        int align_corners, void* stream);
int vst_warp_masked_bwd_input(const float* gout, const float* flow, float* gx, int N, int H, int W,
                              int Cs, int align_corners, void* stream);
/* Affine instance norm: y = s * act(gamma[c] * xhat + beta[c]) + residual, with stats from
 * vst_instnorm_stats; s = 1 (gate NULL) or s = 2|u|/(1+|u|), u = gate_mult * gate[0] (device scalar:
 * ResidualBlock layer_strength, network.py:241-245).  residual may be NULL.  C = 4*2^k <= 1024. */
int vst_instnorm_affine_fwd(const float* x, const float* stats, const float* gamma, const float* beta,
                            const float* gate, float gate_mult, const float* residual, float* y,
                            int N, int HW, int C, int act, float slope, void* stream);
/* Backward: dx written; dgamma/dbeta/dgate/dbias (each may be NULL) written or accumulated
 * (accumulate != 0).  dbias is the gradient of a conv bias feeding the norm (exact per-channel sum
 * of dx).  ws: vst_instnorm_affine_ws_bytes bytes.  Reductions fp64, fixed order. */
size_t vst_instnorm_affine_ws_bytes(int N, int HW, int C);
int vst_instnorm_affine_bwd(const float* gy, const float* x, const float* stats, const float* gamma,
                            const float* beta, const float* gate, float gate_mult, float* dx,
                            float* dgamma, float* dbeta, float* dgate, float* dbias, float* ws, int N,
                            int HW, int C, int act, float slope, int accumulate, void* stream);
/* Nearest 2x upsample of NHWC (Cs % 4 == 0): y [N][2H][2W][Cs]; backward sums each 2x2 block. */
int vst_upsample2x_fwd(const float* x, float* y, int N, int H, int W, int Cs, void* stream);
int vst_upsample2x_bwd(const float* gy, float* gx, int N, int H, int W, int Cs, void* stream);
/* ConvTanh: y = tanh(x/255)*150 + 127.5 on the Cl logical channels (padding channels 0);
 * backward from the saved pre-activation x. */
int vst_scaled_tanh_fwd(const float* x, float* y, long npix, int Cs, int Cl, void* stream);
int vst_scaled_tanh_bwd(const float* x, const float* gy, float* gx, long npix, int Cs, int Cl,
                        void* stream);
/* y = ((x / d0) - mean[c]) / std[c] (mean may be NULL = 0); backward != 0: y = (x / std[c]) / d0.
 * mean/std: device arrays of Cl floats.  Padding channels written 0. */
int vst_channel_normalize(const float* x, float* y, const float* mean, const float* stdv, float d0,
                          long npix, int Cs, int Cl, int backward, void* stream);
/* MaxPool2d(2, 2) (floor mode) on NHWC; backward writes every gx element (first max wins ties). */
int vst_maxpool2_fwd(const float* x, float* y, int N, int H, int W, int Cs, void* stream);
int vst_maxpool2_bwd(const float* gy, const float* x, float* gx, int N, int H, int W, int Cs,
                     void* stream);
/* loss (+)= scale * mean((a - b)^2) over npix*Cl elements; grad (+)= gout*scale*2(a-b)/count. */
int vst_loss_mse(const float* a, const float* b, float* loss, float* part, long npix, int Cs, int Cl,
                 float scale, int accumulate, void* stream);
int vst_loss_mse_bwd(const float* a, const float* b, const float* gout, float* grad, long npix,
                     int Cs, int Cl, float scale, int accumulate, void* stream);
/* calc_tv_loss: loss (+)= scale * sum_{n,y<H-1,x<W-1} sqrt(|I[y+1][x]-I[y][x]|^2 + |I[y][x+1]-I[y][x]|^2)
 * (norms over the Cl <= 4 logical channels); backward writes grad (zero-length terms give 0). */
int vst_loss_tv(const float* img, float* loss, float* part, int N, int H, int W, int Cs, int Cl,
                float scale, int accumulate, void* stream);
int vst_loss_tv_bwd(const float* img, const float* gout, float* grad, int N, int H, int W, int Cs,
                    int Cl, float scale, void* stream);
/* Gram backward weight: S = (dG + dG^T) * scale, [C][C] — dF = F * S is then a 1x1 vst_conv2d_fwd.
 * (The Gram itself, G = F^T F, is vst_conv2d_wgrad of a 1x1 conv with x = dy = F.) */
int vst_gram_sym(const float* dG, float* S, int C, float scale, void* stream);

/* ---- RAFT correlation pyramid ---------------------------------------------- */
/* Level 0 (P = B*H1*W1 planes of H2*W2, plane stride ld0) is the all-pairs GEMM output
 * fmap1^T fmap2 / sqrt(D) produced by vst_conv2d_fwd (1x1 conv, fmap2 as the weight).  Levels
 * 1..levels-1 (avg_pool2d 2x2, floor) follow it packed in the same buffer. */
long vst_corr_pyramid_floats(long P, int H2, int W2, long ld0, int levels);
int vst_corr_pyramid(float* pyr, long P, int H2, int W2, long ld0, int levels, void* stream);
/* out[b][h][w][c] (NHWC, Cs >= levels*(2r+1)^2, extra channels 0): CorrBlock.__call__ window
 * lookup at coords [B][2][H1][W1] (x, y pixel coordinates); channel lvl*(2r+1)^2 + a*(2r+1) + c
 * samples x + (a - r), y + (c - r) at level lvl (align_corners=True bilinear, zeros outside). */
int vst_corr_lookup(const float* pyr, const float* coords, float* out, int B, int H1, int W1, int H2,
                    int W2, long ld0, int levels, int radius, int Cs, void* stream);

/* ---- StarGAN -------------------------------------------------------------- */
/* methods/GAN-based/StarGAN/model.py:59-64: y = NHWC(cat([x, label replicated], 1)), x NCHW
 * [N][Cx][H][W], label [N][Cl], y [N][H][W][Cs] (Cs >= Cx + Cl, extra channels 0). */
int vst_concat_label_nhwc(const float* x, const float* label, float* y, int N, int Cx, int Cl, int H,
                          int W, int Cs, void* stream);
/* nn.InstanceNorm2d(track_running_stats=True) buffers (model.py:13-16): training-mode update from
 * this batch's stats (mean of the per-instance updates, unbiased variance), and the eval-mode
 * stats tensor built from the running buffers. */
int vst_instnorm_running_update(const float* stats, float* running_mean, float* running_var, int N,
                                int C, int HW, float momentum, float eps, void* stream);
int vst_instnorm_stats_from_running(const float* running_mean, const float* running_var,
                                    float* stats, int N, int C, float eps, void* stream);

/* ---- tap-GEMM convolutions with 4 (padded) output channels (generators' last layer) -------- */
/* Z = vst_conv2d_fwd(x, VST_PACK_CK pack of w seen as a 1x1 conv with R*S*4 outputs) holds
 * sum_ci x[q][ci] w[co][ci][r][s] for every source pixel q and tap; vst_tapsum_fwd gathers
 * y[p][co] = act(bias[co] + sum_{r,s} Z[src(p,r,s)][(r*S+s)*4 + co]) for 'same' convolutions
 * (2*pad == R-1 == S-1, zero or reflect padding; y NHWC4).  Replaces the direct conv of
 * networks.py:365-367 (c7s1-3) on the matrix cores. */
int vst_tapsum_fwd(const float* z, int zcs, const float* bias, float* y, int N, int H, int W, int R, int S,
                   int pad, int pad_mode, int act, float slope, void* stream);
/* The same conv with the contraction over (r, ci) on the matrix cores and only the column taps
 * summed afterwards: z[q][(s*4 + co)] = sum_{r,ci} x[src_row(q, r)][ci] w[co][ci][r][s] is the R x 1
 * conv (row padding `pad`, pad_mode) of x with the VST_PACK_SOK pack (+ wsplit planes; 4*S outputs),
 * then y[p][co] = act(bias[co] + sum_s z[(h, src(w + s - pad))][s*4 + co]).  Output Ho x Wo =
 * (H + 2 pad - R + 1) x (W + 2 pad - R + 1); z = caller's buffer of N*Ho*W*4*R floats.  Replaces
 * vst_conv2d_fwd(1x1, R*S*4 outputs) + vst_tapsum_fwd: z is S*16 bytes per pixel instead of R*S*16,
 * and the GEMM's K is R*Cx instead of Cx.  R == S in {3, 5, 7}, Cx % 8 == 0; reflect: 'same' convs
 * (2 pad == R-1); zero: any pad < R (pad R-1 with the rotated-tap pack = the full correlation of a
 * data gradient, whose reflect fold gives the image-input layer's dx: ops.tap_conv_dgrad_h). */
int vst_tapconv_h_fwd(const float* x, const float* wp, const void* wsplit, const float* bias, float* z, float* y,
                      int N, int H, int W, int Cx, int R, int pad, int pad_mode, int act, float slope, int math,
                      void* stream);
/* The weight gradient of the same reflect 'same' conv as the R x 1 conv's: with padding pad+1 (reflect;
 * the extra ring multiplies zero dy) its output frame is (H+2) x (W+S+1), and its dy channel (s, co)
 * at (ho, wo) is g[ho-1][wo-1-s][co] — vst_tapshift_planes writes that as the x6 wgrad's bf16 planes
 * [3][S*4][ldp] (ldp >= N (H+2) (W+S+1)); vst_conv2d_wgrad_pre(x, x_t padded by pad+1, planes,
 * Cyp = 4S, R, S = 1, pad + 1, reflect, Co = 4S, so = Ci*R, si = R) gives t[(s*4+co)][ci][r], and
 * vst_tap_wgrad_scatter_h writes dw[co][ci][r][s] (+)= t.  No R*S-fold of g: 4S channels instead of
 * 4RS. */
int vst_tapshift_planes(const float* g, void* planes, long ldp, int N, int H, int W, int S, void* stream);
int vst_tap_wgrad_scatter_h(const float* t, float* dw, int Co, int Ci, int R, int S, int accumulate, void* stream);
/* The same weight gradient with the GEMM's roles swapped (replaces the R x 1 form in the train step):
 * dw[co][ci][r][s] = sum_q xf[q][ci] * dyP[q + (R-1-r, R-1-s)][co] over the (H+R-1) x (W+R-1+wx) frame q
 * of x reflect-padded by (R-1)/2 (x_planes: its bf16 planes as vst_instnorm_act_fwd_planes writes them,
 * wx = (8 - (W+R-1) % 8) % 8 zero columns) and dy zero-padded by R-1 (made here in ws).  M = R*R*3
 * (tap, co) rows (R*R*4 when Co == 4) instead of the R x 1 form's 4R (column tap, co) x R*Ci (the
 * 3-channel x image: vst_conv2d_wgrad_pre takes any Cx with a caller-made x_t): no tap-shifted dy planes,
 * and the x operand is read once per 64 rows of (tap, co) instead of once per row tap.  Then
 * dw (+)= the result with its taps rotated 180 degrees.  ws: vst_tap_wgrad_swap_ws_bytes. */
int vst_tap_wgrad_swap(const float* g, const void* x_planes, float* dw, float* ws, size_t ws_bytes, int N, int H,
                       int W, int Ci, int R, int Co, int accumulate, int math, void* stream);
/* vst_tap_wgrad_swap plus the conv's bias gradient db[c] (+)= sum_pix g[pix][c] (c < Co; db may be NULL):
 * block sums taken by the pass that stages g for the GEMM, folded in a fixed order (fp64) by the last
 * block of the tap scatter — no separate channel-sum launches (networks.py:365-366's bias). */
int vst_tap_wgrad_swap_db(const float* g, const void* x_planes, float* dw, float* db, float* ws, size_t ws_bytes, int N,
                          int H, int W, int Ci, int R, int Co, int accumulate, int math, void* stream);
size_t vst_tap_wgrad_swap_ws_bytes(int N, int H, int W, int Ci, int R);
/* Plane stride of x_planes: vst_cp_ld(N (H+R-1) (W+R-1+wx)). */
long vst_tap_wgrad_swap_ld(int N, int H, int W, int R);
/* Adjoint gather of the weight gradient: d[q][(r*S+s)*4 + co] = sum_{p: src(p,r,s) = q} g[p][co]
 * (g NHWC4); then vst_conv2d_wgrad(x, d) as a 1x1 wgrad gives t[(r*S+s)*4 + co][ci], and
 * vst_tap_wgrad_scatter writes dw[co][ci][r][s] (+)= t (co < Co <= 4). */
int vst_tapfold(const float* g, float* d, int N, int H, int W, int R, int S, int pad, int pad_mode, void* stream);
/* vst_tapfold writing D as the three bf16 planes [3][R*S*4][ldp] (ldp >= N*H*W, vst_cp_ld) the x6
 * weight gradient takes as its dy image (vst_conv2d_wgrad_pre): no fp32 D, no plane copy. */
int vst_tapfold_planes(const float* g, void* planes, long ldp, int N, int H, int W, int R, int S, int pad,
                       int pad_mode, void* stream);
int vst_tap_wgrad_scatter(const float* t, float* dw, int Co, int Ci, int R, int S, int accumulate, void* stream);
/* Data gradient of a 'same' conv with <= 4 INPUT channels (the generators' first layer, c7s1-64 on
 * the image): z = vst_conv2d_fwd(dy, VST_PACK_KC pack seen as a 1x1 conv with R*S*4 outputs), then
 * y[q][ci] = sum_{r,s} sum_{p: src(p,r,s) = q} z[p][(r*S+s)*4 + ci]  (y NHWC4). */
int vst_tapgather(const float* z, float* y, int N, int H, int W, int R, int S, int pad, int pad_mode,
                  void* stream);

/* ConvTranspose2d(k=3, stride 2, padding 1, output_padding 1) forward (CycleGAN networks.py:357-364)
 * as four sub-pixel phase convolutions on the forward kernels: P_00 = 1x1 conv, P_01 = 1x2 conv
 * (pad 0,1), P_10 = 2x1 (pad 1,0), P_11 = 2x2 (pad 1,1) with the phase's taps of the transposed
 * weight; this interleaves them: y[n][2i+a][2j+b][c] = P_ab[n][i+a][j+b][c] (P_ab is (H+a) x (W+b)). */
int vst_interleave_phases(const float* p00, const float* p01, const float* p10, const float* p11, float* y, int N,
                          int H, int W, int C, void* stream);
/* The same interleave for the data gradient of Conv2d(k=4, stride 2, padding 1) (PatchGAN
 * networks.py:556-578): per output parity two taps per dim (even: w3 at dy[i-1], w1 at dy[i]; odd: w2 at dy[i], w0 at dy[i+1]), i.e. four 2x2 phase convs
 * with padding 1 whose outputs are all (H+1) x (W+1): y[n][2i+a][2j+b][c] = P_ab[n][i+a][j+b][c]. */
int vst_interleave_phases_full(const float* p00, const float* p01, const float* p10, const float* p11, float* y,
                               int N, int H, int W, int C, void* stream);
/* One phase (a, b) in {0,1}^2 of a stride-2 ConvTranspose2d(k3, p1, op1) stored straight into the
 * interleaved output y [N][2H][2W][Cop]: the phase conv vst_conv2d_fwd_hw(x, phase pack, R = 1 + a,
 * S = 1 + b, pad a / b) whose pixel (ph, pw) is y's (2(ph-a)+a, 2(pw-b)+b).  Four calls write every
 * pixel of y once, replacing four phase images + vst_interleave_phases.  wsplit = the phase pack's bf16
 * planes; Cx % 8 == 0; split-bf16 math only (VST_EUNSUPPORTED for VST_MATH_F32). */
int vst_conv2d_fwd_phase(const float* x, const void* wsplit, const float* bias, float* y, int N, int H, int W,
                         int Cx, int Cop, int a, int b, int act, float slope, int math, void* stream);
/* All four phases of that ConvTranspose2d forward in ONE launch (the four vst_conv2d_fwd_phase calls'
 * tiles concatenated, the 2x2 phase first), same output bit for bit.  ws_ab = phase (a, b)'s pack
 * planes.  Cx % 32 == 0, Cop % 4 == 0, split-bf16 math (else VST_EUNSUPPORTED: use the per-phase
 * calls).  Replaces CycleGAN networks.py:357-364's ConvTranspose2d forward. */
int vst_conv2d_convT_s2(const float* x, const void* ws00, const void* ws01, const void* ws10, const void* ws11,
                        const float* bias, float* y, int N, int H, int W, int Cx, int Cop, int act, float slope,
                        int math, void* stream);
/* Data gradient of Conv2d(k4, s2, p1) (PatchGAN networks.py:556-578) in ONE launch: the four 2x2 pad-1
 * phase convs of dy [N][Hd][Wd][Cy] (ws_ab = the bf16 planes of conv4s2 phase pack (a, b)) stored straight
 * into dx [N][2Hd][2Wd][Cop] (dx[2i+a][2j+b] = P_ab[i+a][j+b]); replaces four phase images +
 * vst_interleave_phases_full.  Cy % 32 == 0, Cop % 4 == 0, split-bf16 math (else VST_EUNSUPPORTED). */
int vst_conv4s2_dgrad(const float* dy, const void* ws00, const void* ws01, const void* ws10, const void* ws11,
                      float* dx, int N, int Hd, int Wd, int Cy, int Cop, int math, void* stream);

/* ---- RAFT inference (SURVEY §8 A19 + §8f rank 3) ------------------------------------------ */
/* Forward conv with separate row / column zero padding (SepConvGRU's (1,5) / (5,1) kernels with
 * padding (0,2) / (2,0), update.py:36-43); otherwise identical to vst_conv2d_fwd. */
int vst_conv2d_fwd_hw(const float* x, const float* wp, const void* wsplit, const float* bias, float* y,
                      int N, int H, int W, int Cx, int Cop, int R, int S, int stride, int pad_h, int pad_w,
                      int act, float slope, int math, void* stream);
/* vst_conv2d_fwd_hw with a caller-owned workspace: the split-K plans of vst_conv2d_fwd_ws for grids smaller than
 * the CUs (ws_bytes >= vst_conv2d_fwd_hw_ws_bytes; ws may be NULL when that is 0). */
size_t vst_conv2d_fwd_hw_ws_bytes(int N, int H, int W, int Cx, int Cop, int R, int S, int stride, int pad_h,
                                  int pad_w, int math);
int vst_conv2d_fwd_hw_ws(const float* x, const float* wp, const void* wsplit, const float* bias, float* y, int N,
                         int H, int W, int Cx, int Cop, int R, int S, int stride, int pad_h, int pad_w, int act,
                         float slope, int math, float* ws, size_t ws_bytes, void* stream);
/* vst_conv2d_fwd_hw with a padding mode (VST_PAD_ZERO / VST_PAD_REFLECT). */
int vst_conv2d_fwd_hwp(const float* x, const float* wp, const void* wsplit, const float* bias, float* y, int N, int H,
                       int W, int Cx, int Cop, int R, int S, int stride, int pad_h, int pad_w, int pad_mode, int act,
                       float slope, int math, void* stream);
/* InputPadder.pad (utils/raft/raft/utils/utils.py:7-20, replicate) + raft.py:89-90 2*(x/255)-1:
 * NCHW [B][3][H][W] -> NHWC4 [B][H+pt+pb][W+pl+pr][4]. */
int vst_raft_prep(const float* img, float* out, int B, int H, int W, int pad_l, int pad_r, int pad_t,
                  int pad_b, void* stream);
/* Same from an NHWC image with channel stride src_cs (first 3 channels), e.g. a generator output. */
int vst_raft_prep_nhwc(const float* img, int src_cs, float* out, int B, int H, int W, int pad_l, int pad_r,
                       int pad_t, int pad_b, void* stream);
/* y = relu(a + b) (extractor.py ResidualBlock: relu(x + y)); n % 4 == 0. */
int vst_add_relu(const float* a, const float* b, float* y, long n, void* stream);
/* torch.cat along channels: dst[p][dst_c0 + c] = src[p][src_c0 + c], c < nc. */
int vst_copy_channels(const float* src, int src_cs, int src_c0, float* dst, int dst_cs, int dst_c0, int nc,
                      long npix, void* stream);
/* raft.py:107-109 split of the context features: h = tanh(c[:hdim]) (also hx[:, :hdim]),
 * inp = relu(c[hdim:hdim+cdim]) into hx / rhx channels [hdim, hdim+cdim). */
int vst_raft_ctx_split(const float* c, int cs, int hdim, int cdim, float* h, float* hx, float* rhx, int xcs,
                       long npix, void* stream);
/* raft.py:121: flow = coords1 - coords0 (coords1 NCHW [B][2][h][w]) as NHWC4. */
int vst_raft_flow4(const float* coords1, float* flow4, int B, int h, int w, void* stream);
/* update.py:95-96 + 130: [out[:, :nout] | flow] written to hx and rhx channels [c0, c0+nout+2). */
int vst_raft_motion(const float* out, int ocs, int nout, const float* flow4, float* hx, float* rhx, int xcs,
                    int c0, long npix, void* stream);
/* SepConvGRU halves (update.py:46-58): rhx[:, :hd] = sigmoid(zr[:, hd:]) * h, and
 * h = (1 - z) h + z q with z = sigmoid(zr[:, :hd]) (also into hx[:, :hd]). */
int vst_gru_reset(const float* zr, const float* h, float* rhx, int hd, int xcs, long npix, void* stream);
int vst_gru_update(const float* zr, const float* q, float* h, float* hx, int hd, int xcs, long npix, void* stream);
/* raft.py:127: coords1 += delta_flow (delta NHWC, channels 0/1 of stride dcs). */
int vst_raft_coords_update(float* coords1, const float* delta, int dcs, int B, int h, int w, void* stream);
/* raft.py:72-83 convex upsampling: mask NHWC [B][h][w][mcs >= 576] (0.25 already applied),
 * out NCHW [B][2][8h][8w]. */
int vst_raft_upsample(const float* coords1, const float* mask, int mcs, float* out, int B, int h, int w,
                      void* stream);

/* MoGAN motion losses (MoGAN/models/cycle_gan_model.py:294-311): scale * mean(mask * |a - b|) over
 * npix pixels x Cl logical channels of NHWC (channel stride Cs) tensors, mask [npix] broadcast over
 * channels (nullptr = no mask); backward writes d/da (pass (b, a) for d/db), 0 in padded channels. */
int vst_loss_masked_l1(const float* a, const float* b, const float* mask, float* loss, float* part, long npix,
                       int Cs, int Cl, float scale, void* stream);
int vst_loss_masked_l1_bwd(const float* a, const float* b, const float* mask, const float* gout, float* grad,
                           long npix, int Cs, int Cl, float scale, void* stream);

/* ---- input formats ------------------------------------------------------------ */
/* FC2 sample block -> train-step inputs.  Replaces DatasetFC2.__getitem__'s tensor conversion
 * (methods/GAN-based/CycleGANCon/fc2_dataset.py:35-41 with the T.ToTensor + T.Normalize(0.5, 0.5)
 * transform of :79-81): raw float32 [B][H][W][9] (img1 0:3, img2 3:6, mask 6:7, flow 7:9) ->
 * img1, img2 NHWC4 normalised through the uint8 round trip, mask [B][H][W], flow [B][2][H][W]. */
int vst_fc2_unpack(const float* raw, float* img1, float* img2, float* mask, float* flow, int B, int H,
                   int W, void* stream);
/* uint8 RGB HWC (PIL-decoded style frame, fc2_dataset.py:32) -> ToTensor + Normalize(0.5, 0.5),
 * NHWC4 float32 (channel 3 zero). */
int vst_u8_image_to_nhwc4(const unsigned char* x, float* y, long npix, void* stream);

/* ---- SURVEY §8b spelling of the ABI (abi.hip: host wrappers over the entry points above) ----- *
 * The contract in SURVEY §8b names a conv descriptor, a workspace query and a few entry points the
 * shape-argument API above spells differently.  These wrappers give a binder written from §8b the
 * names it expects; each forwards to the kernels above (no extra launch except where stated).
 *   §8b name                         forwards to
 *   vst_conv2d_fwd/dgrad/wgrad(desc) vst_conv2d_fwd_ws / vst_conv2d_tfwd / vst_conv2d_wgrad (the
 *                                    `_desc` suffix: the shape-argument names are taken above)
 *   vst_workspace_size               vst_conv2d_fwd_ws_bytes / vst_conv2d_wgrad_ws_bytes
 *   vst_warp_bilinear_fwd/bwd_input  vst_warp_fwd / vst_warp_masked_fwd (validity mask flag)
 *   vst_masked_sqdiff_mean_fwd/bwd   vst_loss_temporal(_bwd)   (fused warp + masked squared diff)
 *   vst_l1_mean_fwd/bwd              vst_loss_l1(_bwd)
 *   vst_mse_const_fwd/bwd            vst_loss_mse_const(_bwd)
 *   vst_gram                         per-image 1x1 vst_conv2d_wgrad + vst_axpby (1/HW)
 *   vst_corr_volume                  vst_channel_normalize + vst_weight_split + 1x1 vst_conv2d_fwd per
 *                                    image, then vst_corr_pyramid (vst_corr_pyramid / _lookup above)
 *   vst_adam_multi_tensor            vst_adam_step per tensor
 *   vst_instnorm_act_fwd/bwd         (already the §8b names) */
enum { VST_LAYOUT_NHWC = 0 };
enum { VST_DTYPE_F32 = 0 };
enum { VST_OP_FWD = 0, VST_OP_DGRAD = 1, VST_OP_WGRAD = 2 };
typedef struct vst_conv_desc {
  int N, H, W;            /* input batch and spatial size (a transposed conv: its input) */
  int C, K;               /* input / output channel strides (multiples of 4; padding channels zero) */
  int R, S, stride, pad;  /* filter taps, stride, symmetric padding */
  int pad_mode;           /* VST_PAD_ZERO | VST_PAD_REFLECT (reflect: direct convs) */
  int dilation;           /* 1 (0 is read as 1) */
  int transposed;         /* ConvTranspose2d (weight [Ci][Co][R][S]) */
  int output_padding;     /* transposed only */
  int layout;             /* VST_LAYOUT_NHWC */
  int dtype;              /* VST_DTYPE_F32 */
  int epilogue;           /* VST_ACT_* applied after the bias (forward only) */
  float slope;            /* LeakyReLU slope */
  int math;               /* VST_MATH_* */
} vst_conv_desc;
/* Output spatial size of the descriptor's forward op. */
int vst_conv_desc_out_hw(const vst_conv_desc* d, int* Ho, int* Wo);
/* Bytes of caller workspace op (VST_OP_*) needs for this descriptor (0: none; also 0 for a bad desc). */
size_t vst_workspace_size(const vst_conv_desc* d, int op);
/* Forward: y = act(conv(x) + bias).  wp: VST_PACK_OK pack (+ wsplit planes) of a Conv2d weight, or
 * the VST_PACK_IK pack of a ConvTranspose2d weight.  in_part / in_nsplit: optional InstanceNorm
 * partials (vst_conv2d_fwd_in; direct convs). */
int vst_conv2d_fwd_desc(const vst_conv_desc* d, const float* x, const float* wp, const void* wsplit,
                        const float* bias, float* y, double* in_part, int* in_nsplit, float* ws, size_t ws_bytes,
                        void* stream);
/* Data gradient: dx from dy.  Conv2d: wp = VST_PACK_IK pack (reflect padding folded in-kernel);
 * ConvTranspose2d: wp = the VST_PACK_OK pack of its weight seen as a Conv2d weight [Ci][Co] (+ planes). */
int vst_conv2d_dgrad_desc(const vst_conv_desc* d, const float* dy, const float* wp, const void* wsplit, float* dx,
                          float* ws, size_t ws_bytes, void* stream);
/* Weight gradient into dw (PyTorch layout of the weight, Co x Ci logical output / input channels of
 * the layer; accumulate != 0 adds).  ws: vst_workspace_size(d, VST_OP_WGRAD) bytes. */
int vst_conv2d_wgrad_desc(const vst_conv_desc* d, const float* x, const float* dy, float* dw, int Co, int Ci,
                          int accumulate, float* ws, size_t ws_bytes, void* stream);
int vst_adam_multi_tensor(float* const* p, const float* const* g, float* const* m, float* const* v, const long* n,
                          int ntensors, float lr, float beta1, float beta2, float eps, int step, void* stream);
/* G[b] = F_b^T F_b / HW for NHWC features f [B][HW][C] (fast_style_transfer.py:813-817). */
size_t vst_gram_ws_bytes(int HW, int C);
int vst_gram(const float* f, float* G, int B, int HW, int C, float* ws, size_t ws_bytes, int math, void* stream);
/* CorrBlock volume + pyramid (corr.py:12-60) from NHWC fmaps [B][H][W][Dp] (D logical channels);
 * sqrt_d: device array of D floats = sqrt(D); pyr: vst_corr_pyramid_floats(B*H*W, H, W, ld0, levels) floats
 * with the level-0 plane stride ld0 = H*W rounded up to a multiple of 4. */
size_t vst_corr_volume_ws_bytes(int B, int H, int W, int Dp);
int vst_corr_volume(const float* f1, const float* f2, float* pyr, int B, int H, int W, int Dp, int D,
                    const float* sqrt_d, int levels, float* ws, size_t ws_bytes, int math, void* stream);
int vst_warp_bilinear_fwd(const float* x, const float* flow, float* out, int N, int H, int W, int Cs,
                          int align_corners, int validity_mask, void* stream);
int vst_warp_bilinear_bwd_input(const float* gout, const float* flow, float* gx, int N, int H, int W, int Cs,
                                int align_corners, int validity_mask, void* stream);
int vst_masked_sqdiff_mean_fwd(const float* a, const float* b, const float* flow, const float* mask, float* loss,
                               float* part, int N, int H, int W, int Cs, int Cl, float lambda, void* stream);
int vst_masked_sqdiff_mean_bwd(const float* a, const float* b, const float* flow, const float* mask,
                               const float* gout, float* ga, float* gb, int N, int H, int W, int Cs, int Cl,
                               float lambda, void* stream);
int vst_l1_mean_fwd(const float* a, const float* b, float* loss, float* part, long npix, int Cs, int Cl, float scale,
                    void* stream);
int vst_l1_mean_bwd(const float* a, const float* b, const float* gout, float* grad, long npix, int Cs, int Cl,
                    float scale, void* stream);
int vst_mse_const_fwd(const float* a, float target, float* loss, float* part, long npix, int Cs, int Cl, float scale,
                      void* stream);
int vst_mse_const_bwd(const float* a, float target, const float* gout, float* grad, long npix, int Cs, int Cl,
                      float scale, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* VST_HIP_H */
