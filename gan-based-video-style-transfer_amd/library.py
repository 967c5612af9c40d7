"""``torch.library`` registration of the C-ABI entries as ``vst::*`` operators (SURVEY §8b "Callers").

The module facades (networks.py, perceptual.py, flowtools.py) call libvst_hip through ctypes inside
their own autograd Functions; this module exposes the same kernels as first-class PyTorch operators,
so they are visible to ``torch.ops``, FX / ``torch.compile`` tracing (each op has a fake-tensor
implementation for shape propagation) and ``torch.library.opcheck``.  Every op takes and returns the
reference's NCHW fp32 tensors — the semantics of the PyTorch call it replaces — and converts to the
library's NHWC layout on the device.  Backward passes are themselves ``vst::`` ops.

  vst::conv2d(x, weight, bias?, stride, padding, pad_mode)          nn.Conv2d (+ ReflectionPad2d)
        networks.py:340-367 (reflect 3x3 ResnetBlock convs), :404-426 (s2 down convs), :556-578 (D)
  vst::conv_transpose2d(x, weight, bias?, stride, padding, output_padding)   nn.ConvTranspose2d
        networks.py:408-416 (up-sampling layers)
  vst::instance_norm_act(x, act, slope)        InstanceNorm2d(affine=False) + ReLU / LeakyReLU / none
  vst::warp_bilinear(x, flow)                  utils/flowtools.py:18-32 (F.grid_sample, zeros)
  vst::fbcheck(flow_fw, flow_bw)               utils/flowtools.py:34-58 (fbcCheckTorch)
  vst::temporal_loss(a, b, flow, mask, lam)    CycleGANCon cycle_gan_model.py:191-204
  vst::gram(f)                                 learning-based fast_style_transfer.py:813-817
  vst::adam_(param, grad, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, step)   torch.optim.Adam step

All ops require contiguous float32 CUDA tensors and raise on CPU inputs (no fallback).
"""
from typing import List, Optional, Tuple

import torch
from torch import Tensor

from . import ops

_ACTS = ("none", "relu", "lrelu")


def _nhwc(x):
    return ops.nchw_to_nhwc(x.contiguous())


def _bias_padded(bias, co):
    if bias is None:
        return None
    b = torch.zeros(ops.cpad(co), device=bias.device)
    b[:co] = bias.detach()
    return b


def _check_pad(pad_mode):
    if pad_mode not in ops.PAD:
        raise ValueError("vst: pad_mode must be 'zero' or 'reflect', got %r" % pad_mode)


# ----------------------------------------------------------------------------------- conv2d
@torch.library.custom_op("vst::conv2d", mutates_args=())
def conv2d(x: Tensor, weight: Tensor, bias: Optional[Tensor], stride: int, padding: int,
           pad_mode: str) -> Tensor:
    """y = conv2d(pad(x, padding, pad_mode), weight, bias, stride): the reference's
    [ReflectionPad2d(p)] + Conv2d(k, stride, padding=0 | p) pair as one op."""
    _check_pad(pad_mode)
    ops._dev_check(x, weight)
    Co, Ci, R, S = weight.shape
    if x.shape[1] != Ci:
        raise ValueError("vst::conv2d: x has %d channels, weight expects %d" % (x.shape[1], Ci))
    wp = ops.weight_pack(weight.detach().contiguous(), ops.PACK_FWD)
    y = ops.conv2d_fwd(_nhwc(x), wp, _bias_padded(bias, Co), ops.cpad(Co), R, S, stride, padding, pad_mode)
    return ops.nhwc_to_nchw(y, Co)


@conv2d.register_fake
def _(x, weight, bias, stride, padding, pad_mode):
    N, _, H, W = x.shape
    Co, _, R, S = weight.shape
    return x.new_empty((N, Co, (H + 2 * padding - R) // stride + 1, (W + 2 * padding - S) // stride + 1))


@torch.library.custom_op("vst::conv2d_backward", mutates_args=())
def conv2d_backward(grad: Tensor, x: Tensor, weight: Tensor, stride: int, padding: int,
                    pad_mode: str, need_input: bool = True, need_weight: bool = True) -> Tuple[Tensor, Tensor, Tensor]:
    """(dx, dweight, dbias) of vst::conv2d.  dx: the transposed conv (reflect, stride 1: mirrored
    contributions gathered in-kernel; reflect, stride > 1: the transposed conv onto the padded frame,
    then the reflect fold); dweight: the split-K weight-gradient GEMM; dbias: the per-channel sum of
    grad.  need_input / need_weight = False skip that GEMM (its output is returned as zeros)."""
    _check_pad(pad_mode)
    ops._dev_check(grad, x, weight)
    N, Ci, H, W = x.shape
    Co, _, R, S = weight.shape
    gy = _nhwc(grad)
    if need_input:
        ik = ops.weight_pack(weight.detach().contiguous(), ops.PACK_DGRAD)
        if pad_mode == "reflect" and stride != 1:
            dxp = ops.conv2d_tfwd(gy, ik, None, H + 2 * padding, W + 2 * padding, ops.cpad(Ci), R, S, stride, 0)
            dx = ops.nhwc_to_nchw(ops.reflect_fold(dxp, padding), Ci)
        else:
            dxn = ops.conv2d_tfwd(gy, ik, None, H, W, ops.cpad(Ci), R, S, stride, padding, pad_mode=pad_mode)
            dx = ops.nhwc_to_nchw(dxn, Ci)
    else:
        dx = torch.zeros_like(x)
    dw = torch.zeros_like(weight)
    db = torch.zeros(Co, device=x.device)
    if need_weight:
        ops.conv2d_wgrad(_nhwc(x), gy, dw, db, R, S, stride, padding, pad_mode, Co, Ci, Ci * R * S, R * S,
                         accumulate=False)
    else:
        ops.channel_sum(gy, db, Co, accumulate=False)
    return dx, dw, db


@conv2d_backward.register_fake
def _(grad, x, weight, stride, padding, pad_mode, need_input=True, need_weight=True):
    return torch.empty_like(x), torch.empty_like(weight), weight.new_empty((weight.shape[0],))


def _conv2d_setup(ctx, inputs, output):
    x, weight, bias, stride, padding, pad_mode = inputs
    ctx.save_for_backward(x, weight)
    ctx.conf = (stride, padding, pad_mode, bias is not None)


def _conv2d_bwd(ctx, grad):
    x, weight = ctx.saved_tensors
    stride, padding, pad_mode, has_bias = ctx.conf
    need_x, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
    dx, dw, db = torch.ops.vst.conv2d_backward(grad.contiguous(), x, weight, stride, padding, pad_mode,
                                               need_x, need_w)
    return (dx if need_x else None), (dw if need_w else None), (db if has_bias else None), None, None, None


conv2d.register_autograd(_conv2d_bwd, setup_context=_conv2d_setup)


# -------------------------------------------------------------------------- conv_transpose2d
def _convT_out(n, stride, padding, k, output_padding):
    return (n - 1) * stride - 2 * padding + k + output_padding


@torch.library.custom_op("vst::conv_transpose2d", mutates_args=())
def conv_transpose2d(x: Tensor, weight: Tensor, bias: Optional[Tensor], stride: int, padding: int,
                     output_padding: int) -> Tensor:
    """nn.ConvTranspose2d(Ci, Co, k, stride, padding, output_padding) with weight [Ci][Co][k][k]:
    the gather-form transposed conv (vst_conv2d_tfwd) with the weight read as O = Ci, I = Co."""
    ops._dev_check(x, weight)
    N, Ci, H, W = x.shape
    _, Co, R, S = weight.shape
    Ho, Wo = _convT_out(H, stride, padding, R, output_padding), _convT_out(W, stride, padding, S, output_padding)
    ik = ops.weight_pack(weight.detach().contiguous(), ops.PACK_DGRAD)
    y = ops.conv2d_tfwd(_nhwc(x), ik, _bias_padded(bias, Co), Ho, Wo, ops.cpad(Co), R, S, stride, padding,
                        role="fwd")
    return ops.nhwc_to_nchw(y, Co)


@conv_transpose2d.register_fake
def _(x, weight, bias, stride, padding, output_padding):
    N, _, H, W = x.shape
    _, Co, R, S = weight.shape
    return x.new_empty((N, Co, _convT_out(H, stride, padding, R, output_padding),
                        _convT_out(W, stride, padding, S, output_padding)))


@torch.library.custom_op("vst::conv_transpose2d_backward", mutates_args=())
def conv_transpose2d_backward(grad: Tensor, x: Tensor, weight: Tensor, stride: int,
                              padding: int) -> Tuple[Tensor, Tensor, Tensor]:
    """(dx, dweight, dbias) of vst::conv_transpose2d: dx is the forward conv of grad with the same
    weight (O = Ci, I = Co); dweight is the weight gradient of that conv with x := grad,
    dy := x (include/vst_hip.h, vst_conv2d_wgrad)."""
    ops._dev_check(grad, x, weight)
    N, Ci, H, W = x.shape
    _, Co, R, S = weight.shape
    gy = _nhwc(grad)
    ok = ops.weight_pack(weight.detach().contiguous(), ops.PACK_FWD)
    dx = ops.conv2d_fwd(gy, ok, None, ops.cpad(Ci), R, S, stride, padding, role="bwd")
    if dx.shape[1] != H or dx.shape[2] != W:
        raise ValueError("vst::conv_transpose2d_backward: inconsistent output_padding")
    dw = torch.zeros_like(weight)
    ops.conv2d_wgrad(gy, _nhwc(x), dw, None, R, S, stride, padding, "zero", Ci, Co, Co * R * S, R * S,
                     accumulate=False)
    db = torch.zeros(Co, device=x.device)
    ops.channel_sum(gy, db, Co, accumulate=False)
    return ops.nhwc_to_nchw(dx, Ci), dw, db


@conv_transpose2d_backward.register_fake
def _(grad, x, weight, stride, padding):
    return torch.empty_like(x), torch.empty_like(weight), weight.new_empty((weight.shape[1],))


def _convT_setup(ctx, inputs, output):
    x, weight, bias, stride, padding, _ = inputs
    ctx.save_for_backward(x, weight)
    ctx.conf = (stride, padding, bias is not None)


def _convT_bwd(ctx, grad):
    x, weight = ctx.saved_tensors
    stride, padding, has_bias = ctx.conf
    dx, dw, db = torch.ops.vst.conv_transpose2d_backward(grad.contiguous(), x, weight, stride, padding)
    return dx, dw, (db if has_bias else None), None, None, None


conv_transpose2d.register_autograd(_convT_bwd, setup_context=_convT_setup)


# ------------------------------------------------------------------------ instance_norm_act
@torch.library.custom_op("vst::instance_norm_act", mutates_args=())
def instance_norm_act(x: Tensor, act: str, slope: float) -> Tensor:
    """act(InstanceNorm2d(affine=False, eps=1e-5)(x)); act in none | relu | lrelu (fp64 statistics)."""
    if act not in _ACTS:
        raise ValueError("vst::instance_norm_act: act must be one of %s" % (_ACTS,))
    C = x.shape[1]
    y = _nhwc(x)
    a = ops.instnorm_act_fwd(y, ops.instnorm_stats(y), act, slope)
    return ops.nhwc_to_nchw(a, C)


@instance_norm_act.register_fake
def _(x, act, slope):
    return torch.empty_like(x)


@torch.library.custom_op("vst::instance_norm_act_backward", mutates_args=())
def instance_norm_act_backward(grad: Tensor, x: Tensor, act: str, slope: float) -> Tensor:
    C = x.shape[1]
    y = _nhwc(x)
    dy = ops.instnorm_act_bwd(_nhwc(grad), y, ops.instnorm_stats(y), act, slope)
    return ops.nhwc_to_nchw(dy, C)


@instance_norm_act_backward.register_fake
def _(grad, x, act, slope):
    return torch.empty_like(x)


def _in_setup(ctx, inputs, output):
    x, act, slope = inputs
    ctx.save_for_backward(x)
    ctx.conf = (act, slope)


def _in_bwd(ctx, grad):
    (x,) = ctx.saved_tensors
    return torch.ops.vst.instance_norm_act_backward(grad.contiguous(), x, *ctx.conf), None, None


instance_norm_act.register_autograd(_in_bwd, setup_context=_in_setup)


# ------------------------------------------------------------------------------------ flow
@torch.library.custom_op("vst::warp_bilinear", mutates_args=())
def warp_bilinear(x: Tensor, flow: Tensor) -> Tensor:
    """utils/flowtools.py:18-32: backward bilinear warp of x [B,C,H,W] by flow [B,2,H,W] (pixels,
    channel 0 = x displacement), zeros outside, align_corners=False."""
    ops._dev_check(flow)
    C = x.shape[1]
    return ops.nhwc_to_nchw(ops.warp_nhwc(_nhwc(x), flow.contiguous()), C)


@warp_bilinear.register_fake
def _(x, flow):
    return torch.empty_like(x)


@torch.library.custom_op("vst::warp_bilinear_backward", mutates_args=())
def warp_bilinear_backward(grad: Tensor, flow: Tensor) -> Tensor:
    """Gradient w.r.t. x of vst::warp_bilinear (the bilinear scatter; the flow gets none, as in every
    training path of the reference)."""
    C = grad.shape[1]
    return ops.nhwc_to_nchw(ops.warp_bwd_nhwc(_nhwc(grad), flow.contiguous()), C)


@warp_bilinear_backward.register_fake
def _(grad, flow):
    return torch.empty_like(grad)


def _warp_setup(ctx, inputs, output):
    ctx.save_for_backward(inputs[1])


def _warp_bwd(ctx, grad):
    (flow,) = ctx.saved_tensors
    return torch.ops.vst.warp_bilinear_backward(grad.contiguous(), flow), None


warp_bilinear.register_autograd(_warp_bwd, setup_context=_warp_setup)


@torch.library.custom_op("vst::fbcheck", mutates_args=())
def fbcheck(flow_fw: Tensor, flow_bw: Tensor) -> Tensor:
    """utils/flowtools.py:34-58 fbcCheckTorch: occlusion / motion-boundary mask [B,1,H,W]."""
    return ops.fbcheck(flow_fw.contiguous(), flow_bw.contiguous())


@fbcheck.register_fake
def _(flow_fw, flow_bw):
    B, _, H, W = flow_bw.shape
    return flow_bw.new_empty((B, 1, H, W))


# ---------------------------------------------------------------------------------- losses
@torch.library.custom_op("vst::temporal_loss", mutates_args=())
def temporal_loss(a: Tensor, b: Tensor, flow: Tensor, mask: Tensor, lam: float) -> Tensor:
    """lam * mean((mask * (b - warp(a, flow)))^2) over [B,3,H,W] frames (CycleGANCon
    cycle_gan_model.py:191-204, a = fake_B, b = fake_B2)."""
    C = a.shape[1]
    return ops.loss_temporal(_nhwc(a), _nhwc(b), flow.contiguous(), mask.contiguous(), lam, cl=C)


@temporal_loss.register_fake
def _(a, b, flow, mask, lam):
    return a.new_empty(())


@torch.library.custom_op("vst::temporal_loss_backward", mutates_args=())
def temporal_loss_backward(grad: Tensor, a: Tensor, b: Tensor, flow: Tensor, mask: Tensor,
                           lam: float) -> Tuple[Tensor, Tensor]:
    C = a.shape[1]
    an, bn = _nhwc(a), _nhwc(b)
    ga, gb = torch.zeros_like(an), torch.empty_like(bn)
    ops.loss_temporal_bwd(an, bn, flow.contiguous(), mask.contiguous(), grad.contiguous(), ga, gb, lam, cl=C)
    return ops.nhwc_to_nchw(ga, C), ops.nhwc_to_nchw(gb, C)


@temporal_loss_backward.register_fake
def _(grad, a, b, flow, mask, lam):
    return torch.empty_like(a), torch.empty_like(b)


def _tl_setup(ctx, inputs, output):
    a, b, flow, mask, lam = inputs
    ctx.save_for_backward(a, b, flow, mask)
    ctx.lam = lam


def _tl_bwd(ctx, grad):
    a, b, flow, mask = ctx.saved_tensors
    ga, gb = torch.ops.vst.temporal_loss_backward(grad, a, b, flow, mask, ctx.lam)
    return ga, gb, None, None, None


temporal_loss.register_autograd(_tl_bwd, setup_context=_tl_setup)


@torch.library.custom_op("vst::gram", mutates_args=())
def gram(f: Tensor) -> Tensor:
    """fast_style_transfer.py:813-817 gram_matrix of [B,C,H,W] features: bmm(F, F^T) / (h*w) per
    sample (C % 4 == 0), on the split-K weight-gradient GEMM (ops.gram)."""
    if f.shape[1] % 4:
        raise NotImplementedError("vst::gram: channel count must be a multiple of 4")
    return ops.gram(_nhwc(f))


@gram.register_fake
def _(f):
    B, C = f.shape[0], f.shape[1]
    return f.new_empty((B, C, C))


@torch.library.custom_op("vst::gram_backward", mutates_args=())
def gram_backward(grad: Tensor, f: Tensor) -> Tensor:
    """dF_b = (dG_b + dG_b^T) F_b / (h*w) (ops.gram_bwd: a 1x1 conv with the symmetrised weight)."""
    return ops.nhwc_to_nchw(ops.gram_bwd(_nhwc(f), grad.contiguous()), f.shape[1])


@gram_backward.register_fake
def _(grad, f):
    return torch.empty_like(f)


def _gram_setup(ctx, inputs, output):
    ctx.save_for_backward(inputs[0])


def _gram_bwd(ctx, grad):
    (f,) = ctx.saved_tensors
    return torch.ops.vst.gram_backward(grad.contiguous(), f)


gram.register_autograd(_gram_bwd, setup_context=_gram_setup)


# ----------------------------------------------------------------------------------- Adam
@torch.library.custom_op("vst::adam_", mutates_args=("param", "exp_avg", "exp_avg_sq"))
def adam_(param: Tensor, grad: Tensor, exp_avg: Tensor, exp_avg_sq: Tensor, lr: float, beta1: float,
          beta2: float, eps: float, step: int) -> None:
    """One torch.optim.Adam step (weight_decay 0, amsgrad off, bias-corrected) over flat fp32
    buffers, in place (adam_k)."""
    ops.adam_step(param, grad, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, step)


@adam_.register_fake
def _(param, grad, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, step):
    return None


OPS: List[str] = ["conv2d", "conv2d_backward", "conv_transpose2d", "conv_transpose2d_backward",
                  "instance_norm_act", "instance_norm_act_backward", "warp_bilinear", "warp_bilinear_backward",
                  "fbcheck", "temporal_loss", "temporal_loss_backward", "gram", "gram_backward", "adam_"]
