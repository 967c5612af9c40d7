"""StarGAN generator / discriminator and the WGAN-GP train iteration, HIP-backed.

Drop-in for methods/GAN-based/StarGAN/model.py (``Generator(conv_dim, c_dim, repeat_num)``,
``Discriminator(image_size, conv_dim, c_dim, repeat_num)``, ``ResidualBlock``; identical module
trees and state_dict keys incl. the InstanceNorm running buffers) and the training iteration of
solver.py:241-363 (``StarGANSolver.train_step``: D step with the gradient penalty of
solver.py:187-199 every iteration, G step every ``n_critic``), with ``classification_loss``
(solver.py:234-239) and Adam(lr, [beta1, beta2]) (solver.py:134-135).

MI355X design:
  * The generator is ONE autograd node over NHWC fp32 kernels (like networks.ResnetGenerator):
    label concat kernel, zero-padded implicit-GEMM MFMA convs (7x7, 4x4 s2, 3x3 residual, 4x4 s2
    transposed), affine InstanceNorm(+ReLU, + residual) with fp64 statistics and the running-buffer
    update of track_running_stats=True (eval mode normalises with the running buffers).
  * The discriminator must be twice differentiable (WGAN-GP differentiates ||dD/dx||).  It is built
    from per-layer autograd Functions whose backward is itself made of autograd Functions over the
    same kernels: conv -> (data-gradient, weight-gradient, bias channel-sum); data-gradient ->
    (conv, weight-gradient); weight-gradient -> (data-gradient, conv) with the weight pack of the
    incoming gradient made on the fly; LeakyReLU' masks re-applied by the act-backward kernel.
    torch.autograd then composes the double backward of the gradient penalty from these.
"""
import contextlib

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from .networks import TAP_LAST, Conv2d, ConvTranspose2d, FlatNet, _Marker, _padded_bias
from .ops import cpad
from .optim import FusedAdam


###############################################################################
# twice-differentiable NHWC building blocks (discriminator / gradient penalty)
###############################################################################
class _ToNHWC2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cs):
        ctx.c = x.shape[1]
        return ops.nchw_to_nhwc(x.contiguous(), cs)

    @staticmethod
    def backward(ctx, g):
        return _ToNCHW2.apply(g.contiguous(), ctx.c), None


class _ToNCHW2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, c):
        ctx.cs = y.shape[-1]
        return ops.nhwc_to_nchw(y.contiguous(), c)

    @staticmethod
    def backward(ctx, g):
        return _ToNHWC2.apply(g.contiguous(), ctx.cs), None


# The Conv2d(k4, s2, p1) data gradients on the four-phase kernel (ops.conv4s2_dgrad: the 2x2 phase convs in one
# launch, stored interleaved) instead of the generic transposed-conv gather; False keeps the latter.
SG_PHASES = True
# The gradient penalty's first-order pass (autograd.grad of D's output w.r.t. x_hat) computes only the data
# gradients: the reference's native conv backward skips the weight / bias gradients there (the engine's
# output mask: only x_hat's gradient is requested), which are never part of the penalty's graph.  Set by
# gradient_penalty around its autograd.grad call (a module global: the autograd engine runs the backward on
# its device thread).
_INPUT_GRAD_ONLY = [False]
# Set by StarGANSolver around d_loss.backward(), whose only consumers of the discriminator's parameter gradients
# are their .grad views of the flat gradient buffer: the conv weight / bias gradients (the main pass's and the
# penalty's double-backward contributions) are then accumulated there by the kernels' accumulate mode instead of
# being returned to autograd, whose AccumulateGrad would add each one in a pass of its own (the 1024 -> 2048
# layer's 134 MB three times per iteration).  Never set around autograd.grad calls.
_ACCUM_PARAM_GRADS = [False]
# 0: autograd accumulation, D's parameter gradients in the G step
SG_DIRECT = True


def _direct(p):
    return _ACCUM_PARAM_GRADS[0] and p is not None and p.grad is not None and not torch.is_grad_enabled()


class ConvSpec:
    """Geometry of one conv layer plus its cached weight packs (per weight version)."""

    def __init__(self, owner, mod, stride, pad, act=None, slope=0.0):
        self.owner, self.mod, self.stride, self.pad, self.act, self.slope = owner, mod, stride, pad, act, slope
        w = mod.weight
        self.co, self.ci, self.R = w.shape[0], w.shape[1], w.shape[2]
        self.cop, self.cip = cpad(self.co), cpad(self.ci)
        self.index = 0  # position in the owner's pack list (Discriminator.specs)
        self.phased = SG_PHASES and stride == 2 and self.R == 4 and pad == 1 and self.cop % 32 == 0 and self.cip != 4

    def _make(self):
        """This layer's packs (inside the owner's ops.PackBatch: one launch for the network, re-run in place
        after each weight update): forward pack, transposed pack (unphased layers), padded bias, phase packs."""
        m = self.mod
        ok = ops.weight_pack(m.weight, ops.PACK_FWD)
        ik = None if self.phased else ops.weight_pack(m.weight, ops.PACK_DGRAD)
        ph = ops.conv4s2_dgrad_phase_packs(m.weight) if self.phased else None
        return ok, ik, _padded_bias(m), ph

    def packs(self):
        """(forward pack, transposed pack or None, padded bias) of the current weight version."""
        return self.owner.packs()[self.index][:3]

    def phase_packs(self):
        """conv4s2_dgrad's phase packs of the current weight version."""
        return self.owner.packs()[self.index][3]

    def out_hw(self, H, W):
        return ((H + 2 * self.pad - self.R) // self.stride + 1, (W + 2 * self.pad - self.R) // self.stride + 1)


def _conv_raw(x, ok, spec, bias=None, act="none"):
    return ops.conv2d_fwd(x, ok, bias, spec.cop, spec.R, spec.R, spec.stride, spec.pad, "zero", act=act,
                          slope=spec.slope, role="fwd")


def _dgrad_raw(gz, ik, spec, H, W, phases=None):
    if phases is not None and H == 2 * gz.shape[1] and W == 2 * gz.shape[2]:
        return ops.conv4s2_dgrad(gz, phases, spec.cip)
    if ik is None:  # a phased layer on an odd-sized input
        ik = ops.weight_pack(spec.mod.weight.detach(), ops.PACK_DGRAD)
    return ops.conv2d_tfwd(gz, ik, None, H, W, spec.cip, spec.R, spec.R, spec.stride, spec.pad)


def _wgrad_raw(x, gz, spec, out=None):
    """The weight gradient as a new tensor, or (out: a .grad buffer) accumulated into out."""
    gw = torch.empty((spec.co, spec.ci, spec.R, spec.R), device=x.device) if out is None else out
    ops.conv2d_wgrad(x, gz, gw, None, spec.R, spec.R, spec.stride, spec.pad, "zero", spec.co, spec.ci,
                     spec.ci * spec.R * spec.R, spec.R * spec.R, accumulate=out is not None)
    return gw


class _Conv(torch.autograd.Function):
    """a = act(conv(x, W) + b) on NHWC; backward built from differentiable Functions."""

    @staticmethod
    def forward(ctx, x, w, b, spec):
        ok, _, bias = spec.packs()
        a = _conv_raw(x, ok, spec, bias, "lrelu" if spec.act else "none")
        ctx.spec = spec
        ctx.save_for_backward(x, w, a)
        return a

    @staticmethod
    def backward(ctx, g):
        x, w, a = ctx.saved_tensors
        spec = ctx.spec
        g = g.contiguous()
        gz = _ActBwd.apply(g, a, spec.slope) if spec.act else g
        gx = _Dgrad.apply(gz, w, spec, x.shape[1], x.shape[2]) if ctx.needs_input_grad[0] else None
        only_x = _INPUT_GRAD_ONLY[0]
        gw = gb = None
        m = spec.mod
        if ctx.needs_input_grad[1] and not only_x:
            if _direct(m.weight):
                _wgrad_raw(x, gz, spec, out=m.weight.grad)
            else:
                gw = _Wgrad.apply(x, gz, spec)
        if ctx.needs_input_grad[2] and not only_x:
            if _direct(m.bias):
                ops.channel_sum(gz, m.bias.grad, spec.co, accumulate=True)
            else:
                gb = _ChSum.apply(gz, spec.co)
        return gx, gw, gb, None


class _ActBwd(torch.autograd.Function):
    """g * lrelu'(a) (a = the activation output); d/dg = lrelu'(a), d/da = 0 almost everywhere."""

    @staticmethod
    def forward(ctx, g, a, slope):
        ctx.save_for_backward(a)
        ctx.slope = slope
        return ops.act_bwd(g, a, "lrelu", slope)

    @staticmethod
    def backward(ctx, gg):
        (a,) = ctx.saved_tensors
        return ops.act_bwd(gg.contiguous(), a, "lrelu", ctx.slope), None, None


class _Dgrad(torch.autograd.Function):
    """gx = conv^T(gz; W): bilinear in (gz, W)."""

    @staticmethod
    def forward(ctx, gz, w, spec, H, W):
        _, ik, _ = spec.packs()
        ctx.spec = spec
        ctx.save_for_backward(gz, w)
        return _dgrad_raw(gz, ik, spec, H, W, spec.phase_packs() if spec.phased else None)

    @staticmethod
    def backward(ctx, ggx):
        gz, w = ctx.saved_tensors
        spec = ctx.spec
        ggx = ggx.contiguous()
        ok, _, _ = spec.packs()
        d_gz = _conv_raw(ggx, ok, spec) if ctx.needs_input_grad[0] else None
        d_w = None
        if ctx.needs_input_grad[1]:
            if _direct(spec.mod.weight):
                _wgrad_raw(ggx, gz, spec, out=spec.mod.weight.grad)
            else:
                d_w = _wgrad_raw(ggx, gz, spec)
        return d_gz, d_w, None, None, None


class _Wgrad(torch.autograd.Function):
    """gW = sum_p x_gather (x) gz: bilinear in (x, gz)."""

    @staticmethod
    def forward(ctx, x, gz, spec):
        ctx.spec = spec
        ctx.save_for_backward(x, gz)
        return _wgrad_raw(x, gz, spec)

    @staticmethod
    def backward(ctx, ggw):
        x, gz = ctx.saved_tensors
        spec = ctx.spec
        ggw = ggw.contiguous()
        ok = ops.weight_pack(ggw, ops.PACK_FWD)
        ik = ops.weight_pack(ggw, ops.PACK_DGRAD)
        d_x = _dgrad_raw(gz, ik, spec, x.shape[1], x.shape[2]) if ctx.needs_input_grad[0] else None
        d_gz = _conv_raw(x, ok, spec) if ctx.needs_input_grad[1] else None
        return d_x, d_gz, None


class _ChSum(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gz, co):
        ctx.shape = gz.shape
        db = torch.empty(co, device=gz.device)
        ops.channel_sum(gz, db, co, accumulate=False)
        return db

    @staticmethod
    def backward(ctx, gdb):
        # d(sum_p gz[p][c]) / d gz = 1: broadcast (never reached by the gradient penalty, whose
        # double backward only follows the data-gradient path)
        out = torch.zeros(ctx.shape, device=gdb.device)
        out[..., :gdb.numel()] = gdb
        return out, None


def conv_layer(x, spec):
    m = spec.mod
    return _Conv.apply(x, m.weight, m.bias, spec)


###############################################################################
# Discriminator (model.py:68-88)
###############################################################################
class Discriminator(FlatNet):
    """PatchGAN with a source head (3x3 -> 1) and a domain head (k x k -> c_dim, k = image/2^repeat)."""

    def __init__(self, image_size=128, conv_dim=64, c_dim=5, repeat_num=6):
        super().__init__()
        layers = [Conv2d(3, conv_dim, 4, stride=2, padding=1), _Marker("LeakyReLU(0.01)")]
        curr = conv_dim
        for _ in range(1, repeat_num):
            layers += [Conv2d(curr, curr * 2, 4, stride=2, padding=1), _Marker("LeakyReLU(0.01)")]
            curr *= 2
        k = int(image_size / np.power(2, repeat_num))
        self.main = nn.Sequential(*layers)
        self.conv1 = Conv2d(curr, 1, 3, stride=1, padding=1, bias=False)
        self.conv2 = Conv2d(curr, c_dim, k, bias=False)
        self.image_size, self.c_dim, self.k = image_size, c_dim, k
        self._flatten()
        self._specs = None

    def specs(self):
        if self._specs is None:
            main = [ConvSpec(self, m, 2, 1, act=True, slope=0.01) for m in self.main if isinstance(m, Conv2d)]
            self._specs = main + [ConvSpec(self, self.conv1, 1, 1), ConvSpec(self, self.conv2, 1, 0)]
            for i, sp in enumerate(self._specs):
                sp.index = i
        return self._specs

    def _make_packs(self):
        return [sp._make() for sp in self.specs()]

    def _flatten(self):
        super()._flatten()
        self._specs = None

    def forward(self, x):
        """x: NCHW [B, 3, H, W] -> (out_src [B, 1, h, w], out_cls [B, c_dim])."""
        sp = self.specs()
        h = _ToNHWC2.apply(x, cpad(3))
        for s in sp[:-2]:
            h = conv_layer(h, s)
        out_src = _ToNCHW2.apply(conv_layer(h, sp[-2]), 1)
        out_cls = _ToNCHW2.apply(conv_layer(h, sp[-1]), self.c_dim)
        return out_src, out_cls.reshape(out_cls.size(0), out_cls.size(1))


###############################################################################
# Generator (model.py:7-65)
###############################################################################
class InstanceNormTracked(nn.Module):
    """Holder with nn.InstanceNorm2d(affine=True, track_running_stats=True)'s state."""

    def __init__(self, c, momentum=0.1):
        super().__init__()
        self.num_features, self.momentum = c, momentum
        self.weight = nn.Parameter(torch.ones(c))
        self.bias = nn.Parameter(torch.zeros(c))
        self.register_buffer("running_mean", torch.zeros(c))
        self.register_buffer("running_var", torch.ones(c))
        self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long))

    def extra_repr(self):
        return f"{self.num_features}, eps=1e-05, momentum={self.momentum}, affine=True, track_running_stats=True"


class ResidualBlock(nn.Module):
    def __init__(self, dim_in, dim_out):
        super().__init__()
        self.main = nn.Sequential(
            Conv2d(dim_in, dim_out, 3, stride=1, padding=1, bias=False), InstanceNormTracked(dim_out),
            _Marker("ReLU(inplace=True)"), Conv2d(dim_out, dim_out, 3, stride=1, padding=1, bias=False),
            InstanceNormTracked(dim_out))


class Generator(FlatNet):
    def __init__(self, conv_dim=64, c_dim=5, repeat_num=6):
        super().__init__()
        L = [Conv2d(3 + c_dim, conv_dim, 7, stride=1, padding=3, bias=False), InstanceNormTracked(conv_dim),
             _Marker("ReLU(inplace=True)")]
        curr = conv_dim
        for _ in range(2):
            L += [Conv2d(curr, curr * 2, 4, stride=2, padding=1, bias=False), InstanceNormTracked(curr * 2),
                  _Marker("ReLU(inplace=True)")]
            curr *= 2
        for _ in range(repeat_num):
            L.append(ResidualBlock(curr, curr))
        for _ in range(2):
            L += [ConvTranspose2d(curr, curr // 2, 4, stride=2, padding=1, bias=False),
                  InstanceNormTracked(curr // 2), _Marker("ReLU(inplace=True)")]
            curr //= 2
        L += [Conv2d(curr, 3, 7, stride=1, padding=3, bias=False), _Marker("Tanh()")]
        self.main = nn.Sequential(*L)
        self.conv_dim, self.c_dim, self.repeat_num = conv_dim, c_dim, repeat_num
        self.input_nc, self.output_nc = 3 + c_dim, 3
        self._flatten()

    def _parts(self):
        m = self.main
        down = [(m[0], m[1], 7, 1, 3), (m[3], m[4], 4, 2, 1), (m[6], m[7], 4, 2, 1)]
        res = [m[9 + i].main for i in range(self.repeat_num)]
        j = 9 + self.repeat_num
        up = [(m[j], m[j + 1]), (m[j + 3], m[j + 4])]
        return down, res, up, m[j + 6]

    def _make_packs(self):
        down, res, up, last = self._parts()
        P = {"down": [(ops.weight_pack(c.weight, ops.PACK_FWD), ops.weight_pack(c.weight, ops.PACK_DGRAD))
                      for c, *_ in down],
             "res": [tuple((ops.weight_pack(b[i].weight, ops.PACK_FWD), ops.weight_pack(b[i].weight, ops.PACK_IKF))
                           for i in (0, 3)) for b in res],
             "up": [(ops.weight_pack(c.weight, ops.PACK_FWD), ops.weight_pack(c.weight, ops.PACK_DGRAD))
                    for c, _ in up],
             "last": (ops.weight_pack(last.weight, ops.PACK_FWD), ops.weight_pack(last.weight, ops.PACK_DGRAD))}
        if TAP_LAST:  # 64 -> 3 output channels: tap GEMM on the matrix cores (ops.tap_conv_fwd)
            P["last_tap"] = ops.weight_pack(last.weight, ops.PACK_CK)
        if SG_PHASES:
            # the last layer's data gradient as a forward conv over the 4-channel dy (the direct 4-channel kernel,
            # ops.conv2d_dgrad_s1) and the Conv2d(k4, s2, p1) down convs' as phase convs (ops.conv4s2_dgrad),
            # instead of the generic transposed-conv gathers
            P["last_ikf"] = ops.weight_pack(last.weight, ops.PACK_IKF)
            P["down_ph"] = [ops.conv4s2_dgrad_phase_packs(c.weight) if k == 4 and st == 2 and pd == 1 else None
                            for c, _, k, st, pd in down]
            # the ConvTranspose2d(k4, s2, p1) forwards: the data gradient of a Conv2d with the same weight (read as
            # [out = Ci_t][in = Co_t]), i.e. its phase convs
            P["up_ph"] = [ops.conv4s2_dgrad_phase_packs(c.weight) for c, _ in up]
            # the first conv's data gradient onto the 3 image channels only (the label channels' is discarded):
            # the R x 1 tap conv + column sums of the 4-channel route (ops.tap_conv_dgrad_h)
            P["down0_sokd"] = ops.dgrad_sok_pack(down[0][0].weight, ci_real=3)
        return P

    def forward(self, x, c):
        """model.py:59-64: x [B,3,H,W], c [B,c_dim] -> [B,3,H,W]."""
        xc = _ConcatLabel.apply(x.float().contiguous(), c.float().contiguous().to(x.device))
        y = _StarGFn.apply(xc, self._anchor(), self)
        return _ToNCHW2.apply(y, 3)


class _ConcatLabel(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, c):
        ctx.cx = x.shape[1]
        return ops.concat_label_nhwc(x, c)

    @staticmethod
    def backward(ctx, g):
        return ops.nhwc_to_nchw(g.contiguous(), ctx.cx), None


def _in_stats(y, norm, training):
    if training:
        s = ops.instnorm_stats(y)
        ops.instnorm_running_update(s, norm.running_mean, norm.running_var, y.shape[1] * y.shape[2],
                                    norm.momentum)
        # (nn.InstanceNorm2d never advances num_batches_tracked: F.instance_norm leaves it at 0)
        return s
    return ops.instnorm_stats_from_running(norm.running_mean, norm.running_var, y.shape[0])


def _aff(norm):
    return norm.weight.detach(), norm.bias.detach()


class _StarGFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, net):
        P = net.packs()
        down, res, up, last = net._parts()
        role = "fwd" if any(ctx.needs_input_grad[:2]) else "infer"
        tr = net.training
        sv = {}
        a = x
        for i, (conv, norm, k, st, pad) in enumerate(down):
            y = ops.conv2d_fwd(a, P["down"][i][0], None, cpad(conv.weight.shape[0]), k, k, st, pad, "zero",
                               role=role)
            s = _in_stats(y, norm, tr)
            g, b = _aff(norm)
            an = ops.instnorm_affine_fwd(y, s, g, b, "relu")
            sv[("down", i)] = (a, y, s)
            a = an
        h = a
        for i, blk in enumerate(res):
            (ok1, _), (ok2, _) = P["res"][i]
            C = h.shape[-1]
            t = ops.conv2d_fwd(h, ok1, None, C, 3, 3, 1, 1, "zero", role=role)
            s1 = _in_stats(t, blk[1], tr)
            g1, b1 = _aff(blk[1])
            u = ops.instnorm_affine_fwd(t, s1, g1, b1, "relu")
            v = ops.conv2d_fwd(u, ok2, None, C, 3, 3, 1, 1, "zero", role=role)
            s2 = _in_stats(v, blk[4], tr)
            g2, b2 = _aff(blk[4])
            hn = ops.instnorm_affine_fwd(v, s2, g2, b2, "none", residual=h)
            sv[("res", i)] = (h, t, s1, u, v, s2)
            h = hn
        a = h
        for i, (conv, norm) in enumerate(up):
            _, ik = P["up"][i]
            cout = conv.weight.shape[1]
            if "up_ph" in P and a.shape[-1] % 32 == 0:  # ConvTranspose2d(k4, s2, p1) = the four 2x2 phase convs
                y = ops.conv4s2_dgrad(a, P["up_ph"][i], cpad(cout), role=role)
            else:
                y = ops.conv2d_tfwd(a, ik, None, 2 * a.shape[1], 2 * a.shape[2], cpad(cout), 4, 4, 2, 1, role=role)
            s = _in_stats(y, norm, tr)
            g, b = _aff(norm)
            an = ops.instnorm_affine_fwd(y, s, g, b, "relu")
            sv[("up", i)] = (a, y, s)
            a = an
        if "last_tap" in P:
            out = ops.tap_conv_fwd(a, P["last_tap"], None, 7, 3, "zero", act="tanh", role=role)
        else:
            out = ops.conv2d_fwd(a, P["last"][0], None, cpad(3), 7, 7, 1, 3, "zero", act="tanh", role=role)
        sv["last"] = (a, out)
        ctx.sv, ctx.net, ctx.P = sv, net, P
        ctx.train_w = anchor.requires_grad
        return out

    @staticmethod
    def backward(ctx, gout):
        sv, net, P = ctx.sv, ctx.net, ctx.P
        down, res, up, last = net._parts()
        tw = ctx.train_w

        def wgrad(mod, x, dy, k, st, pad):
            if tw:
                w = mod.weight
                ops.conv2d_wgrad(x, dy, w.grad, None, k, k, st, pad, "zero", w.shape[0], w.shape[1],
                                 w.shape[1] * k * k, k * k, accumulate=True)

        def in_bwd(g, y, s, norm, act):
            gm, bt = _aff(norm)
            kw = dict(dgamma=norm.weight.grad, dbeta=norm.bias.grad) if tw else {}
            return ops.instnorm_affine_bwd(g, y, s, gm, bt, act, accumulate=True, **kw)

        a, out = sv["last"]
        g = ops.act_bwd(gout.contiguous(), out, "tanh")
        if "last_tap" in P:
            if tw:
                ops.tap_conv_wgrad(a, g, last.weight.grad, 7, 3, "zero", accumulate=True)
        else:
            wgrad(last, a, g, 7, 1, 3)
        if "last_ikf" in P and g.shape[-1] == 4:
            g = ops.conv2d_dgrad_s1(g, P["last_ikf"], a.shape[1], a.shape[2], a.shape[-1], 7, 3, "zero")
        else:
            g = ops.conv2d_tfwd(g, P["last"][1], None, a.shape[1], a.shape[2], a.shape[-1], 7, 7, 1, 3)
        for i in (1, 0):
            conv, norm = up[i]
            a_in, y, s = sv[("up", i)]
            dy = in_bwd(g, y, s, norm, "relu")
            if tw:
                # ConvTranspose2d weight [Ci][Co][4][4]: the wgrad of the equivalent conv dy -> a_in
                ci_t, co_t = conv.weight.shape[0], conv.weight.shape[1]
                ops.conv2d_wgrad(dy, a_in, conv.weight.grad, None, 4, 4, 2, 1, "zero", ci_t, co_t, co_t * 16, 16,
                                 accumulate=True)
            g = ops.conv2d_fwd(dy, P["up"][i][0], None, a_in.shape[-1], 4, 4, 2, 1, "zero", role="bwd")
        gh = g
        for i in reversed(range(len(res))):
            blk = res[i]
            (_, ikf1), (_, ikf2) = P["res"][i]
            h, t, s1, u, v, s2 = sv[("res", i)]
            dv = in_bwd(gh, v, s2, blk[4], "none")
            wgrad(blk[3], u, dv, 3, 1, 1)
            du = ops.conv2d_dgrad_s1(dv, ikf2, u.shape[1], u.shape[2], u.shape[-1], 3, 1, "zero")
            dt = in_bwd(du, t, s1, blk[1], "relu")
            wgrad(blk[0], h, dt, 3, 1, 1)
            gh = ops.conv2d_dgrad_s1(dt, ikf1, h.shape[1], h.shape[2], h.shape[-1], 3, 1, "zero", addend=gh)
        g = gh
        gx = None
        for i in (2, 1, 0):
            conv, norm, k, st, pad = down[i]
            a_in, y, s = sv[("down", i)]
            dy = in_bwd(g, y, s, norm, "relu")
            wgrad(conv, a_in, dy, k, st, pad)
            if i > 0 or ctx.needs_input_grad[0]:
                ph = P["down_ph"][i] if "down_ph" in P else None
                if i == 0 and "down0_sokd" in P and k == 7 and st == 1 and dy.shape[-1] % 8 == 0:
                    g4 = ops.tap_conv_dgrad_h(dy, P["down0_sokd"], 7, pad, "zero")  # NHWC4: the 3 image channels
                    g = torch.zeros(a_in.shape, device=g4.device)  # (the label channels' gradient: zero, unused)
                    g[..., :4] = g4
                elif ph is not None and a_in.shape[1] == 2 * dy.shape[1] and a_in.shape[2] == 2 * dy.shape[2]:
                    g = ops.conv4s2_dgrad(dy, ph, a_in.shape[-1])
                else:
                    g = ops.conv2d_tfwd(dy, P["down"][i][1], None, a_in.shape[1], a_in.shape[2], a_in.shape[-1], k,
                                        k, st, pad)
                if i == 0:
                    gx = g
        ctx.sv = None
        return gx, None, None


###############################################################################
# Solver iteration (solver.py:187-199, 234-363)
###############################################################################
# Host tensors (labels, GP weights) onto the device through pinned memory, non-blocking; False: plain .to(device)
H2D_PINNED = True


def _h2d(t, device):
    """A small host tensor onto the device without blocking the host: a pageable host -> device copy waits for the
    whole stream to drain (every queued kernel) before it returns, so the host stops running ahead of the GPU and the
    launches after it arrive one by one; from pinned memory the copy is queued like a kernel."""
    device = torch.device(device)
    if not H2D_PINNED or t.device.type != "cpu" or device.type != "cuda":
        return t.to(device)
    return t.pin_memory().to(device, non_blocking=True)


def label2onehot(labels, dim, device):
    out = torch.zeros(labels.size(0), dim)
    out[np.arange(labels.size(0)), labels.long().cpu()] = 1
    return _h2d(out, device)


def classification_loss(logit, target, dataset="CelebA"):
    """solver.py:234-239."""
    if dataset == "CelebA":
        return F.binary_cross_entropy_with_logits(logit, target, reduction="sum") / logit.size(0)
    elif dataset == "RaFD":
        return F.cross_entropy(logit, target)
    raise NotImplementedError(dataset)


def gradient_penalty(y, x):
    """solver.py:187-199: mean over the batch of (||dy/dx||_2 - 1)^2, differentiable (create_graph)."""
    weight = torch.ones(y.size(), device=y.device)
    _INPUT_GRAD_ONLY[0] = True
    try:
        dydx = torch.autograd.grad(outputs=y, inputs=x, grad_outputs=weight, retain_graph=True, create_graph=True,
                                   only_inputs=True)[0]
    finally:
        _INPUT_GRAD_ONLY[0] = False
    dydx = dydx.view(dydx.size(0), -1)
    dydx_l2norm = torch.sqrt(torch.sum(dydx ** 2, dim=1))
    return torch.mean((dydx_l2norm - 1) ** 2)


@contextlib.contextmanager
def _params_frozen(net):
    ps = [p for p in net.parameters() if p.requires_grad and SG_DIRECT]
    for p in ps:
        p.requires_grad_(False)
    try:
        yield
    finally:
        for p in ps:
            p.requires_grad_(True)


class StarGANSolver:
    """The model/optimizer half of solver.py's Solver (build_model :125-140, train loop body
    :298-363, update_lr :170-175, reset_grad :177-180) on device-resident batches."""

    def __init__(self, image_size=256, c_dim=4, g_conv_dim=64, d_conv_dim=64, g_repeat_num=6, d_repeat_num=6,
                 lambda_cls=1.0, lambda_rec=10.0, lambda_gp=10.0, g_lr=1e-4, d_lr=1e-4, n_critic=5, beta1=0.5,
                 beta2=0.999, dataset="CelebA", device="cuda", grad_hook=None):
        """grad_hook(nets): called on [D] / [G] between backward and the optimizer step — the data-parallel
        gradient exchange (dp.GradExchange) plugs in here; each rank then runs on its own B_local."""
        self.device = torch.device(device)
        self.grad_hook = grad_hook
        self.c_dim, self.dataset, self.n_critic = c_dim, dataset, n_critic
        self.lambda_cls, self.lambda_rec, self.lambda_gp = lambda_cls, lambda_rec, lambda_gp
        self.G = Generator(g_conv_dim, c_dim, g_repeat_num).to(self.device)
        self.D = Discriminator(image_size, d_conv_dim, c_dim, d_repeat_num).to(self.device)
        self.g_optimizer = FusedAdam([self.G], lr=g_lr, betas=(beta1, beta2))
        self.d_optimizer = FusedAdam([self.D], lr=d_lr, betas=(beta1, beta2))
        self.i = 0

    def reset_grad(self):
        self.g_optimizer.zero_grad()
        self.d_optimizer.zero_grad()

    def update_lr(self, g_lr, d_lr):
        for pg in self.g_optimizer.param_groups:
            pg["lr"] = g_lr
        for pg in self.d_optimizer.param_groups:
            pg["lr"] = d_lr

    def train_step(self, x_real, label_org, label_trg, alpha=None):
        """One iteration of solver.py:298-363.  label_* are class indices [B]; alpha [B,1,1,1] (the
        gradient-penalty interpolation weights; torch.rand if None).  Returns the loss dict."""
        x_real = _h2d(x_real, self.device).float().contiguous()
        c_org = label2onehot(label_org, self.c_dim, self.device)
        c_trg = label2onehot(label_trg, self.c_dim, self.device)
        # 2. discriminator (real and fake through D as one batch: D is per-sample).  x_fake is only read detached, but
        # G runs with autograd as in the reference: its training-role arithmetic (the "mixed" policy computes
        # no-grad forwards at bf16x3) is what the reference's fp32 forward is matched against
        x_fake = self.G(x_real, c_trg)
        B = x_real.shape[0]
        out_src, out_cls = self.D(torch.cat([x_real, x_fake.detach()]))
        d_loss_real = -torch.mean(out_src[:B])
        d_loss_cls = classification_loss(out_cls[:B], c_org, self.dataset)
        d_loss_fake = torch.mean(out_src[B:])
        if alpha is None:
            alpha = torch.rand(x_real.size(0), 1, 1, 1)
        alpha = _h2d(alpha, self.device)
        x_hat = (alpha * x_real.data + (1 - alpha) * x_fake.data).requires_grad_(True)
        out_src, _ = self.D(x_hat)
        d_loss_gp = gradient_penalty(out_src, x_hat)
        d_loss = d_loss_real + d_loss_fake + self.lambda_cls * d_loss_cls + self.lambda_gp * d_loss_gp
        self.reset_grad()
        _ACCUM_PARAM_GRADS[0] = SG_DIRECT
        try:
            d_loss.backward()
        finally:
            _ACCUM_PARAM_GRADS[0] = False
        if self.grad_hook is not None:
            self.grad_hook([self.D])
        self.d_optimizer.step()
        loss = {"D/loss_real": d_loss_real.detach(), "D/loss_fake": d_loss_fake.detach(),
                "D/loss_cls": d_loss_cls.detach(), "D/loss_gp": d_loss_gp.detach()}
        # 3. generator
        if (self.i + 1) % self.n_critic == 0:
            x_fake = self.G(x_real, c_trg)
            # D's parameter gradients of the G step (the reference back-propagates into them) are zeroed by the
            # next reset_grad before anything reads them: D runs here with its parameters frozen
            with _params_frozen(self.D):
                out_src, out_cls = self.D(x_fake)
            g_loss_fake = -torch.mean(out_src)
            g_loss_cls = classification_loss(out_cls, c_trg, self.dataset)
            x_reconst = self.G(x_fake, c_org)
            g_loss_rec = torch.mean(torch.abs(x_real - x_reconst))
            g_loss = g_loss_fake + self.lambda_rec * g_loss_rec + self.lambda_cls * g_loss_cls
            self.reset_grad()
            g_loss.backward()
            if self.grad_hook is not None:
                self.grad_hook([self.G])
            self.g_optimizer.step()
            loss.update({"G/loss_fake": g_loss_fake.detach(), "G/loss_rec": g_loss_rec.detach(),
                         "G/loss_cls": g_loss_cls.detach()})
        self.i += 1
        return loss


from . import _lib as _lib_routes  # noqa: E402
_lib_routes.apply_route_overrides(__name__, globals())
