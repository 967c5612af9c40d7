"""Johnson fast-style transformer net and its perceptual-loss train step, HIP-backed.

Drop-in for methods/learning-based/network.py:80-298 (``FastStyleNet`` with ``ConvLayer``,
``ConvInstRelu``, ``UpsampleConvInstRelu``, ``ResidualBlock``, ``ConvTanh``; identical module tree
and state_dict keys, ``SelectiveLoadModule`` loading) and fs_johnson.py:5-52 (``Johnson`` train /
infer methods) on top of fast_style_transfer.py's loss helpers (perceptual.py).

MI355X design: the whole net is one autograd node over NHWC fp32 tensors —
  * reflect-padded convs (9x9, 3x3 s2, 3x3) on the implicit-GEMM MFMA kernels with the padding
    folded into the operand gather; stride-2 reflect data-gradients go through a padded buffer and
    the reflect-fold kernel;
  * affine InstanceNorm (+ReLU) with fp64 statistics, and the ResidualBlock's ``layer_strength``
    gate 2|s*l|/(1+|s*l|) and residual add fused into the normalise pass (gate gradient reduced in
    the same backward pass);
  * nearest 2x upsampling materialised by a streaming kernel (its backward sums 2x2 blocks);
  * ConvTanh's tanh(x/255)*150+127.5 as a streaming epilogue kernel.
Only ``n_styles == 1`` (plain InstanceNorm2d(affine=True)) is on the HIP path; the conditional
(embedding) norm of multi-style models raises NotImplementedError.
"""
import torch
import torch.nn as nn

from . import ops, perceptual
from .networks import Conv2d, FlatNet, _Marker, _ToNCHW, _ToNHWC, _pad_channels, _padded_bias
from .ops import cpad
from .optim import FusedAdam

# The 3x3 stride-1 data gradients (residual blocks, upsampling convs) as forward convs over the rotated taps on the
# split-bf16 kernel with the reflect border GEMM (ops.conv2d_dgrad_s1, the generator's route) instead of the
# transposed conv on the fp32-operand kernel; False keeps the latter
FS_DGRAD_FPROP = True
# The 9x9 32 -> 3 output layer on the tap routes of the generator's 7x7 output layer: forward as the 1x1 conv into
# (tap, co) channels + the tap sum (ops.tap_conv_fwd), weight gradient as the swapped GEMM (tap_conv_wgrad_swap),
# data gradient as the forward conv of the 8-channel-padded dy over the rotated taps + reflect fold; instead of the
# VALU skinny kernels and the fp32-operand transposed conv.  False keeps those.
FS_TAP = True
# The loss network's two forwards (styled image, content image) as one batch (perceptual._VggMultiFn);
# False: two calls
VGG_BATCHED = True


class InstanceNormAffine(nn.Module):
    """Parameter holder with nn.InstanceNorm2d(affine=True)'s state (weight=1, bias=0)."""

    def __init__(self, c):
        super().__init__()
        self.num_features = c
        self.weight = nn.Parameter(torch.ones(c))
        self.bias = nn.Parameter(torch.zeros(c))

    def extra_repr(self):
        return f"{self.num_features}, eps=1e-05, affine=True"


class ConvLayer(nn.Module):
    """network.py:95-107: ReflectionPad2d(k//2) + Conv2d(stride)."""

    def __init__(self, cin, cout, kernel_size, stride, bias=True):
        super().__init__()
        k = kernel_size
        self.reflection_pad = _Marker("ReflectionPad2d(%d)" % (k // 2))
        self.conv2d = Conv2d(cin, cout, k, stride=stride, bias=bias)
        self.k, self.stride = k, stride


class ConvTanh(ConvLayer):
    """network.py:110-118: tanh(conv(x)/255)*150 + 255/2."""

    def __init__(self, cin, cout, kernel_size, stride):
        super().__init__(cin, cout, kernel_size, stride)
        self.tanh = _Marker("Tanh")


class ConvInstRelu(ConvLayer):
    """network.py:146-170 (n_styles == 1)."""

    def __init__(self, cin, cout, kernel_size, stride, n_styles=1):
        super().__init__(cin, cout, kernel_size, stride)
        if n_styles != 1:
            raise NotImplementedError("conditional instance norm (n_styles > 1) is not on the HIP path")
        self.n_styles = n_styles
        self.instance = InstanceNormAffine(cout)
        self.relu = _Marker("ReLU")


class UpsampleConvInstRelu(nn.Module):
    """network.py:173-217: nearest upsample x2, ReflectionPad2d(k//2), conv, IN(affine), ReLU."""

    def __init__(self, cin, cout, kernel_size, stride, upsample=None, n_styles=1):
        super().__init__()
        k = kernel_size
        if n_styles != 1:
            raise NotImplementedError("conditional instance norm (n_styles > 1) is not on the HIP path")
        if upsample not in (None, 2) or stride != 1:
            raise NotImplementedError("UpsampleConvInstRelu: upsample 2 / stride 1 only on the HIP path")
        self.upsample = upsample
        self.reflection_pad = _Marker("ReflectionPad2d(%d)" % (k // 2))
        self.conv2d = Conv2d(cin, cout, k, stride=stride)
        self.n_styles = n_styles
        self.instance = InstanceNormAffine(cout)
        self.relu = _Marker("ReLU")
        self.k, self.stride = k, stride


class ResidualBlock(nn.Module):
    """network.py:219-261: x + strength * IN2(conv2(relu(IN1(conv1(x))))),
    strength = 2|s*layer_strength| / (1 + |s*layer_strength|)."""

    def __init__(self, cin, cout, kernel_size=3, stride=1, n_styles=1):
        super().__init__()
        self.conv1 = ConvLayer(cin, cout, kernel_size, stride)
        self.in1 = InstanceNormAffine(cout)
        self.in2 = InstanceNormAffine(cout)
        self.conv2 = ConvLayer(cout, cout, kernel_size, stride)
        self.relu = _Marker("ReLU")
        self.layer_strength = nn.Parameter(torch.tensor([1], dtype=torch.float32))


class FastStyleNet(FlatNet):
    """network.py:263-298.  forward(x, style_strength=1.0, s_id=0) -> (features, image), NCHW;
    x is the [0, 1] image (3 channels, or 7 for the ReCoNet-style stacked input)."""

    def __init__(self, num_inp, n_styles=1):
        super().__init__()
        self.input_nc, self.output_nc = num_inp, 3
        self.conv1 = ConvInstRelu(num_inp, 32, kernel_size=9, stride=1, n_styles=n_styles)
        self.conv2 = ConvInstRelu(32, 64, kernel_size=3, stride=2, n_styles=n_styles)
        self.conv3 = ConvInstRelu(64, 128, kernel_size=3, stride=2, n_styles=n_styles)
        self.res1 = ResidualBlock(128, 128, n_styles=n_styles)
        self.res2 = ResidualBlock(128, 128, n_styles=n_styles)
        self.res3 = ResidualBlock(128, 128, n_styles=n_styles)
        self.res4 = ResidualBlock(128, 128, n_styles=n_styles)
        self.res5 = ResidualBlock(128, 128, n_styles=n_styles)
        self.deconv1 = UpsampleConvInstRelu(128, 64, kernel_size=3, stride=1, upsample=2, n_styles=n_styles)
        self.deconv2 = UpsampleConvInstRelu(64, 32, kernel_size=3, stride=1, upsample=2, n_styles=n_styles)
        self.deconv3 = ConvTanh(32, 3, kernel_size=9, stride=1)
        self._init_torch_default()
        self._flatten()

    def _init_torch_default(self):
        """nn.Conv2d's default init (kaiming_uniform a=sqrt(5), bias U(+-1/sqrt(fan_in)))."""
        for m in self.modules():
            if isinstance(m, Conv2d):
                nn.init.kaiming_uniform_(m.weight, a=5 ** 0.5)
                fan_in = m.weight.shape[1] * m.weight.shape[2] * m.weight.shape[3]
                nn.init.uniform_(m.bias, -1 / fan_in ** 0.5, 1 / fan_in ** 0.5)

    def load_state_dict(self, state_dict, strict=False):
        """SelectiveLoadModule.load_state_dict (network.py:82-92): copy only the names we own."""
        own = self.state_dict()
        with torch.no_grad():
            for name, param in state_dict.items():
                if name in own:
                    own[name].copy_(param)
        self.bump_version()

    def blocks(self):
        return [self.res1, self.res2, self.res3, self.res4, self.res5]

    def _make_packs(self):
        P = {}
        for name, m in self.named_modules():
            if isinstance(m, Conv2d):
                # + the rotated pack of the 3x3 stride-1 layers' data gradient as a forward conv (conv2d_dgrad_s1)
                s1 = m.kernel_size == 3 and m.stride == 1
                P[name] = (ops.weight_pack(m.weight, ops.PACK_FWD), ops.weight_pack(m.weight, ops.PACK_DGRAD),
                           _padded_bias(m), ops.weight_pack(m.weight, ops.PACK_IKF) if s1 else None)
        if FS_TAP:  # the output layer's (CK pack of the tap forward, 8-output IKF pack of its data gradient)
            w = self.deconv3.conv2d.weight
            P["deconv3.tap"] = (ops.weight_pack(w, ops.PACK_CK), ops.weight_pack(w, ops.PACK_IKF, Op=8))
        return P

    def forward_nhwc(self, x, style_strength=1.0):
        return _FastStyleFn.apply(x, self._anchor(), self, float(style_strength))

    def forward(self, x, style_strength=1.0, s_id=0):
        feats, img = self.forward_nhwc(_ToNHWC.apply(x, cpad(self.input_nc)), style_strength)
        return _ToNCHW.apply(feats, 128), _ToNCHW.apply(img, 3)


def _aff(mod):
    return mod.weight.detach(), mod.bias.detach()


class _FastStyleFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, net, strength):
        ctx.set_materialize_grads(False)
        P = net.packs()
        role = "fwd" if any(ctx.needs_input_grad[:2]) else "infer"
        sv = {"x": x}

        def conv(inp, key, cout, k, st):
            kc, _, b, _ = P[key]
            return ops.conv2d_fwd(inp, kc, b, cpad(cout), k, k, st, k // 2, "reflect", role=role)

        def cir(inp, layer, key, cout, k, st):
            y = conv(inp, key, cout, k, st)
            s = ops.instnorm_stats(y)
            g, b = _aff(layer.instance)
            return y, s, ops.instnorm_affine_fwd(y, s, g, b, "relu")

        a = x
        for name, cout, k, st in (("conv1", 32, 9, 1), ("conv2", 64, 3, 2), ("conv3", 128, 3, 2)):
            y, s, an = cir(a, getattr(net, name), name + ".conv2d", cout, k, st)
            sv[name] = (a, y, s)
            a = an
        h = a
        for i, blk in enumerate(net.blocks()):
            key = "res%d" % (i + 1)
            t = conv(h, key + ".conv1.conv2d", 128, 3, 1)
            s1 = ops.instnorm_stats(t)
            g1, b1 = _aff(blk.in1)
            u = ops.instnorm_affine_fwd(t, s1, g1, b1, "relu")
            v = conv(u, key + ".conv2.conv2d", 128, 3, 1)
            s2 = ops.instnorm_stats(v)
            g2, b2 = _aff(blk.in2)
            hn = ops.instnorm_affine_fwd(v, s2, g2, b2, "none", gate=blk.layer_strength.detach(),
                                         gate_mult=strength, residual=h)
            sv[key] = (h, t, s1, u, v, s2)
            h = hn
        feats = h
        a = h
        for name, cout in (("deconv1", 64), ("deconv2", 32)):
            up = ops.upsample2x(a)
            y, s, an = cir(up, getattr(net, name), name + ".conv2d", cout, 3, 1)
            sv[name] = (up, y, s)
            a = an
        if "deconv3.tap" in P:
            y = ops.tap_conv_fwd(a, P["deconv3.tap"][0], P["deconv3.conv2d"][2], 9, 4, "reflect", role=role)
        else:
            y = conv(a, "deconv3.conv2d", 3, 9, 1)
        out = ops.scaled_tanh(y, 3)
        sv["deconv3"] = (a, y)
        ctx.sv, ctx.net, ctx.P, ctx.strength = sv, net, P, strength
        ctx.train_w = anchor.requires_grad
        return feats, out

    @staticmethod
    def backward(ctx, gfeat, gout):
        sv, net, P, strength = ctx.sv, ctx.net, ctx.P, ctx.strength
        train_w = ctx.train_w

        def wgrad(mod, inp, dy, k, st, db=False):
            if not train_w:
                return
            w = mod.weight
            co, ci = w.shape[0], w.shape[1]
            ops.conv2d_wgrad(inp, dy, w.grad, mod.bias.grad if db else None, k, k, st, k // 2, "reflect",
                             co, ci, ci * k * k, k * k, accumulate=True)

        def dgrad(dy, key, xin, k, st, addend=None):
            _, ck, _, ikf = P[key]
            N, H, W, C = xin.shape
            p = k // 2
            if st == 1 and ikf is not None and FS_DGRAD_FPROP:  # interior conv + border GEMM (the generator's route)
                return ops.conv2d_dgrad_s1(dy, ikf, H, W, C, k, p, "reflect", addend=addend)
            if st == 1:
                return ops.conv2d_tfwd(dy, ck, None, H, W, C, k, k, 1, p, pad_mode="reflect", addend=addend)
            # strided reflect conv: data gradient of the valid conv into the padded frame, then fold
            dxp = ops.conv2d_tfwd(dy, ck, None, H + 2 * p, W + 2 * p, C, k, k, st, 0)
            return ops.reflect_fold(dxp, p, addend)

        def in_bwd(g, y, s, layer, conv_mod, act, gate=None):
            gam, bet = _aff(layer)
            kw = {}
            if train_w:
                kw = dict(dgamma=layer.weight.grad, dbeta=layer.bias.grad, dbias=conv_mod.bias.grad)
                if gate is not None:
                    kw["dgate"] = gate.grad
            return ops.instnorm_affine_bwd(g, y, s, gam, bet, act, gate=None if gate is None else gate.detach(),
                                           gate_mult=strength, accumulate=True, **kw)

        g = None
        if gout is not None:
            a, y = sv["deconv3"]
            gy = ops.scaled_tanh_bwd(y, gout.contiguous(), 3)
            m = net.deconv3.conv2d
            tap = P.get("deconv3.tap")
            if tap is not None and train_w and ops.tap_conv_wgrad_swap_ok(a, 9, 4, "reflect", co=m.weight.shape[0]):
                ops.tap_conv_wgrad_swap(a, gy, m.weight.grad, 9, 4, "reflect", accumulate=True, db=m.bias.grad)
            else:
                wgrad(m, a, gy, 9, 1, db=True)
            if tap is not None:
                gp = _pad_channels(gy, 8)
                gp.vst_real_c = 3  # (tools/convflops: the MACs of the 3 real channels)
                g = ops.conv2d_dgrad_s1(gp, tap[1], a.shape[1], a.shape[2], a.shape[-1], 9, 4, "reflect")
            else:
                g = dgrad(gy, "deconv3.conv2d", a, 9, 1)
            for name in ("deconv2", "deconv1"):
                up, y, s = sv[name]
                layer = getattr(net, name)
                dy = in_bwd(g, y, s, layer.instance, layer.conv2d, "relu")
                wgrad(layer.conv2d, up, dy, 3, 1)
                g = ops.upsample2x_bwd(dgrad(dy, name + ".conv2d", up, 3, 1))
        if gfeat is not None:
            gfeat = gfeat.contiguous()
            if g is None:
                g = gfeat.clone()
            else:
                ops.axpby(gfeat, g, 1.0, 1.0)
        if g is None:
            return None, None, None, None
        gh = g
        for i in reversed(range(5)):
            blk = net.blocks()[i]
            key = "res%d" % (i + 1)
            h, t, s1, u, v, s2 = sv[key]
            dv = in_bwd(gh, v, s2, blk.in2, blk.conv2.conv2d, "none", gate=blk.layer_strength)
            wgrad(blk.conv2.conv2d, u, dv, 3, 1)
            du = dgrad(dv, key + ".conv2.conv2d", u, 3, 1)
            dt = in_bwd(du, t, s1, blk.in1, blk.conv1.conv2d, "relu")
            wgrad(blk.conv1.conv2d, h, dt, 3, 1)
            gh = dgrad(dt, key + ".conv1.conv2d", h, 3, 1, addend=gh)
        g = gh
        gx = None
        for name, k, st in (("conv3", 3, 2), ("conv2", 3, 2), ("conv1", 9, 1)):
            a_in, y, s = sv[name]
            layer = getattr(net, name)
            dy = in_bwd(g, y, s, layer.instance, layer.conv2d, "relu")
            wgrad(layer.conv2d, a_in, dy, k, st)
            if name != "conv1":
                g = dgrad(dy, name + ".conv2d", a_in, k, st)
            elif ctx.needs_input_grad[0]:
                gx = dgrad(dy, name + ".conv2d", a_in, k, st)
        ctx.sv = None
        return gx, None, None, None


class Johnson:
    """fs_johnson.py:5-52 Johnson method + the FastStyle training plumbing it relies on
    (fast_style_transfer.py:226-248 Adam loop, 762-793 prep_training/prep_adam, 741-756 style
    Grams), on device-resident batches.

    ``train_step(img)`` = prep_adam + train_method + adam.step for one [B,3,H,W] batch in [0,1];
    returns (loss, content, style, tv) as device scalars and the styled image (NHWC4, 0..255)."""

    def __init__(self, style_imgs, emphasis=(1.0, 1e5, 1e-6), lr=1e-3, batch_sz=16, device="cuda",
                 vgg=None, model=None):
        self.device = torch.device(device)
        self.model = model if model is not None else FastStyleNet(3, 1).to(self.device)
        self.vgg = vgg if vgg is not None else perceptual.Vgg16(self.device)
        self.adam = FusedAdam([self.model], lr=lr)
        self.batch_sz = batch_sz
        self.alpha, self.beta, self.delta = emphasis
        # loadStyles: normalize -> VGG -> gram per level, one style (n_styles == 1)
        self.styles = [perceptual.style_grams(self.vgg, s.to(self.device)) for s in style_imgs]
        self._gram_cache = {}
        self.itr = 0

    def _style_targets(self, B):
        if B not in self._gram_cache:
            # broadcast of the [1, C, C] style Gram against the batch's [B, C, C] (fs_johnson.py:41)
            self._gram_cache[B] = [g.expand(B, -1, -1).contiguous() for g in self.styles[0]]
        return self._gram_cache[B]

    def prep_adam(self, itr):
        """fast_style_transfer.py:788-793: zero grads; lr /= 1.2 every 500/batch_sz iterations."""
        self.adam.zero_grad()
        if (itr + 1) % int(500 / self.batch_sz) == 0:
            for pg in self.adam.param_groups:
                pg["lr"] = max(pg["lr"] / 1.2, 1e-4)

    def losses_nhwc(self, img_nhwc):
        """train_method's loss graph on an NHWC4 [0,1] image batch -> (loss, cl, sl, tv, styled)."""
        _, styled = self.model.forward_nhwc(img_nhwc)
        if VGG_BATCHED:  # styled (differentiated) and the content image through the VGG as one batch, the content
            # image through the slices its loss reads only (relu3_3)
            with torch.no_grad():
                xc = perceptual.normalize_nhwc(img_nhwc)
            styled_f, img_f = self.vgg.forward_multi_nhwc([perceptual.normalize_nhwc(styled, d0=255.0), xc],
                                                          [len(self.vgg.slices_idx), 3])
        else:
            styled_f = self.vgg.forward_nhwc(perceptual.normalize_nhwc(styled, d0=255.0))
            with torch.no_grad():
                img_f = self.vgg.forward_nhwc(perceptual.normalize_nhwc(img_nhwc))
        content = perceptual.mse_loss(styled_f[2], img_f[2], self.alpha)
        grams = self._style_targets(img_nhwc.shape[0])
        style = None
        for f, gs in zip(styled_f, grams):
            t = perceptual.mse_loss(perceptual.gram_nhwc(f), gs, self.beta)
            style = t if style is None else style + t
        # calc_tv_loss(styled / 255) == calc_tv_loss(styled) / 255 (positively homogeneous)
        tv = perceptual.tv_loss_nhwc(styled, self.delta / 255.0, 3)
        loss = content + style + tv
        return loss, content, style, tv, styled

    def train_step(self, img):
        self.prep_adam(self.itr)
        x = ops.nchw_to_nhwc(img.to(self.device).float().contiguous())
        loss, cl, sl, tv, styled = self.losses_nhwc(x)
        loss.backward()
        self.adam.step()
        self.itr += 1
        return (loss.detach(), cl.detach(), sl.detach(), tv.detach()), styled

    @torch.no_grad()
    def infer_method(self, frame):
        """fs_johnson.py:50-52: styled frame / 255."""
        _, styled = self.model(frame.to(self.device).float())
        return styled / 255.0


from . import _lib as _lib_routes  # noqa: E402
_lib_routes.apply_route_overrides(__name__, globals())
