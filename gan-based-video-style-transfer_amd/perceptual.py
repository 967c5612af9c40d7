"""VGG perceptual networks and the Gram / content / TV style losses, HIP-backed.

Drop-in for methods/learning-based/network.py:10-78 (``Vgg16`` relu1_2..relu4_3, ``Vgg19``
relu1_1..relu5_1, namedtuple outputs) and fast_style_transfer.py:795-822 (``calc_tv_loss``,
``gram_matrix``, ``normalize``) plus the loss composition of fs_johnson.py:35-47.

MI355X design:
  * The VGG feature stack (3x3 zero-pad convs + ReLU epilogue, 2x2 max pools) runs as ONE autograd
    node on NHWC fp32 tensors: convs on the implicit-GEMM MFMA kernels (ReLU fused in the
    epilogue), max pool / its argmax-routed backward on HBM-streaming kernels.  The reference
    freezes VGG (``requires_grad = False``) so the backward is data-gradient only (no wgrad).
  * ``gram`` is the split-K MFMA weight-gradient kernel of a 1x1 conv with x = dy = F (fixed-order,
    deterministic); its backward is a 1x1 conv with weight (dG + dG^T) / hw.
  * Pretrained torchvision weights cannot be fetched offline: the modules initialise like
    torchvision's VGG (kaiming-normal fan_out, zero bias) from a seed and accept
    ``load_torchvision_features`` / ``load_state_dict`` for real weights.
"""
import os
from collections import namedtuple

import torch
import torch.nn as nn

from . import ops
from .networks import Conv2d, FlatNet, _Marker, _ToNCHW, _ToNHWC
from .ops import cpad

VGG_CFG = {
    "vgg16": [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"],
    "vgg19": [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M",
              512, 512, 512, 512, "M"],
}
# slice boundaries in torchvision `features` indices (network.py:17-28 and 52-67)
VGG_SLICES = {"vgg16": [(0, 4), (4, 9), (9, 16), (16, 23)],
              "vgg19": [(0, 2), (2, 7), (7, 12), (12, 21), (21, 30)]}
VGG_NAMES = {"vgg16": ["relu1_2", "relu2_2", "relu3_3", "relu4_3"],
             "vgg19": ["relu1_1", "relu2_1", "relu3_1", "relu4_1", "relu5_1"]}
VGG16_MEAN = [0.485, 0.456, 0.406]   # fast_style_transfer.py:174-175
VGG16_STD = [0.229, 0.224, 0.225]


def _features(cfg):
    """torchvision VGG `features` as (kind, cin, cout) per index: 'conv' / 'relu' / 'pool'."""
    out, cin = [], 3
    for v in cfg:
        if v == "M":
            out.append(("pool", cin, cin))
        else:
            out.append(("conv", cin, v))
            out.append(("relu", v, v))
            cin = v
    return out


# VGG data gradients (3x3, zero pad 1) as forward convs over the rotated taps on the split-bf16 kernel (the
# generator's route) instead of the transposed conv on the fp32-operand kernel; False keeps the latter
VGG_DGRAD_FPROP = True


class _VGG(FlatNet):
    def __init__(self, arch, device=None, seed=0):
        super().__init__()
        self.arch = arch
        feats = _features(VGG_CFG[arch])
        self.slices_idx = VGG_SLICES[arch]
        self.layers = []  # (feature index, kind, cin, cout, module or None)
        for k, (a, b) in enumerate(self.slices_idx):
            seq = nn.Sequential()
            for x in range(a, b):
                kind, cin, cout = feats[x]
                m = Conv2d(cin, cout, 3, padding=1) if kind == "conv" else \
                    _Marker("ReLU(inplace=True)" if kind == "relu" else "MaxPool2d(2, 2)")
                seq.add_module(str(x), m)
                self.layers.append((x, kind, cin, cout, m if kind == "conv" else None))
            setattr(self, "slice%d" % (k + 1), seq)
        self.input_nc = 3
        g = torch.Generator().manual_seed(seed)
        for _, kind, cin, cout, m in self.layers:
            if kind == "conv":
                with torch.no_grad():
                    # torchvision VGG init: kaiming_normal_(fan_out, relu), bias 0
                    std = (2.0 / (cout * 9)) ** 0.5
                    m.weight.copy_(torch.randn(m.weight.shape, generator=g) * std)
                    m.bias.zero_()
        for p in self.parameters():
            p.requires_grad = False
        self._flatten()
        if device is not None:
            self.to(device)

    def load_torchvision_features(self, sd):
        """Load a torchvision ``vgg16/vgg19().features`` state dict ('N.weight', 'features.N.weight' or
        either under a DataParallel 'module.' prefix).  Every conv weight and bias of the sliced net
        must be present: a dict that maps none or only some of them (another architecture, a
        classifier-only dict) raises instead of leaving the seeded weights in place."""
        own = {}
        for k, (a, b) in enumerate(self.slices_idx):
            for x in range(a, b):
                own[str(x)] = "slice%d.%d" % (k + 1, x)
        mapped = {}
        for key, v in sd.items():
            for pre in ("module.", "features."):
                key = key[len(pre):] if key.startswith(pre) else key
            idx, _, name = key.partition(".")
            if idx in own and name in ("weight", "bias"):
                mapped[own[idx] + "." + name] = v
        expected = [n for n, _ in self.named_parameters()]
        missing = [n for n in expected if n not in mapped]
        if missing:
            raise KeyError("VGG state dict lacks %d of %d conv tensors (first: %s)" % (len(missing), len(expected),
                                                                                      missing[0]))
        self.load_state_dict(mapped, strict=True)
        self.bump_version()

    def _make_packs(self):
        P = {}
        for x, kind, cin, cout, m in self.layers:
            if kind == "conv":
                # forward pack, transposed pack (the 3-channel first layer's data gradient), bias, and the
                # rotated pack of the data gradient as a forward conv on the split-bf16 kernel (conv2d_dgrad_s1)
                P[x] = (ops.weight_pack(m.weight, ops.PACK_FWD), ops.weight_pack(m.weight, ops.PACK_DGRAD),
                        m.bias.detach(), ops.weight_pack(m.weight, ops.PACK_IKF) if cin > 4 else None)
        return P

    def forward_nhwc(self, x):
        """x: NHWC4 normalised image -> tuple of NHWC slice outputs."""
        return _VggFn.apply(x, self)

    def forward_multi_nhwc(self, xs, levels):
        """Images xs (NHWC4, normalised; the first one differentiable) through the net as one batch, xs[k] through its
        first levels[k] slices (non-increasing) -> a list per image of its slice outputs (_VggMultiFn)."""
        flat = _VggMultiFn.apply(xs[0], self, tuple(levels), *xs[1:])
        out, off = [], 0
        for n in levels:
            out.append(flat[off:off + n])
            off += n
        return out

    def forward(self, X):
        outs = self.forward_nhwc(_ToNHWC.apply(X, cpad(3)))
        names = VGG_NAMES[self.arch]
        nt = namedtuple("VggOutputs", names)
        return nt(*[_ToNCHW.apply(o, o.shape[-1]) for o in outs])


class Vgg16(_VGG):
    """network.py:10-43 (outputs relu1_2, relu2_2, relu3_3, relu4_3)."""

    def __init__(self, device=None, seed=0):
        super().__init__("vgg16", device, seed)


class Vgg19(_VGG):
    """network.py:45-78 (outputs relu1_1, relu2_1, relu3_1, relu4_1, relu5_1)."""

    def __init__(self, device=None, seed=0):
        super().__init__("vgg19", device, seed)


class _VggFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, net):
        if any(p.requires_grad for p in net.parameters()):
            raise NotImplementedError("VGG weights are frozen on the HIP path (network.py:30-31, 69-70)")
        ctx.set_materialize_grads(False)
        P = net.packs()
        role = "fwd" if ctx.needs_input_grad[0] else "infer"
        acts = [x]       # acts[i] = activation entering layer i
        outs = []
        a = x
        ends = {b - 1 for _, b in net.slices_idx}
        for x_idx, kind, cin, cout, m in net.layers:
            if kind == "conv":
                kc, _, b, _ = P[x_idx]
                # the ReLU at x_idx + 1 is fused into the conv epilogue
                a = ops.conv2d_fwd(a, kc, b, cpad(cout), 3, 3, 1, 1, "zero", act="relu", role=role)
            elif kind == "pool":
                a = ops.maxpool2(a)
            acts.append(a)
            if x_idx in ends:
                outs.append(a)
        ctx.acts, ctx.net, ctx.P = acts, net, P
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gouts):
        g = _vgg_backward(ctx.acts, ctx.net, ctx.P, gouts, ctx.needs_input_grad[0])
        ctx.acts = None
        return g, None


def _vgg_backward(acts, net, P, gouts, need_x, B0=None):
    """The input gradient from the slice outputs' gradients (None = no gradient); B0: the activations hold a
    larger batch whose first B0 images are the differentiated ones (_VggMultiFn)."""
    cut = (lambda t: t[:B0]) if B0 is not None else (lambda t: t)
    ends = [b - 1 for _, b in net.slices_idx]
    gmap = {e: g for e, g in zip(ends, gouts)}
    g = None
    for i in reversed(range(len(net.layers))):
        x_idx, kind, cin, cout, m = net.layers[i]
        go = gmap.get(x_idx)
        if go is not None:
            go = go.contiguous()
            if g is None:
                g = go.clone()
            else:
                ops.axpby(go, g, 1.0, 1.0)
        if g is None:
            continue
        if kind == "relu":
            # acts[i + 1] is the fused conv+ReLU output
            g = ops.act_bwd(g, cut(acts[i + 1]), "relu")
        elif kind == "conv":
            if i == 0 and not need_x:
                return None
            xin = acts[i]
            _, ck, _, ikf = P[x_idx]
            if ikf is not None and VGG_DGRAD_FPROP:
                g = ops.conv2d_dgrad_s1(g, ikf, xin.shape[1], xin.shape[2], xin.shape[-1], 3, 1, "zero")
            else:
                g = ops.conv2d_tfwd(g, ck, None, xin.shape[1], xin.shape[2], xin.shape[-1], 3, 3, 1, 1)
        else:
            g = ops.maxpool2_bwd(g, cut(acts[i]))
    return g


class _VggMultiFn(torch.autograd.Function):
    """Several NHWC4 images through the VGG as ONE batch (the perceptual losses: the differentiated image first, then
    the no-grad targets), image k through its first levels[k] slices only: the inputs are ordered by non-increasing
    levels, so the images a slice no longer needs are cut from the end of the batch (a contiguous prefix stays).
    Per-image arithmetic is the separate calls' (every layer is per sample); only the GEMM plans see a larger M.
    Returns the first image's slice outputs, then each other image's (detached copies)."""

    @staticmethod
    def forward(ctx, x0, net, levels, *rest):
        if any(p.requires_grad for p in net.parameters()):
            raise NotImplementedError("VGG weights are frozen on the HIP path (network.py:30-31, 69-70)")
        ins = (x0,) + rest
        if len(levels) != len(ins) or any(levels[k] < levels[k + 1] for k in range(len(ins) - 1)):
            raise ValueError("_VggMultiFn: one level count per image, non-increasing")
        ctx.set_materialize_grads(False)
        P = net.packs()
        role = "fwd" if ctx.needs_input_grad[0] else "infer"
        Bs = [t.shape[0] for t in ins]
        a = torch.cat([t.contiguous() for t in ins]) if len(ins) > 1 else x0
        acts = [a]
        ends = [b - 1 for _, b in net.slices_idx]
        outs = [[] for _ in ins]
        live = len(ins)
        for x_idx, kind, cin, cout, m in net.layers:
            if kind == "conv":
                kc, _, b, _ = P[x_idx]
                a = ops.conv2d_fwd(a, kc, b, cpad(cout), 3, 3, 1, 1, "zero", act="relu", role=role)
            elif kind == "pool":
                a = ops.maxpool2(a)
            acts.append(a)
            if x_idx in ends:
                lvl = ends.index(x_idx) + 1
                off = 0
                for k in range(live):
                    outs[k].append(a[off:off + Bs[k]])
                    off += Bs[k]
                if lvl == levels[0]:
                    break
                while live > 1 and levels[live - 1] == lvl:
                    live -= 1
                a = a[:sum(Bs[:live])]
        rest_outs = [o.clone() for k in range(1, len(ins)) for o in outs[k]]
        ctx.mark_non_differentiable(*rest_outs)
        ctx.acts, ctx.net, ctx.P, ctx.B0, ctx.n0, ctx.nrest = acts, net, P, Bs[0], len(outs[0]), len(rest)
        return tuple(outs[0]) + tuple(rest_outs)

    @staticmethod
    def backward(ctx, *gouts):
        g = _vgg_backward(ctx.acts, ctx.net, ctx.P, gouts[:ctx.n0], ctx.needs_input_grad[0], ctx.B0)
        ctx.acts = None
        return (g, None, None) + (None,) * ctx.nrest


# ------------------------------------------------------------------------------------ losses
class _GramFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, f):
        ctx.save_for_backward(f)
        return ops.gram(f, role="fwd" if ctx.needs_input_grad[0] else "infer")

    @staticmethod
    def backward(ctx, dG):
        (f,) = ctx.saved_tensors
        return ops.gram_bwd(f, dG.contiguous())


def gram_nhwc(f):
    """G[b] = F_b^T F_b / (h*w) of NHWC features (channel stride = logical channels)."""
    return _GramFn.apply(f)


def gram_matrix(inp):
    """fast_style_transfer.py:813-817 on NCHW input: bmm(F, F^T) / (h*w)."""
    b, c, h, w = inp.size()
    if c % 4:
        raise NotImplementedError("gram_matrix: channel count must be a multiple of 4 on the HIP path")
    return gram_nhwc(_ToNHWC.apply(inp, c))


class _NormalizeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, img, mean, std, d0, cl):
        ctx.std, ctx.d0, ctx.cl = std, d0, cl
        return ops.channel_normalize(img, mean, std, d0, cl)

    @staticmethod
    def backward(ctx, g):
        return ops.channel_normalize(g.contiguous(), None, ctx.std, ctx.d0, ctx.cl, backward=True), \
            None, None, None, None


_NORM_CACHE = {}


def _mean_std(device):
    key = str(device)
    if key not in _NORM_CACHE:
        _NORM_CACHE[key] = (torch.tensor(VGG16_MEAN, device=device), torch.tensor(VGG16_STD, device=device))
    return _NORM_CACHE[key]


def normalize_nhwc(img, d0=1.0):
    """((img / d0) - mean) / std on NHWC4 images (fast_style_transfer.py:819-822; d0 = 255 folds the
    fs_johnson.py:31 ``styled_img1 /= 255.0`` into the same pass)."""
    mean, std = _mean_std(img.device)
    return _NormalizeFn.apply(img, mean, std, float(d0), 3)


def normalize(img):
    """NCHW drop-in of fast_style_transfer.py:819-822."""
    return _ToNCHW.apply(normalize_nhwc(_ToNHWC.apply(img, cpad(3))), 3)


class _MSEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, scale, cl):
        ctx.save_for_backward(a, b)
        ctx.scale, ctx.cl = scale, cl
        return ops.loss_mse(a, b, scale, cl)

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        g = g.contiguous()
        ga = ops.loss_mse_bwd(a, b, g, ctx.scale, ctx.cl) if ctx.needs_input_grad[0] else None
        gb = ops.loss_mse_bwd(b, a, g, ctx.scale, ctx.cl) if ctx.needs_input_grad[1] else None
        return ga, gb, None, None


def mse_loss(a, b, scale=1.0, cl=None):
    """scale * nn.MSELoss()(a, b) over the cl logical channels of NHWC tensors (or [B, C, C] Grams)."""
    return _MSEFn.apply(a.contiguous(), b.contiguous(), float(scale), cl)


class _TVFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, img, scale, cl):
        ctx.save_for_backward(img)
        ctx.scale, ctx.cl = scale, cl
        return ops.loss_tv(img, scale, cl)

    @staticmethod
    def backward(ctx, g):
        (img,) = ctx.saved_tensors
        return ops.loss_tv_bwd(img, g.contiguous(), ctx.scale, ctx.cl), None, None


def tv_loss_nhwc(img, scale=1.0, cl=3):
    return _TVFn.apply(img, float(scale), cl)


def calc_tv_loss(I):
    """fast_style_transfer.py:795-803 on an NCHW image."""
    c = I.shape[1]
    return tv_loss_nhwc(_ToNHWC.apply(I, cpad(c)), 1.0, c)


def style_grams(vgg, style_img_nchw):
    """Target Grams of a style image (fast_style_transfer.py:741-756 loadStyles, minus file IO):
    VGG(normalize(style)) -> gram per level, detached."""
    with torch.no_grad():
        feats = vgg.forward_nhwc(normalize_nhwc(ops.nchw_to_nhwc(style_img_nchw.contiguous())))
        return [gram_nhwc(f) for f in feats]


from . import _lib as _lib_routes  # noqa: E402
_lib_routes.apply_route_overrides(__name__, globals())
