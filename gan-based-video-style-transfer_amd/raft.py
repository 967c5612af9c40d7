"""RAFT optical flow (inference), HIP-backed (SURVEY §8 A19 + §8f rank 3).

Drop-in for utils/raft/raft/raft.py ``RAFT(args)`` (the full model, ``args.small = False``) with
its BasicEncoder feature / context networks (extractor.py:117-189), BasicUpdateBlock
(update.py:114-139: BasicMotionEncoder, SepConvGRU, FlowHead, mask head), CorrBlock (raft_corr.py)
and convex upsampling; identical module tree / state_dict keys, so a RAFT checkpoint loads by name.
``InputPadder`` and ``compute_raft`` mirror utils/utils.py:7-24 and the callers' ``computeRAFT``
(MoGAN/models/cycle_gan_model.py:125-132, utils/sintel_eval.py:53-60).  Inference only — every
reference caller runs RAFT under ``torch.no_grad()`` in eval mode.

MI355X design: all activations NHWC fp32 on the implicit-GEMM MFMA conv kernels; eval-mode
BatchNorm of the context encoder is folded into its conv weights at pack time; the GRU's z and r
convs are one conv with concatenated weights (384 -> 256); the GRU inputs live in two persistent
[P, 384] concat buffers ([h | inp | motion] and [r*h | inp | motion]) so torch.cat never runs —
the glue kernels write straight into their channel slices; the mask head runs only where its
output is used (every iteration unless test_mode, else the last); the 0.25 mask scale is folded
into the last mask conv (a power-of-two scale is exact).
"""
import torch
import torch.nn as nn

from . import ops
from .ops import cpad
from .raft_corr import CorrBlock, coords_grid


###############################################################################
# parameter holders (reference module tree)
###############################################################################
class Conv(nn.Module):
    """nn.Conv2d state: weight [Co, Ci, kh, kw], bias [Co]."""

    def __init__(self, cin, cout, k, padding=0, stride=1, bias=True):
        super().__init__()
        kh, kw = (k, k) if isinstance(k, int) else k
        ph, pw = (padding, padding) if isinstance(padding, int) else padding
        self.cin, self.cout, self.kh, self.kw, self.ph, self.pw, self.stride = cin, cout, kh, kw, ph, pw, stride
        self.weight = nn.Parameter(torch.empty(cout, cin, kh, kw))
        nn.init.kaiming_normal_(self.weight, mode="fan_out", nonlinearity="relu")
        self.bias = nn.Parameter(torch.zeros(cout)) if bias else None

    def extra_repr(self):
        return f"{self.cin}, {self.cout}, kernel_size=({self.kh}, {self.kw}), stride={self.stride}, " \
               f"padding=({self.ph}, {self.pw})"


class BatchNorm(nn.Module):
    """nn.BatchNorm2d state (eval mode only: folded into the preceding conv)."""

    def __init__(self, c, eps=1e-5):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(c))
        self.bias = nn.Parameter(torch.zeros(c))
        self.register_buffer("running_mean", torch.zeros(c))
        self.register_buffer("running_var", torch.ones(c))
        self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long))


class _Norm(nn.Module):
    """InstanceNorm2d(affine=False) / no norm: no state."""

    def __init__(self, kind):
        super().__init__()
        self.kind = kind

    def extra_repr(self):
        return self.kind


def _norm(kind, c):
    if kind == "batch":
        return BatchNorm(c)
    if kind in ("instance", "none"):
        return _Norm(kind)
    raise NotImplementedError("norm_fn %s (group norm is not used by RAFT's full model)" % kind)


class ResidualBlock(nn.Module):
    def __init__(self, in_planes, planes, norm_fn, stride=1):
        super().__init__()
        self.conv1 = Conv(in_planes, planes, 3, padding=1, stride=stride)
        self.conv2 = Conv(planes, planes, 3, padding=1)
        self.norm1, self.norm2 = _norm(norm_fn, planes), _norm(norm_fn, planes)
        self.stride = stride
        if stride != 1:
            self.norm3 = _norm(norm_fn, planes)
            self.downsample = nn.Sequential(Conv(in_planes, planes, 1, stride=stride), self.norm3)
        else:
            self.downsample = None


class BasicEncoder(nn.Module):
    def __init__(self, output_dim=128, norm_fn="batch"):
        super().__init__()
        self.norm_fn = norm_fn
        self.norm1 = _norm(norm_fn, 64)
        self.conv1 = Conv(3, 64, 7, padding=3, stride=2)
        self.layer1 = nn.Sequential(ResidualBlock(64, 64, norm_fn, 1), ResidualBlock(64, 64, norm_fn, 1))
        self.layer2 = nn.Sequential(ResidualBlock(64, 96, norm_fn, 2), ResidualBlock(96, 96, norm_fn, 1))
        self.layer3 = nn.Sequential(ResidualBlock(96, 128, norm_fn, 2), ResidualBlock(128, 128, norm_fn, 1))
        self.conv2 = Conv(128, output_dim, 1)
        self.output_dim = output_dim


class BasicMotionEncoder(nn.Module):
    def __init__(self, cor_planes):
        super().__init__()
        self.convc1 = Conv(cor_planes, 256, 1)
        self.convc2 = Conv(256, 192, 3, padding=1)
        self.convf1 = Conv(2, 128, 7, padding=3)
        self.convf2 = Conv(128, 64, 3, padding=1)
        self.conv = Conv(64 + 192, 128 - 2, 3, padding=1)


class SepConvGRU(nn.Module):
    def __init__(self, hidden_dim=128, input_dim=192 + 128):
        super().__init__()
        c = hidden_dim + input_dim
        self.convz1 = Conv(c, hidden_dim, (1, 5), padding=(0, 2))
        self.convr1 = Conv(c, hidden_dim, (1, 5), padding=(0, 2))
        self.convq1 = Conv(c, hidden_dim, (1, 5), padding=(0, 2))
        self.convz2 = Conv(c, hidden_dim, (5, 1), padding=(2, 0))
        self.convr2 = Conv(c, hidden_dim, (5, 1), padding=(2, 0))
        self.convq2 = Conv(c, hidden_dim, (5, 1), padding=(2, 0))


class FlowHead(nn.Module):
    def __init__(self, input_dim=128, hidden_dim=256):
        super().__init__()
        self.conv1 = Conv(input_dim, hidden_dim, 3, padding=1)
        self.conv2 = Conv(hidden_dim, 2, 3, padding=1)


class BasicUpdateBlock(nn.Module):
    def __init__(self, corr_levels, corr_radius, hidden_dim=128):
        super().__init__()
        self.encoder = BasicMotionEncoder(corr_levels * (2 * corr_radius + 1) ** 2)
        self.gru = SepConvGRU(hidden_dim=hidden_dim, input_dim=128 + hidden_dim)
        self.flow_head = FlowHead(hidden_dim, hidden_dim=256)
        self.mask = nn.Sequential(Conv(128, 256, 3, padding=1), _Norm("ReLU"), Conv(256, 64 * 9, 1))


###############################################################################
# packs
###############################################################################
# The correlation features' channel stride: 4 levels x 81 = 324 padded to 328, so that convc1 (1x1, 324 -> 256) runs
# on the split-bf16 kernel (K in 8-channel chunks) instead of the fp32-operand one; False keeps 324
_CORR_CS = 328


def _pack(w, b, ip=None):
    """OK pack (+ bf16 split planes) and the channel-padded bias of a conv weight [Co, Ci, kh, kw]; ip: the input
    channel stride the pack is laid out for (default cpad)."""
    co = w.shape[0]
    bp = None
    if b is not None:
        bp = torch.zeros(cpad(co), device=w.device)
        bp[:co] = b
    return ops.weight_pack(w.contiguous(), ops.PACK_FWD, Ip=ip), bp


def _fold_bn(conv, bn):
    """Eval BatchNorm after a conv: w' = w * g / sqrt(rv + eps), b' = (b - rm) * g / sqrt(rv + eps) + beta."""
    w, b = conv.weight.detach(), conv.bias.detach() if conv.bias is not None else None
    if not isinstance(bn, BatchNorm):
        return w, b
    scale = bn.weight.detach() / torch.sqrt(bn.running_var + bn.eps)
    b0 = b if b is not None else torch.zeros_like(bn.running_mean)
    return w * scale.view(-1, 1, 1, 1), (b0 - bn.running_mean) * scale + bn.bias.detach()


class _ConvOp:
    def __init__(self, conv, bn=None, scale=None, cat_with=None, ip=None):
        w, b = _fold_bn(conv, bn) if bn is not None else (conv.weight.detach(), conv.bias.detach()
                                                          if conv.bias is not None else None)
        if cat_with is not None:
            w = torch.cat([w, cat_with.weight.detach()], 0)
            b = torch.cat([b, cat_with.bias.detach()], 0)
        if scale is not None:
            w, b = w * scale, b * scale
        self.wp, self.bias = _pack(w, b, ip)
        self.cop = cpad(w.shape[0])
        self.kh, self.kw, self.ph, self.pw, self.stride = conv.kh, conv.kw, conv.ph, conv.pw, conv.stride

    def __call__(self, x, act="none", role="fwd"):
        if self.ph == self.pw and self.kh == self.kw:
            return ops.conv2d_fwd(x, self.wp, self.bias, self.cop, self.kh, self.kw, self.stride, self.ph, "zero",
                                  act=act, role=role)
        return ops.conv2d_fwd_hw(x, self.wp, self.bias, self.cop, self.kh, self.kw, self.stride, self.ph, self.pw,
                                 act=act, role=role)


###############################################################################
# RAFT
###############################################################################
class RAFT(nn.Module):
    """raft.py:24-144 (full model).  ``args`` needs ``small`` (False), optionally ``mixed_precision``
    (ignored: fp32 arithmetic), ``alternate_corr`` (False), ``dropout`` (0, inference)."""

    def __init__(self, args):
        super().__init__()
        self.args = args
        if getattr(args, "small", False):
            raise NotImplementedError("RAFT small model (SmallEncoder / SmallUpdateBlock) is not ported")
        if getattr(args, "alternate_corr", False):
            raise NotImplementedError("alternate_corr (the CUDA sampler extension) is not ported")
        self.hidden_dim = hdim = 128
        self.context_dim = cdim = 128
        args.corr_levels = 4
        args.corr_radius = 4
        self.fnet = BasicEncoder(output_dim=256, norm_fn="instance")
        self.cnet = BasicEncoder(output_dim=hdim + cdim, norm_fn="batch")
        self.update_block = BasicUpdateBlock(args.corr_levels, args.corr_radius, hidden_dim=hdim)
        self.role = "fwd"  # conv arithmetic role (ops policy); fp32-equivalent by default
        self.use_graphs = True  # compute_raft replays a captured HIP graph per input shape
        self._packs, self._pkey = None, None
        self._graphs = {}

    def freeze_bn(self):
        pass  # BatchNorm is always evaluated with its running statistics here

    def _key(self):
        return (sum(p._version for p in self.parameters()), sum(b._version for b in self.buffers()),
                self.fnet.conv1.weight.data_ptr())

    def packs(self):
        key = self._key()
        if self._packs is None or self._pkey != key:
            self._graphs.clear()  # captured graphs read the previous packs
            with torch.no_grad():
                self._packs = self._make_packs()
            self._pkey = key
        return self._packs

    def graphed(self, image1, image2, iters, pads=(0, 0, 0, 0), nhwc=False):
        """test_mode forward replayed from a HIP graph captured once per (shape, iters, pads, layout):
        the ~20 launches per GRU iteration become one graph launch.  Returns fresh copies of
        (flow_low, flow_up)."""
        self.packs()
        key = (tuple(image1.shape), int(iters), tuple(pads), bool(nhwc), image1.device)
        ent = self._graphs.get(key)
        if ent is None:
            s1, s2 = image1.detach().clone(), image2.detach().clone()
            side = torch.cuda.Stream(device=image1.device)
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):  # warm-up outside capture (allocator, first-touch)
                self.forward(s1, s2, iters=iters, test_mode=True, pads=pads, nhwc=nhwc)
            torch.cuda.current_stream().wait_stream(side)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                out = self.forward(s1, s2, iters=iters, test_mode=True, pads=pads, nhwc=nhwc)
            ent = (g, s1, s2, out)
            self._graphs[key] = ent
        g, s1, s2, out = ent
        s1.copy_(image1)
        s2.copy_(image2)
        g.replay()
        return out[0].clone(), out[1].clone()

    def _make_packs(self):
        def enc(e):
            bn = e.norm_fn == "batch"
            P = {"conv1": _ConvOp(e.conv1, e.norm1 if bn else None), "conv2": _ConvOp(e.conv2), "blocks": []}
            for layer in (e.layer1, e.layer2, e.layer3):
                for blk in layer:
                    d = {"c1": _ConvOp(blk.conv1, blk.norm1 if bn else None),
                         "c2": _ConvOp(blk.conv2, blk.norm2 if bn else None)}
                    if blk.downsample is not None:
                        d["ds"] = _ConvOp(blk.downsample[0], blk.norm3 if bn else None)
                    P["blocks"].append(d)
            return P
        u = self.update_block
        g = u.gru
        return {"fnet": enc(self.fnet), "cnet": enc(self.cnet),
                "convc1": _ConvOp(u.encoder.convc1, ip=_CORR_CS), "convc2": _ConvOp(u.encoder.convc2),
                "convf1": _ConvOp(u.encoder.convf1), "convf2": _ConvOp(u.encoder.convf2),
                "conv": _ConvOp(u.encoder.conv),
                "zr1": _ConvOp(g.convz1, cat_with=g.convr1), "q1": _ConvOp(g.convq1),
                "zr2": _ConvOp(g.convz2, cat_with=g.convr2), "q2": _ConvOp(g.convq2),
                "fh1": _ConvOp(u.flow_head.conv1), "fh2": _ConvOp(u.flow_head.conv2),
                "m1": _ConvOp(u.mask[0]), "m2": _ConvOp(u.mask[2], scale=0.25)}

    # ---------------------------------------------------------------------------- encoders
    def _encode(self, P, norm_fn, x):
        role = self.role

        def norm_act(y, act):
            if norm_fn == "instance":
                return ops.instnorm_act_fwd(y, ops.instnorm_stats(y), act)
            return y

        epi = "none" if norm_fn == "instance" else "relu"
        y = norm_act(P["conv1"](x, epi, role), "relu")
        for d in P["blocks"]:
            t = norm_act(d["c1"](y, epi, role), "relu")
            t = norm_act(d["c2"](t, epi, role), "relu")
            xs = norm_act(d["ds"](y, "none", role), "none") if "ds" in d else y
            y = ops.add_relu(xs, t)
        return P["conv2"](y, "none", role)

    # ----------------------------------------------------------------------------- forward
    def forward(self, image1, image2, iters=12, flow_init=None, upsample=True, test_mode=False, pads=(0, 0, 0, 0),
                nhwc=False):
        """raft.py:86-144.  image1/2: NCHW [B,3,H,W] in the caller's scale (the reference maps
        2*(x/255)-1 regardless); pads = replicate padding (l, r, t, b) applied on the way in (the
        caller's InputPadder, fused).  Returns (flow_low, flow_up) in test_mode, else the list of
        flow_up per iteration.  nhwc=True: images are NHWC [B,H,W,Cs>=3] (e.g. generator outputs)
        and the flows come back as NHWC4 (2 logical channels)."""
        P = self.packs()
        role = self.role
        B = image1.shape[0]
        H, W = (image1.shape[1], image1.shape[2]) if nhwc else (image1.shape[2], image1.shape[3])
        l, r, t, b = pads
        imgs = torch.empty((2 * B, H + t + b, W + l + r, 4), device=image1.device)
        for k, im in enumerate((image1, image2)):
            ops.raft_prep(im.float().contiguous(), pads, nhwc=nhwc, out=imgs[k * B:(k + 1) * B])
        Hp, Wp = imgs.shape[1], imgs.shape[2]
        if Hp % 8 or Wp % 8:
            raise ValueError("RAFT: padded image size must be divisible by 8 (use InputPadder)")
        fmaps = self._encode(P["fnet"], "instance", imgs)
        corr_fn = CorrBlock.from_nhwc(fmaps[:B], fmaps[B:], 256, self.args.corr_levels, self.args.corr_radius,
                                      role=role)
        cnet = self._encode(P["cnet"], "batch", imgs[:B])
        h8, w8 = cnet.shape[1], cnet.shape[2]
        dev = cnet.device
        hd, cd = self.hidden_dim, self.context_dim
        xcs = hd + cd + 128
        h = torch.empty((B, h8, w8, hd), device=dev)
        hx = torch.empty((B, h8, w8, xcs), device=dev)
        rhx = torch.empty((B, h8, w8, xcs), device=dev)
        ops.raft_ctx_split(cnet, hd, cd, h, hx, rhx)
        coords1 = coords_grid(B, h8, w8, device=dev)
        if flow_init is not None:
            coords1 = coords1 + flow_init.to(dev).float()
        coords1 = coords1.contiguous()
        flow4 = torch.empty((B, h8, w8, 4), device=dev)
        cat = torch.empty((B, h8, w8, 256), device=dev)
        preds = []
        for it in range(iters):
            corr = corr_fn.lookup_nhwc(coords1, cs=_CORR_CS)
            ops.raft_flow4(coords1, flow4)
            # BasicMotionEncoder (update.py:88-98)
            cor = P["convc2"](P["convc1"](corr, "relu", role), "relu", role)
            flo = P["convf2"](P["convf1"](flow4, "relu", role), "relu", role)
            ops.copy_channels(cor, 0, cat, 0, 192)
            ops.copy_channels(flo, 0, cat, 192, 64)
            out = P["conv"](cat, "relu", role)
            ops.raft_motion(out, 126, flow4, hx, rhx, hd + cd)
            # SepConvGRU (update.py:46-58): horizontal then vertical
            for zk, qk in (("zr1", "q1"), ("zr2", "q2")):
                zr = P[zk](hx, "none", role)
                ops.gru_reset(zr, h, rhx)
                q = P[qk](rhx, "tanh", role)
                ops.gru_update(zr, q, h, hx)
            delta = P["fh2"](P["fh1"](h, "relu", role), "none", role)
            ops.raft_coords_update(coords1, delta)
            if not test_mode or it == iters - 1:
                mask = P["m2"](P["m1"](h, "relu", role), "none", role)
                up = ops.raft_upsample(coords1, mask)
                preds.append(ops.nchw_to_nhwc(up) if nhwc else up)
        if test_mode:
            ops.raft_flow4(coords1, flow4)
            return (flow4 if nhwc else ops.nhwc_to_nchw(flow4, 2)), preds[-1]
        return preds


class InputPadder:
    """utils/raft/raft/utils/utils.py:7-24 (replicate padding to a multiple of 8)."""

    def __init__(self, dims, mode="sintel"):
        self.ht, self.wd = dims[-2:]
        pad_ht = (((self.ht // 8) + 1) * 8 - self.ht) % 8
        pad_wd = (((self.wd // 8) + 1) * 8 - self.wd) % 8
        if mode == "sintel":
            self._pad = [pad_wd // 2, pad_wd - pad_wd // 2, pad_ht // 2, pad_ht - pad_ht // 2]
        else:
            self._pad = [pad_wd // 2, pad_wd - pad_wd // 2, 0, pad_ht]

    @property
    def pads(self):
        return tuple(self._pad)

    def unpad(self, x):
        ht, wd = x.shape[-2:]
        c = [self._pad[2], ht - self._pad[3], self._pad[0], wd - self._pad[1]]
        return x[..., c[0]:c[1], c[2]:c[3]]


def compute_raft(model, img1, img2, it=20):
    """MoGAN/models/cycle_gan_model.py:125-132 computeRAFT: pad, run test_mode, return flow_up (at the
    padded size, as the reference does)."""
    with torch.no_grad():
        padder = InputPadder(img1.shape)
        if model.use_graphs:
            return model.graphed(img1, img2, it, padder.pads)[1]
        _, flow_up = model(img1, img2, iters=it, test_mode=True, pads=padder.pads)
    return flow_up


def raft_flops(B, H, W, iters):
    """Algorithmic conv + corr FLOPs of one RAFT call at padded size HxW (for throughput reporting)."""
    h, w = H // 8, W // 8
    P8 = B * h * w

    def conv(pix, ci, co, k):
        return 2.0 * pix * ci * co * k

    enc = 0.0
    for nimg, out in ((2 * B, 256), (B, 256)):
        H2, W2, H4, W4 = H // 2, W // 2, H // 4, W // 4
        enc += conv(nimg * H2 * W2, 3, 64, 49) + 4 * conv(nimg * H2 * W2, 64, 64, 9)
        enc += conv(nimg * H4 * W4, 64, 96, 9) + 3 * conv(nimg * H4 * W4, 96, 96, 9) + conv(nimg * H4 * W4, 64, 96, 1)
        enc += conv(nimg * h * w, 96, 128, 9) + 3 * conv(nimg * h * w, 128, 128, 9) + conv(nimg * h * w, 96, 128, 1)
        enc += conv(nimg * h * w, 128, out, 1)
    corr = 2.0 * B * (h * w) ** 2 * 256
    upd = (conv(P8, 324, 256, 1) + conv(P8, 256, 192, 9) + conv(P8, 2, 128, 49) + conv(P8, 128, 64, 9)
           + conv(P8, 256, 126, 9) + 2 * (conv(P8, 384, 256, 5) + conv(P8, 384, 128, 5))
           + conv(P8, 128, 256, 9) + conv(P8, 256, 2, 9))
    mask = conv(P8, 128, 256, 9) + conv(P8, 256, 576, 1)
    return enc + corr + iters * upd + mask
