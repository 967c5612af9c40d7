"""Flow ops — drop-in for utils/flowtools.py (warp 18-32, fbcCheckTorch 34-58, gradient 12-16).

``warp(x, f)`` and ``fbcCheckTorch(ff, bf, device)`` take and return NCHW tensors exactly like the
reference; on the GPU they run the libvst_hip warp / consistency kernels (the warp is
differentiable w.r.t. x — the only gradient any training path needs).  ``warp_nhwc``
is the zero-copy entry for NHWC tensors used inside the HIP models.
"""
import torch

from . import ops


class _WarpNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, flow, align_corners):
        ctx.save_for_backward(flow)
        ctx.align = align_corners
        return ops.warp_nhwc(x, flow, align_corners)

    @staticmethod
    def backward(ctx, g):
        (flow,) = ctx.saved_tensors
        return ops.warp_bwd_nhwc(g.contiguous(), flow, ctx.align), None, None


def warp_nhwc(x, flow, align_corners=False):
    """x: [B,H,W,Cs] (Cs % 4 == 0), flow: [B,2,H,W] -> [B,H,W,Cs]."""
    return _WarpNHWC.apply(x.contiguous(), flow.contiguous(), bool(align_corners))


def warp(x, f, align_corners=False):
    """utils/flowtools.py:18-32 — backward bilinear warp of NCHW x by flow f (pixels, ch0 = x)."""
    B, C, H, W = x.shape
    y = warp_nhwc(_nchw_to_nhwc(x), f.float(), align_corners)
    return _nhwc_to_nchw(y, C)


def gradient(x):
    """utils/flowtools.py:12-16 (zero-padded central differences / 2), on torch ops — helper only,
    the fused path is inside fbcCheckTorch."""
    import torch.nn.functional as F
    dx = (F.pad(x, (0, 1, 0, 0))[:, :, 1:] - F.pad(x, (1, 0, 0, 0))[:, :, :-1]) / 2
    dy = (F.pad(x, (0, 0, 0, 1))[:, 1:, :] - F.pad(x, (0, 0, 1, 0))[:, :-1, :]) / 2
    return torch.stack([dx, dy])


def fbcCheckTorch(ff, bf, device="cuda"):
    """utils/flowtools.py:34-58 — occlusion / motion-boundary mask [B,1,H,W] in {0,1}, one kernel."""
    ff = ff.to(device).float().contiguous()
    bf = bf.to(device).float().contiguous()
    return ops.fbcheck(ff, bf)


class _NCHW2NHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.c = x.shape[1]
        return ops.nchw_to_nhwc(x.contiguous().float())

    @staticmethod
    def backward(ctx, g):
        return ops.nhwc_to_nchw(g.contiguous(), ctx.c)


class _NHWC2NCHW(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, c):
        ctx.cs = x.shape[-1]
        return ops.nhwc_to_nchw(x.contiguous(), c)

    @staticmethod
    def backward(ctx, g):
        return ops.nchw_to_nhwc(g.contiguous(), ctx.cs), None


def _nchw_to_nhwc(x):
    return _NCHW2NHWC.apply(x)


def _nhwc_to_nchw(x, c):
    return _NHWC2NCHW.apply(x, c)
