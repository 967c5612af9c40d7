"""Drop-in for methods/learning-based/fs_lib.py (warp, 5-39), HIP-backed.

``warp(x, flo)`` = grid_sample(x, grid) * (grid_sample(ones, grid) >= 0.9999) with the grid
normalised by max(W-1, 1) / max(H-1, 1) and the container-default align_corners=False — the
sample and its validity come out of one kernel pass (vst_warp_masked_fwd); the backward scatters
only through kept samples (no gradient flows into the flow or the mask, as in the reference).
"""
import torch

from . import ops
from .flowtools import _nchw_to_nhwc, _nhwc_to_nchw


class _WarpMaskedNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, flow, align_corners):
        ctx.save_for_backward(flow)
        ctx.align = align_corners
        return ops.warp_masked_nhwc(x, flow, align_corners)

    @staticmethod
    def backward(ctx, g):
        (flow,) = ctx.saved_tensors
        return ops.warp_masked_bwd_nhwc(g.contiguous(), flow, ctx.align), None, None


def warp_nhwc(x, flow, align_corners=False):
    """x: [B,H,W,Cs] (Cs % 4 == 0), flow: [B,2,H,W] -> masked warp [B,H,W,Cs]."""
    return _WarpMaskedNHWC.apply(x.contiguous(), flow.contiguous().float(), bool(align_corners))


def warp(x, flo):
    """fs_lib.py:5-39 on NCHW x [B,C,H,W] and flow [B,2,H,W] (pixels, channel 0 = x)."""
    C = x.shape[1]
    return _nhwc_to_nchw(warp_nhwc(_nchw_to_nhwc(x), flo), C)
