"""RAFT all-pairs correlation volume, pyramid and window lookup, HIP-backed.

Drop-in for utils/raft/raft/corr.py:12-60 ``CorrBlock(fmap1, fmap2, num_levels=4, radius=4)`` and
its ``__call__(coords)`` (+ utils/raft/raft/utils/utils.py:57-71 ``bilinear_sampler``, which it
uses with align_corners=True).

MI355X design:
  * the all-pairs volume corr[b, i, j] = <fmap1[b,:,i], fmap2[b,:,j]> / sqrt(D) is a GEMM
    [H1W1 x D] x [D x H2W2]; it runs on the implicit-GEMM MFMA conv kernel as a 1x1 convolution
    whose "weight" is fmap2 in NHWC ([H2W2][D] is exactly the VST_PACK_OK layout of a 1x1 conv),
    writing the level-0 planes straight into one pyramid buffer (row stride = padded H2W2);
  * 1/sqrt(D) is applied to fmap1 before the GEMM (exact for power-of-two D, e.g. RAFT's 256);
  * levels 1..L-1 are 2x2 average pools of the previous level (one streaming kernel per level,
    ATen's summation order), packed after level 0;
  * the (2r+1)^2 window lookup per level is one gather kernel writing NHWC; the NCHW
    [B, L*(2r+1)^2, H1, W1] result of the reference is produced by the layout kernel.
"""
import torch

from . import ops
from .ops import cpad


class CorrBlock:
    def __init__(self, fmap1, fmap2, num_levels=4, radius=4, role="infer"):
        B, D, H, W = fmap1.shape
        if tuple(fmap2.shape) != (B, D, H, W):
            raise ValueError("CorrBlock: fmap1 and fmap2 must have the same shape")
        Dp = cpad(D)
        self._build(ops.nchw_to_nhwc(fmap1.float().contiguous(), Dp), ops.nchw_to_nhwc(fmap2.float().contiguous(), Dp),
                    D, num_levels, radius, role)

    @classmethod
    def from_nhwc(cls, f1, f2, D, num_levels=4, radius=4, role="infer"):
        """Build from NHWC feature maps [B, H, W, cpad(D)] (RAFT's fnet output, no layout pass)."""
        self = cls.__new__(cls)
        self._build(f1.contiguous(), f2.contiguous(), D, num_levels, radius, role)
        return self

    def _build(self, f1, f2, D, num_levels, radius, role):
        self.num_levels, self.radius = num_levels, radius
        B, H, W, Dp = f1.shape
        if num_levels > 1 and ((H >> (num_levels - 1)) < 2 or (W >> (num_levels - 1)) < 2):
            raise ValueError("CorrBlock: the coarsest level must be at least 2x2")
        self.B, self.H, self.W, self.D = B, H, W, D
        dev = f1.device
        # corr.py:58-59: matmul / torch.sqrt(torch.tensor(dim).float())
        sq = float(torch.sqrt(torch.tensor(D).float()))
        f1 = ops.channel_normalize(f1, None, torch.full((D,), sq, device=dev), 1.0, D)
        HW = H * W
        self.ld0 = cpad(HW)
        P = B * HW
        n = ops.corr_pyramid_floats(P, H, W, self.ld0, num_levels)
        self.pyr = torch.empty(n, device=dev)
        for b in range(B):
            if self.ld0 == HW:
                wp = f2[b].reshape(HW, 1, 1, Dp)
            else:
                wp = torch.zeros((self.ld0, 1, 1, Dp), device=dev)
                wp[:HW] = f2[b].reshape(HW, 1, 1, Dp)
            ops.split_planes(wp)
            out = self.pyr[b * HW * self.ld0:(b + 1) * HW * self.ld0].view(1, H, W, self.ld0)
            ops.conv2d_fwd(f1[b:b + 1], wp, None, self.ld0, 1, 1, 1, 0, out=out, role=role)
        ops.corr_pyramid(self.pyr, P, H, W, self.ld0, num_levels)

    def level(self, i):
        """Pyramid level i as the reference's corr_pyramid[i]: [B*H*W, 1, H>>i, W>>i] (level 0 is
        gathered out of its padded-stride planes)."""
        H, W, P = self.H, self.W, self.B * self.H * self.W
        if i == 0:
            return self.pyr[:P * self.ld0].view(P, self.ld0)[:, :H * W].reshape(P, 1, H, W)
        off = P * self.ld0
        h, w = H, W
        for lv in range(1, i + 1):
            h, w = h // 2, w // 2
            if lv < i:
                off += P * h * w
        return self.pyr[off:off + P * h * w].view(P, 1, h, w)

    def lookup_nhwc(self, coords, cs=None):
        """[B, H, W, cs or cpad(L*(2r+1)^2)] window features at coords [B, 2, H, W] (x, y pixels); the channels
        past L*(2r+1)^2 are zero."""
        return ops.corr_lookup(self.pyr, coords.float().contiguous(), self.B, self.H, self.W, self.H,
                               self.W, self.ld0, self.num_levels, self.radius, cs=cs)

    def __call__(self, coords):
        K = 2 * self.radius + 1
        return ops.nhwc_to_nchw(self.lookup_nhwc(coords), self.num_levels * K * K)

    @staticmethod
    def corr(fmap1, fmap2):
        """corr.py:53-60: [B, H, W, 1, H, W] all-pairs volume / sqrt(D)."""
        cb = CorrBlock(fmap1, fmap2, num_levels=1, radius=0)
        return cb.level(0).reshape(cb.B, cb.H, cb.W, 1, cb.H, cb.W)


def coords_grid(batch, ht, wd, device="cuda"):
    """utils/raft/raft/utils/utils.py coords_grid: [B, 2, H, W] (x, y) pixel grid."""
    ys, xs = torch.meshgrid(torch.arange(ht, device=device), torch.arange(wd, device=device), indexing="ij")
    return torch.stack([xs, ys], 0).float()[None].repeat(batch, 1, 1, 1)


def corr_flops(B, D, H, W):
    """Algorithmic FLOPs of the all-pairs GEMM: 2 * B * (HW)^2 * D."""
    return 2.0 * B * (H * W) ** 2 * D


def corr_bytes(B, H, W, levels=4):
    """Algorithmic HBM bytes of volume + pyramid: level-0 write, then per level read + write."""
    hw = H * W
    total = 4.0 * B * hw * hw
    h, w = H, W
    for _ in range(1, levels):
        prev = h * w
        h, w = h // 2, w // 2
        total += 4.0 * B * hw * (prev + h * w)
    return total
