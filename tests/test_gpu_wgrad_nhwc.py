"""The weight gradient over NHWC operands (vst_conv2d_wgrad_nhwc, round 6): x fp32 NHWC and dy as its NHWC bf16
planes (instnorm_act_bwd(apre=True)), read through k-major stage images and ds_read_b64_tr_b16.  Same split plan,
per-stage MFMA sequence and lane k assignment as the channel-major route (vst_conv2d_wgrad_pre with the IN
backward's channel-major planes), so the two must agree BIT FOR BIT; and both against torch's fp32 weight gradient
(conv tolerance CONV_TOL["bf16x6"], relative to max|ref|).  Reference: the ResnetBlock convs'
weight gradients, methods/GAN-based/CycleGAN/models/networks.py:404-426."""
import pytest
import torch
import torch.nn.functional as F

from conftest import CONV_TOL

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module")
def ops():
    import gbvst
    from gbvst import ops as o
    gbvst._lib.load()
    return o


def _g(seed, shape, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g) * scale


CASES = [
    # name, N, H, W, C, stride, pad mode
    ("res_N8", 8, 64, 64, 256, 1, "reflect"),    # the batched G_A calls (whole 256x128 rounds)
    ("res_N12", 12, 64, 64, 256, 1, "reflect"),  # the N=12 calls
    ("res_N1", 1, 64, 64, 256, 1, "reflect"),    # B=1 (many splits)
    ("res_N2_32", 2, 32, 32, 256, 1, "reflect"),
    ("res_C3_size", 1, 109, 256, 256, 1, "reflect"),  # the 436x1024 ResnetBlocks (C3 / C5)
    ("zero_pad", 2, 32, 64, 256, 1, "zero"),
    ("stride2", 2, 64, 64, 256, 2, "zero"),
]


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_wgrad_nhwc_bit_identical(ops, case):
    name, N, H, W, C, st, mode = case
    prev = ops.set_conv_math("bf16x6")
    try:
        Ho, Wo = (H + 2 - 3) // st + 1, (W + 2 - 3) // st + 1
        assert ops.wgrad_nhwc_ok(N, H, W, C, Ho, Wo, C, 3, st, 1, "bf16x6"), name
        x = _g(11, (N, H, W, C)).to(DEV)
        y = _g(12, (N, Ho, Wo, C)).to(DEV)
        ga = _g(13, (N, Ho, Wo, C)).to(DEV)
        s = ops.instnorm_stats(y)
        dy, pl = ops.instnorm_act_bwd(ga, y, s, "relu", planes=True)   # fp32 dy + its channel-major planes
        dyn = ops.instnorm_act_bwd(ga, y, s, "relu", apre=True)         # its NHWC planes only
        assert dyn.vst_planes_only
        dw0 = torch.zeros(C, C, 3, 3, device=DEV)
        dw1 = torch.zeros(C, C, 3, 3, device=DEV)
        ops.conv2d_wgrad(x, dy, dw0, None, 3, 3, st, 1, mode, C, C, C * 9, 9, dy_planes=pl)
        ops.conv2d_wgrad(x, dyn, dw1, None, 3, 3, st, 1, mode, C, C, C * 9, 9)  # -> vst_conv2d_wgrad_nhwc
        assert torch.equal(dw0, dw1), (name, (dw0 - dw1).abs().max().item())
        # accumulate: a second call adds in place
        ops.conv2d_wgrad(x, dyn, dw1, None, 3, 3, st, 1, mode, C, C, C * 9, 9)
        assert torch.allclose(dw1, 2 * dw0, rtol=1e-6, atol=0), name
        # vs torch fp32 (NCHW): dW of conv(pad(x), W) with output gradient dy
        xc = x.permute(0, 3, 1, 2).cpu().double()
        gy = dy.permute(0, 3, 1, 2).cpu().double()
        xp = F.pad(xc, (1,) * 4, mode="reflect") if mode == "reflect" else F.pad(xc, (1,) * 4)
        ref = torch.nn.grad.conv2d_weight(xp, (C, C, 3, 3), gy, stride=st)
        err = (dw0.cpu().double() - ref).abs().max().item()
        assert err <= CONV_TOL["bf16x6"] * ref.abs().max().item(), (name, err)
    finally:
        ops.set_conv_math(prev)


def test_wgrad_nhwc_declines(ops):
    """Shapes off the 256x128 / 128x128 x6 plans (image-layer channel counts, Wo not a multiple of 32, other
    policies) decline: the caller keeps the channel-major route.  128 channels take the 128x128 plan."""
    prev = ops.set_conv_math("bf16x6")
    try:
        assert ops.wgrad_nhwc_ok(2, 64, 64, 128, 64, 64, 128, 3, 1, 1, "bf16x6")
        assert not ops.wgrad_nhwc_ok(2, 64, 64, 4, 64, 64, 64, 3, 1, 1, "bf16x6")
        assert not ops.wgrad_nhwc_ok(2, 20, 20, 256, 20, 20, 256, 3, 1, 1, "bf16x6")
        ops.set_conv_math("fp32")
        assert not ops.wgrad_nhwc_ok(2, 64, 64, 256, 64, 64, 256, 3, 1, 1, ops.get_conv_math())
    finally:
        ops.set_conv_math(prev)


F32_CASES = [
    # name, N, H, W, Cx, Cyp, R, stride, pad mode  (x [N][H][W][Cx], dy fp32 [N][Ho][Wo][Cyp])
    ("d0_s2", 2, 256, 256, 64, 128, 3, 2, "zero"),      # the generator's first down conv (128x128 tiles)
    ("d1_s2", 2, 128, 128, 128, 256, 3, 2, "zero"),     # the second (also the u0 ConvTranspose's equivalent conv)
    ("D_4x4_s2", 2, 128, 128, 64, 128, 4, 2, "zero"),   # PatchGAN layer 1 (256x128 tiles)
    ("D_4x4_s2_b", 2, 64, 64, 128, 256, 4, 2, "zero"),
    ("res_f32", 2, 64, 64, 256, 256, 3, 1, "reflect"),  # the ResnetBlock shape with an fp32 dy
]


@pytest.mark.parametrize("case", F32_CASES, ids=[c[0] for c in F32_CASES])
def test_wgrad_nhwc_f32_bit_identical(ops, case):
    """vst_conv2d_wgrad_nhwc_f32 (dy fp32 NHWC split in the kernel) == the channel-major route that copies x into
    its padded channel-major image and dy into planes (same split, same plan) bit for bit; and vs torch fp32."""
    name, N, H, W, Cx, Cyp, R, st, mode = case
    prev = ops.set_conv_math("bf16x6")
    prev_f = ops.WGRAD_NHWC_F32
    try:
        Ho, Wo = (H + 2 - R) // st + 1, (W + 2 - R) // st + 1
        assert ops.wgrad_nhwc_f32_ok(N, H, W, Cx, Ho, Wo, Cyp, R, st, 1), name
        x = _g(21, (N, H, W, Cx)).to(DEV)
        dy = _g(22, (N, Ho, Wo, Cyp)).to(DEV)
        dw0 = torch.zeros(Cyp, Cx, R, R, device=DEV)
        dw1 = torch.zeros(Cyp, Cx, R, R, device=DEV)
        ops.WGRAD_NHWC_F32 = False
        ops.conv2d_wgrad(x, dy, dw0, None, R, R, st, 1, mode, Cyp, Cx, Cx * R * R, R * R)
        ops.WGRAD_NHWC_F32 = True
        ops.conv2d_wgrad(x, dy, dw1, None, R, R, st, 1, mode, Cyp, Cx, Cx * R * R, R * R)
        assert torch.equal(dw0, dw1), (name, (dw0 - dw1).abs().max().item())
        xc = x.permute(0, 3, 1, 2).cpu().double()
        gy = dy.permute(0, 3, 1, 2).cpu().double()
        xp = F.pad(xc, (1,) * 4, mode="reflect") if mode == "reflect" else F.pad(xc, (1,) * 4)
        ref = torch.nn.grad.conv2d_weight(xp, (Cyp, Cx, R, R), gy, stride=st)
        err = (dw1.cpu().double() - ref).abs().max().item()
        assert err <= CONV_TOL["bf16x6"] * ref.abs().max().item(), (name, err)
    finally:
        ops.WGRAD_NHWC_F32 = prev_f
        ops.set_conv_math(prev)


IM2COL_CASES = [
    # name, N, H, W, Cx, Cyp, R, stride, pad, pad mode  (output rows Wo % 32 != 0: the im2col form)
    ("sg_d4", 4, 32, 32, 256, 512, 4, 2, 1, "zero"),       # StarGAN D 256 -> 512, out 16x16 (split slabs)
    ("sg_d5", 4, 16, 16, 512, 1024, 4, 2, 1, "zero"),      # 512 -> 1024, out 8x8 (one split, straight into dw)
    ("sg_d6", 4, 8, 8, 1024, 2048, 4, 2, 1, "zero"),       # the widest layer, out 4x4
    ("refl_3x3", 2, 16, 16, 64, 128, 3, 1, 1, "reflect"),  # many slabs: the two-level reduction
]


@pytest.mark.parametrize("case", IM2COL_CASES, ids=[c[0] for c in IM2COL_CASES])
def test_wgrad_nhwc_f32_im2col(ops, case):
    """vst_conv2d_wgrad_nhwc_f32's im2col form (Wo % 32 != 0, few pixels): vs torch fp64 within the x6 conv
    tolerance, accumulating in place; and the route is taken (vst_conv2d_wgrad_nhwc_f32_ok, not the plain plan)."""
    name, N, H, W, Cx, Cyp, R, st, pad, mode = case
    prev = ops.set_conv_math("bf16x6")
    try:
        Ho, Wo = (H + 2 * pad - R) // st + 1, (W + 2 * pad - R) // st + 1
        assert Wo % 32 and not ops.wgrad_nhwc_ok(N, H, W, Cx, Ho, Wo, Cyp, R, st, pad, "bf16x6")
        assert ops.wgrad_nhwc_f32_ok(N, H, W, Cx, Ho, Wo, Cyp, R, st, pad), name
        x = _g(31, (N, H, W, Cx)).to(DEV)
        dy = _g(32, (N, Ho, Wo, Cyp)).to(DEV)
        base = _g(33, (Cyp, Cx, R, R)).to(DEV)
        dw = base.clone()
        ops.conv2d_wgrad(x, dy, dw, None, R, R, st, pad, mode, Cyp, Cx, Cx * R * R, R * R)  # accumulate
        xc = x.permute(0, 3, 1, 2).cpu().double()
        gy = dy.permute(0, 3, 1, 2).cpu().double()
        xp = F.pad(xc, (pad,) * 4, mode="reflect") if mode == "reflect" else F.pad(xc, (pad,) * 4)
        ref = torch.nn.grad.conv2d_weight(xp, (Cyp, Cx, R, R), gy, stride=st)
        got = (dw - base).cpu().double()
        err = (got - ref).abs().max().item()
        assert err <= CONV_TOL["bf16x6"] * ref.abs().max().item(), (name, err)
    finally:
        ops.set_conv_math(prev)


def test_wgrad_nhwc_f32_im2col_padded_channels(ops):
    """The im2col form when the weight has fewer input channels than x carries (Ci < Cx: one split but not the
    weight's own layout, so through a slab and the transposing reduction), and a shape it declines (N Ho Wo not a
    multiple of 32)."""
    prev = ops.set_conv_math("bf16x6")
    try:
        N, H, W, Cx, Ci, Cyp, R, st, pad = 4, 8, 8, 1024, 1000, 2048, 4, 2, 1
        Ho = Wo = (H + 2 * pad - R) // st + 1
        assert ops.wgrad_nhwc_f32_ok(N, H, W, Cx, Ho, Wo, Cyp, R, st, pad)
        assert not ops.wgrad_nhwc_f32_ok(1, H, W, Cx, Ho, Wo, Cyp, R, st, pad)  # P = 16
        x = _g(41, (N, H, W, Cx)).to(DEV)
        x[..., Ci:] = 0.0
        dy = _g(42, (N, Ho, Wo, Cyp)).to(DEV)
        dw = torch.zeros(Cyp, Ci, R, R, device=DEV)
        ops.conv2d_wgrad(x, dy, dw, None, R, R, st, pad, "zero", Cyp, Ci, Ci * R * R, R * R)
        xc = x[..., :Ci].permute(0, 3, 1, 2).cpu().double()
        gy = dy.permute(0, 3, 1, 2).cpu().double()
        ref = torch.nn.grad.conv2d_weight(F.pad(xc, (pad,) * 4), (Cyp, Ci, R, R), gy, stride=st)
        err = (dw.cpu().double() - ref).abs().max().item()
        assert err <= CONV_TOL["bf16x6"] * ref.abs().max().item(), err
    finally:
        ops.set_conv_math(prev)
