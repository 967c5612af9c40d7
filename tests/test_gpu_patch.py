"""The PatchGAN head — Conv2d(8*ndf, 1, 4, stride 1, padding 1), networks.py:576-578 — on its row
kernels (csrc/patch.hip): forward (vst_conv2d_fwd_co, co_real = 1), weight gradient (vst_conv2d_wgrad
with Co = 1) and data gradient (vst_conv2d_tfwd_co) against torch fp32 autograd on the same inputs.
fp32 FMA chains on both sides, only the summation order differs: |err| <= 2e-5 * max|ref| + 1e-6.
Shapes: the C2 head (N = 8 / 4 at 31x31x512), the C3 Sintel-size head (27 x 64 input: column
segments), a three-segment row, the narrowest and widest channel layouts (Cin / 4 = 16 .. 256 channel
quads), a 3x3 kernel, and a channel count the row kernels do not take (the generic path)."""
import pytest
import torch
import torch.nn.functional as F

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


def _close(got, ref, tol=2e-5, what=""):
    got = got.detach().float().cpu()
    ref = ref.detach().float().cpu()
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    scale = ref.abs().max().item() + 1e-12
    err = (got - ref).abs().max().item()
    assert err <= tol * scale + 1e-6, f"{what}: max|err|={err:.3e} scale={scale:.3e}"


HEAD_CASES = [
    # N, Ci, H, W, k, act
    (8, 512, 31, 31, 4, "none"),     # C2 backward_D (real + fake batched)
    (4, 512, 31, 31, 4, "none"),     # C2 backward_G
    (2, 512, 27, 64, 4, "none"),     # C3 Sintel-size head: 63 outputs per row, two column segments
    (1, 256, 9, 130, 4, "lrelu"),    # three segments, 64 channel quads (four column groups)
    (2, 64, 7, 7, 4, "none"),        # 16 channel quads: a wave spans four column groups
    (1, 1024, 6, 5, 4, "none"),      # 256 channel quads: one column group
    (2, 128, 10, 12, 3, "none"),     # 3x3 taps
    (2, 36, 5, 6, 4, "none"),        # Cin / 4 does not divide 256: the generic VALU path
]


@pytest.mark.parametrize("case", HEAD_CASES, ids=lambda c: "N%d_C%d_%dx%d_k%d" % c[:5])
def test_patch_head_fwd_wgrad_dgrad(ops, case):
    N, Ci, H, W, k, act = case
    pad = 1
    x = _g(81, (N, Ci, H, W))
    w = _g(82, (1, Ci, k, k), 0.05)
    b = _g(83, (1,), 0.1)
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    yr = F.conv2d(xr, wr, br, padding=pad)
    if act == "lrelu":
        yr = F.leaky_relu(yr, 0.2)
    gy = _g(84, tuple(yr.shape))
    yr.backward(gy)
    wd = w.to(DEV)
    kc = ops.weight_pack(wd, ops.PACK_FWD)
    ck = ops.weight_pack(wd, ops.PACK_DGRAD)
    bp = torch.zeros(4, device=DEV)
    bp[0] = b[0]
    xn = ops.nchw_to_nhwc(x.to(DEV).contiguous())
    y = ops.conv2d_fwd(xn, kc, bp, 4, k, k, 1, pad, "zero", act=act, slope=0.2, co_real=1)
    _close(ops.nhwc_to_nchw(y.contiguous(), 1).cpu(), yr, what="head fwd")
    assert torch.all(y[..., 1:] == 0)
    # the gradients (of the pre-activation output: gy through the activation)
    g = gy if act == "none" else gy * torch.where(F.conv2d(x, w, b, padding=pad) > 0, 1.0, 0.2)
    gn = ops.nchw_to_nhwc(g.to(DEV).contiguous(), 4)
    assert gn.shape[-1] == 4 and torch.all(gn[..., 1:] == 0)
    dw = torch.full((1, Ci, k, k), 0.5, device=DEV)
    db = torch.full((1,), 0.25, device=DEV)
    ops.conv2d_wgrad(xn, gn, dw, db, k, k, 1, pad, "zero", 1, Ci, Ci * k * k, k * k, accumulate=True)
    _close(dw.cpu() - 0.5, wr.grad, what="head wgrad")
    _close(db.cpu() - 0.25, br.grad, what="head bgrad")
    dx = ops.conv2d_tfwd(gn, ck, None, H, W, xn.shape[-1], k, k, 1, pad, co_real=1)
    _close(ops.nhwc_to_nchw(dx.contiguous(), Ci).cpu(), xr.grad, what="head dgrad")
    dx4 = ops.conv2d_tfwd(gn, ck, None, H, W, xn.shape[-1], k, k, 1, pad)
    _close(dx4, dx, what="head dgrad vs the 4-channel transposed conv")


def test_patch_head_deterministic(ops):
    """The weight gradient's partials are summed in a fixed order: two runs are bit-identical."""
    N, Ci, H = 8, 512, 31
    xn = ops.nchw_to_nhwc(_g(91, (N, Ci, H, H)).to(DEV).contiguous())
    gn = torch.zeros((N, H - 1, H - 1, 4), device=DEV)
    gn[..., 0] = _g(92, (N, H - 1, H - 1)).to(DEV)
    outs = []
    for _ in range(2):
        dw = torch.zeros((1, Ci, 4, 4), device=DEV)
        ops.conv2d_wgrad(xn, gn, dw, None, 4, 4, 1, 1, "zero", 1, Ci, Ci * 16, 16, accumulate=False)
        outs.append(dw)
    assert torch.equal(outs[0], outs[1])


IMG_CASES = [
    # N, Ci, H, W, Co, k, stride, pad
    (8, 3, 256, 256, 64, 4, 2, 1),   # C2 backward_D: the PatchGAN first layer, real + fake batched
    (2, 3, 32, 32, 16, 4, 2, 1),
    (3, 3, 17, 18, 64, 4, 2, 1),     # odd height: a partial last pixel pair
    (2, 2, 20, 20, 32, 3, 1, 1),     # 3x3 stride 1, two real channels
    (1, 1, 9, 11, 8, 4, 2, 1),       # one channel, 8 outputs
]


@pytest.mark.parametrize("with_db", [True, False])
@pytest.mark.parametrize("case", IMG_CASES, ids=lambda c: "N%d_C%d_%dx%d_co%d_k%ds%d" % c[:7])
def test_image_input_wgrad(ops, case, with_db):
    """The image-input weight gradient on fp32 MFMA (patch.hip img_wgrad_k), with the bias gradient from
    its constant-1 operand column (vst_conv2d_wgrad_bias) or without (vst_conv2d_wgrad), vs torch."""
    N, Ci, H, W, Co, k, st, pad = case
    x = _g(101, (N, Ci, H, W))
    w = _g(102, (Co, Ci, k, k), 0.1)
    b = _g(103, (Co,), 0.1)
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    yr = F.conv2d(xr, wr, br, stride=st, padding=pad)
    gy = _g(104, tuple(yr.shape))
    yr.backward(gy)
    xn = ops.nchw_to_nhwc(x.to(DEV).contiguous(), 4)
    xn[..., 3] = 7.0  # the padding channel is never read as data
    gn = ops.nchw_to_nhwc(gy.to(DEV).contiguous())
    dw = torch.full((Co, Ci, k, k), 0.5, device=DEV)
    db = torch.full((Co,), 0.25, device=DEV) if with_db else None
    ops.conv2d_wgrad(xn, gn, dw, db, k, k, st, pad, "zero", Co, Ci, Ci * k * k, k * k, accumulate=True)
    _close(dw.cpu() - 0.5, wr.grad, what="image wgrad")
    if with_db:
        _close(db.cpu() - 0.25, br.grad, what="image bgrad")
