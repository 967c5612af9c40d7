"""vst::* torch.library operators (gbvst.library, SURVEY §8b "Callers").

CPU: every op is registered under torch.ops.vst with its schema, shape propagation through the fake
(meta) implementations, and CPU tensors are refused (no fallback).  GPU: each op and its autograd
backward against the PyTorch fp32 op it replaces (F.conv2d / reflect pad, F.conv_transpose2d,
F.instance_norm + act, F.grid_sample warp, the Gram matrix), at the conv tolerance of
tests/conftest.py (CONV_TOL, relative to max|ref|)."""
import pytest
import torch
import torch.nn.functional as F

import gbvst
from gbvst import library  # noqa: F401  (registers torch.ops.vst.*)


def test_all_ops_registered():
    for name in library.OPS:
        op = getattr(torch.ops.vst, name)
        assert op.default._schema.name == "vst::" + name


def test_fake_shapes():
    from torch._subclasses.fake_tensor import FakeTensorMode
    with FakeTensorMode():
        x = torch.empty(2, 64, 32, 32)
        w = torch.empty(128, 64, 3, 3)
        assert torch.ops.vst.conv2d(x, w, None, 2, 1, "zero").shape == (2, 128, 16, 16)
        assert torch.ops.vst.conv2d(x, torch.empty(64, 64, 3, 3), None, 1, 1, "reflect").shape == (2, 64, 32, 32)
        wt = torch.empty(64, 32, 3, 3)
        assert torch.ops.vst.conv_transpose2d(x, wt, None, 2, 1, 1).shape == (2, 32, 64, 64)
        assert torch.ops.vst.instance_norm_act(x, "relu", 0.0).shape == x.shape
        flow = torch.empty(2, 2, 32, 32)
        assert torch.ops.vst.warp_bilinear(x, flow).shape == x.shape
        assert torch.ops.vst.fbcheck(flow, flow).shape == (2, 1, 32, 32)
        assert torch.ops.vst.gram(x).shape == (2, 64, 64)
        img = torch.empty(2, 3, 32, 32)
        assert torch.ops.vst.temporal_loss(img, img, flow, torch.empty(2, 1, 32, 32), 10.0).shape == ()
        dx, dw, db = torch.ops.vst.conv2d_backward(torch.empty(2, 128, 16, 16), x, w, 2, 1, "zero")
        assert dx.shape == x.shape and dw.shape == w.shape and db.shape == (128,)


def test_cpu_tensors_refused():
    x = torch.randn(1, 4, 8, 8)
    w = torch.randn(4, 4, 3, 3)
    with pytest.raises(RuntimeError):
        torch.ops.vst.conv2d(x, w, None, 1, 1, "zero")
    with pytest.raises(RuntimeError):
        torch.ops.vst.warp_bilinear(x, torch.zeros(1, 2, 8, 8))


def _rel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.fixture
def gpu_fp32_math():
    from gbvst import ops
    gbvst._lib.load()
    prev = ops.set_conv_math("bf16x6")
    yield
    ops.set_conv_math(prev)


CONV_CASES = [  # (N, Ci, Co, H, k, stride, pad, pad_mode, bias)
    (2, 64, 64, 16, 3, 1, 1, "reflect", True),     # ResnetBlock conv
    (2, 64, 128, 16, 3, 2, 1, "zero", True),       # G down-sampling
    (2, 3, 64, 20, 7, 1, 3, "reflect", True),      # c7s1-64
    (2, 64, 128, 16, 4, 2, 1, "zero", True),       # PatchGAN s2
    (1, 32, 8, 12, 3, 1, 1, "zero", False),
    (2, 16, 32, 16, 3, 2, 1, "reflect", True),     # strided reflect: padded-frame dgrad + fold
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv2d_vs_torch(case, gpu_fp32_math):
    N, Ci, Co, H, k, st, pad, mode, has_b = case
    g = torch.Generator().manual_seed(7)
    x = torch.randn(N, Ci, H, H, generator=g).cuda().requires_grad_(True)
    w = (torch.randn(Co, Ci, k, k, generator=g) * 0.05).cuda().requires_grad_(True)
    b = (torch.randn(Co, generator=g) * 0.1).cuda().requires_grad_(True) if has_b else None
    y = torch.ops.vst.conv2d(x, w, b, st, pad, mode)
    xr, wr = x.detach().clone().requires_grad_(True), w.detach().clone().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True) if has_b else None
    xp = F.pad(xr, (pad,) * 4, mode="reflect") if mode == "reflect" else xr
    yr = F.conv2d(xp, wr, br, stride=st, padding=0 if mode == "reflect" else pad)
    assert y.shape == yr.shape
    assert _rel(y, yr) < 2e-5
    gy = torch.randn(y.shape, generator=g).cuda()
    y.backward(gy)
    yr.backward(gy)
    assert _rel(x.grad, xr.grad) < 2e-5
    assert _rel(w.grad, wr.grad) < 2e-5
    if has_b:
        assert _rel(b.grad, br.grad) < 1e-5


@pytest.mark.gpu
def test_conv_transpose2d_vs_torch(gpu_fp32_math):
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 128, 16, 16, generator=g).cuda().requires_grad_(True)
    w = (torch.randn(128, 64, 3, 3, generator=g) * 0.05).cuda().requires_grad_(True)
    b = (torch.randn(64, generator=g) * 0.1).cuda().requires_grad_(True)
    y = torch.ops.vst.conv_transpose2d(x, w, b, 2, 1, 1)
    xr, wr, br = (t.detach().clone().requires_grad_(True) for t in (x, w, b))
    yr = F.conv_transpose2d(xr, wr, br, stride=2, padding=1, output_padding=1)
    assert y.shape == yr.shape == (2, 64, 32, 32)
    assert _rel(y, yr) < 2e-5
    gy = torch.randn(y.shape, generator=g).cuda()
    y.backward(gy)
    yr.backward(gy)
    for a, r in ((x.grad, xr.grad), (w.grad, wr.grad), (b.grad, br.grad)):
        assert _rel(a, r) < 2e-5


@pytest.mark.gpu
@pytest.mark.parametrize("act", ["none", "relu", "lrelu"])
def test_instance_norm_act_vs_torch(act):
    g = torch.Generator().manual_seed(5)
    x = (torch.randn(2, 64, 16, 16, generator=g) * 3 + 1).cuda().requires_grad_(True)
    y = torch.ops.vst.instance_norm_act(x, act, 0.2)
    xr = x.detach().clone().requires_grad_(True)
    yr = F.instance_norm(xr, eps=1e-5)
    yr = {"none": yr, "relu": F.relu(yr), "lrelu": F.leaky_relu(yr, 0.2)}[act]
    assert _rel(y, yr) < 1e-5
    gy = torch.randn(y.shape, generator=g).cuda()
    y.backward(gy)
    yr.backward(gy)
    assert _rel(x.grad, xr.grad) < 1e-4


@pytest.mark.gpu
def test_warp_fbcheck_temporal_gram_adam():
    from gbvst import flowtools
    g = torch.Generator().manual_seed(9)
    x = torch.randn(2, 3, 24, 32, generator=g).cuda().requires_grad_(True)
    flow = (torch.randn(2, 2, 24, 32, generator=g) * 2).cuda()
    y = torch.ops.vst.warp_bilinear(x, flow)
    # the reference warp (utils/flowtools.py:18-32) restated with grid_sample
    B, C, H, W = x.shape
    xx = torch.arange(W, device="cuda").view(1, -1).expand(H, W).float()
    yy = torch.arange(H, device="cuda").view(-1, 1).expand(H, W).float()
    grid = torch.stack([xx, yy]).unsqueeze(0) + flow
    grid = torch.stack([2 * grid[:, 0] / max(W - 1, 1) - 1, 2 * grid[:, 1] / max(H - 1, 1) - 1], dim=-1)
    xr = x.detach().clone().requires_grad_(True)
    yr = F.grid_sample(xr, grid, align_corners=False, padding_mode="zeros")
    assert _rel(y, yr) < 1e-5
    gy = torch.randn(y.shape, generator=g).cuda()
    y.backward(gy)
    yr.backward(gy)
    assert _rel(x.grad, xr.grad) < 1e-5
    # fbcheck / temporal loss: the same kernels as the module API
    bflow = (torch.randn(2, 2, 24, 32, generator=g) * 2).cuda()
    assert torch.equal(torch.ops.vst.fbcheck(flow, bflow), flowtools.fbcCheckTorch(flow, bflow))
    a = torch.randn(2, 3, 24, 32, generator=g).cuda().requires_grad_(True)
    b = torch.randn(2, 3, 24, 32, generator=g).cuda().requires_grad_(True)
    mask = (torch.rand(2, 1, 24, 32, generator=g) > 0.3).float().cuda()
    loss = torch.ops.vst.temporal_loss(a, b, flow, mask, 10.0)
    ar, br = a.detach().clone().requires_grad_(True), b.detach().clone().requires_grad_(True)
    lr = ((mask * (br - flowtools.warp(ar, flow))) ** 2).mean() * 10.0
    assert abs(float(loss) - float(lr)) <= 1e-5 * abs(float(lr))
    loss.backward()
    lr.backward()
    assert _rel(a.grad, ar.grad) < 1e-5 and _rel(b.grad, br.grad) < 1e-5
    f = torch.randn(2, 64, 8, 8, generator=g).cuda().requires_grad_(True)
    G = torch.ops.vst.gram(f)
    fr = f.detach().clone().requires_grad_(True)
    Gr = torch.bmm(fr.flatten(2), fr.flatten(2).transpose(1, 2)) / 64
    assert _rel(G, Gr) < 2e-5
    dG = torch.randn(G.shape, generator=g).cuda()
    G.backward(dG)
    Gr.backward(dG)
    assert _rel(f.grad, fr.grad) < 2e-5
    # Adam: one step vs torch.optim.Adam
    p = torch.randn(1000, generator=g).cuda()
    gr = torch.randn(1000, generator=g).cuda()
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    pt = torch.nn.Parameter(p.clone())
    opt = torch.optim.Adam([pt], lr=2e-4, betas=(0.5, 0.999))
    pt.grad = gr.clone()
    opt.step()
    torch.ops.vst.adam_(p, gr, m, v, 2e-4, 0.5, 0.999, 1e-8, 1)
    assert _rel(p, pt.detach()) < 1e-6


@pytest.mark.gpu
def test_conv2d_backward_skips_unneeded_gemms(gpu_fp32_math):
    """a frozen weight gets no weight-gradient GEMM (and no dw), an input without
    requires_grad no data-gradient conv; the remaining gradients are unchanged."""
    from unittest import mock
    from gbvst import ops
    g = torch.Generator().manual_seed(9)
    x = torch.randn(2, 16, 12, 12, generator=g).cuda()
    w = (torch.randn(32, 16, 3, 3, generator=g) * 0.05).cuda()
    b = (torch.randn(32, generator=g) * 0.1).cuda()
    xr, wr, br = x.clone().requires_grad_(True), w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    F.conv2d(F.pad(xr, (1,) * 4, mode="reflect"), wr, br).sum().backward()
    xg = x.clone().requires_grad_(True)
    bg = b.clone().requires_grad_(True)
    with mock.patch.object(ops, "conv2d_wgrad", side_effect=AssertionError("wgrad ran")):
        torch.ops.vst.conv2d(xg, w, bg, 1, 1, "reflect").sum().backward()
    assert _rel(xg.grad, xr.grad) < 2e-5 and _rel(bg.grad, br.grad) < 1e-5
    wg = w.clone().requires_grad_(True)
    with mock.patch.object(ops, "conv2d_tfwd", side_effect=AssertionError("dgrad ran")):
        torch.ops.vst.conv2d(x, wg, None, 1, 1, "reflect").sum().backward()
    assert _rel(wg.grad, wr.grad) < 2e-5
