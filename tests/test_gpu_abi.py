"""The SURVEY §8b spelling of the C ABI (include/vst_hip.h, csrc/abi.hip): vst_conv_desc with
vst_workspace_size and vst_conv2d_{fwd,dgrad,wgrad}_desc for direct and transposed convs, vst_gram,
vst_corr_volume and the renamed loss / warp / Adam entries — each called through ctypes exactly as a
non-Python binder written from §8b would, and compared with stock torch fp32 on the same inputs
(|err| <= 2e-5 * max|ref| + 1e-6 for convs under the fp32-equivalent bf16x6 arithmetic)."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"
X6 = 2  # VST_MATH_BF16X6


@pytest.fixture(scope="module")
def env():
    import gbvst
    from gbvst import _lib, ops
    gbvst._lib.load()
    return _lib, ops


def _g(seed, shape, scale=1.0):
    return torch.randn(*shape, generator=torch.Generator().manual_seed(seed)) * scale


def _close(got, ref, tol=2e-5, what=""):
    got, ref = got.detach().float().cpu(), ref.detach().float().cpu()
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    err = (got - ref).abs().max().item()
    assert err <= tol * ref.abs().max().item() + 1e-6, (what, err)


def _desc(_lib, **kw):
    d = _lib.VstConvDesc()
    d.dilation, d.layout, d.dtype, d.math = 1, 0, 0, X6
    for k, v in kw.items():
        setattr(d, k, v)
    return d


def _rc(_lib, rc):
    _lib.check(rc, "abi")


def _ws(lib, d, op):
    nb = int(lib.vst_workspace_size(ctypes.byref(d), op))
    return torch.empty(max(1, (nb + 3) // 4), device=DEV), nb


@pytest.mark.parametrize("case", [("res_reflect", 2, 32, 16, 16, 32, 3, 1, 1, "reflect"),
                                  ("down_s2", 2, 16, 16, 16, 32, 3, 2, 1, "zero"),
                                  ("D_4x4_s1", 2, 32, 9, 12, 64, 4, 1, 1, "zero")],
                         ids=lambda c: c[0])
def test_conv_desc_fwd_dgrad_wgrad(env, case):
    _lib, ops = env
    lib = _lib.load()
    name, N, Ci, H, W, Co, k, st, pad, mode = case
    x, w, b = _g(1, (N, Ci, H, W)), _g(2, (Co, Ci, k, k), 0.1), _g(3, (Co,), 0.1)
    xr, wr = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    xp = F.pad(xr, (pad,) * 4, mode="reflect") if mode == "reflect" else xr
    yr = F.conv2d(xp, wr, b, stride=st, padding=0 if mode == "reflect" else pad)
    gy = _g(4, tuple(yr.shape))
    yr.backward(gy)
    Cp, Kp = ops.cpad(Ci), ops.cpad(Co)
    d = _desc(_lib, N=N, H=H, W=W, C=Cp, K=Kp, R=k, S=k, stride=st, pad=pad, pad_mode=ops.PAD[mode])
    Ho, Wo = ctypes.c_int(), ctypes.c_int()
    _rc(_lib, lib.vst_conv_desc_out_hw(ctypes.byref(d), ctypes.byref(Ho), ctypes.byref(Wo)))
    assert (Ho.value, Wo.value) == tuple(yr.shape[2:])
    wd = w.to(DEV)
    wok, wik = ops.weight_pack(wd, ops.PACK_OK), ops.weight_pack(wd, ops.PACK_IK)
    bp = torch.zeros(Kp, device=DEV)
    bp[:Co] = b.to(DEV)
    xn = ops.nchw_to_nhwc(x.to(DEV))
    y = torch.empty((N, Ho.value, Wo.value, Kp), device=DEV)
    ws, nb = _ws(lib, d, 0)
    _rc(_lib, lib.vst_conv2d_fwd_desc(ctypes.byref(d), xn.data_ptr(), wok.data_ptr(), wok.vst_split.data_ptr(),
                                      bp.data_ptr(), y.data_ptr(), None, None, ws.data_ptr(), nb,
                                      torch.cuda.current_stream().cuda_stream))
    _close(ops.nhwc_to_nchw(y, Co), yr, what=name + " fwd")
    gyn = ops.nchw_to_nhwc(gy.to(DEV))
    dx = torch.empty((N, H, W, Cp), device=DEV)
    ws, nb = _ws(lib, d, 1)
    _rc(_lib, lib.vst_conv2d_dgrad_desc(ctypes.byref(d), gyn.data_ptr(), wik.data_ptr(), wik.vst_split.data_ptr(),
                                        dx.data_ptr(), ws.data_ptr(), nb, torch.cuda.current_stream().cuda_stream))
    _close(ops.nhwc_to_nchw(dx, Ci), xr.grad, what=name + " dgrad")
    dw = torch.empty((Co, Ci, k, k), device=DEV)
    ws, nb = _ws(lib, d, 2)
    _rc(_lib, lib.vst_conv2d_wgrad_desc(ctypes.byref(d), xn.data_ptr(), gyn.data_ptr(), dw.data_ptr(), Co, Ci, 0,
                                        ws.data_ptr(), nb, torch.cuda.current_stream().cuda_stream))
    _close(dw, wr.grad, what=name + " wgrad")


def test_conv_desc_transposed(env):
    """ConvTranspose2d(k3, s2, p1, op1) as in the generator's up-sampling (networks.py:357-364)."""
    _lib, ops = env
    lib = _lib.load()
    N, Ci, H, W, Co = 2, 32, 8, 8, 16
    x, w, b = _g(11, (N, Ci, H, W)), _g(12, (Ci, Co, 3, 3), 0.1), _g(13, (Co,), 0.1)
    xr, wr = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    yr = F.conv_transpose2d(xr, wr, b, stride=2, padding=1, output_padding=1)
    gy = _g(14, tuple(yr.shape))
    yr.backward(gy)
    d = _desc(_lib, N=N, H=H, W=W, C=Ci, K=Co, R=3, S=3, stride=2, pad=1, pad_mode=0, transposed=1,
              output_padding=1)
    wd = w.to(DEV)
    wik = ops.weight_pack(wd, ops.PACK_IK, transposed=True)   # tfwd operand of the ConvT weight
    wok = ops.weight_pack(wd, ops.PACK_OK)                    # [Ci][Co] seen as a Conv2d weight
    xn = ops.nchw_to_nhwc(x.to(DEV))
    y = torch.empty((N, 2 * H, 2 * W, Co), device=DEV)
    s = torch.cuda.current_stream().cuda_stream
    _rc(_lib, lib.vst_conv2d_fwd_desc(ctypes.byref(d), xn.data_ptr(), wik.data_ptr(), None,
                                      b.to(DEV).data_ptr(), y.data_ptr(), None, None, None, 0, s))
    _close(ops.nhwc_to_nchw(y, Co), yr, what="convT fwd")
    gyn = ops.nchw_to_nhwc(gy.to(DEV))
    dx = torch.empty((N, H, W, Ci), device=DEV)
    ws, nb = _ws(lib, d, 1)
    _rc(_lib, lib.vst_conv2d_dgrad_desc(ctypes.byref(d), gyn.data_ptr(), wok.data_ptr(), wok.vst_split.data_ptr(),
                                        dx.data_ptr(), ws.data_ptr(), nb, s))
    _close(ops.nhwc_to_nchw(dx, Ci), xr.grad, what="convT dgrad")
    dw = torch.empty((Ci, Co, 3, 3), device=DEV)
    ws, nb = _ws(lib, d, 2)
    _rc(_lib, lib.vst_conv2d_wgrad_desc(ctypes.byref(d), xn.data_ptr(), gyn.data_ptr(), dw.data_ptr(), Co, Ci, 0,
                                        ws.data_ptr(), nb, s))
    _close(dw, wr.grad, what="convT wgrad")


def test_gram_and_corr_volume(env):
    _lib, ops = env
    lib = _lib.load()
    s = torch.cuda.current_stream().cuda_stream
    B, C, h, w = 2, 64, 12, 16
    f = _g(21, (B, C, h, w))
    ref = torch.bmm(f.view(B, C, h * w), f.view(B, C, h * w).transpose(1, 2)) / (h * w)
    fn = ops.nchw_to_nhwc(f.to(DEV))
    G = torch.empty((B, C, C), device=DEV)
    nb = int(lib.vst_gram_ws_bytes(h * w, C))
    ws = torch.empty((nb + 3) // 4, device=DEV)
    _rc(_lib, lib.vst_gram(fn.data_ptr(), G.data_ptr(), B, h * w, C, ws.data_ptr(), nb, X6, s))
    _close(G, ref, what="gram")
    # corr.py:53-60 level 0 + the 4-level pyramid against the Python CorrBlock (itself oracle-checked)
    from gbvst import raft_corr
    D, H, W = 64, 16, 24
    f1, f2 = _g(22, (1, D, H, W)).to(DEV), _g(23, (1, D, H, W)).to(DEV)
    cb = raft_corr.CorrBlock(f1, f2, 4, 4)
    n1, n2 = ops.nchw_to_nhwc(f1), ops.nchw_to_nhwc(f2)
    pyr = torch.empty_like(cb.pyr)
    sq = torch.full((D,), float(torch.sqrt(torch.tensor(D).float())), device=DEV)
    nb = int(lib.vst_corr_volume_ws_bytes(1, H, W, D))
    ws = torch.empty((nb + 3) // 4, device=DEV)
    _rc(_lib, lib.vst_corr_volume(n1.data_ptr(), n2.data_ptr(), pyr.data_ptr(), 1, H, W, D, D, sq.data_ptr(), 4,
                                  ws.data_ptr(), nb, X6, s))
    _close(pyr, cb.pyr, what="corr pyramid vs CorrBlock")
    vol = torch.matmul(f1.cpu().view(D, H * W).t(), f2.cpu().view(D, H * W)) / (D ** 0.5)
    _close(cb.level(0).reshape(H * W, H * W), vol, what="corr level 0")


def test_renamed_loss_warp_adam_entries(env):
    """The §8b names give the same results as the entries they forward to."""
    _lib, ops = env
    lib = _lib.load()
    s = torch.cuda.current_stream().cuda_stream
    N, H, W = 2, 16, 20
    a = ops.nchw_to_nhwc(_g(31, (N, 3, H, W)).to(DEV))
    b = ops.nchw_to_nhwc(_g(32, (N, 3, H, W)).to(DEV))
    flow = (_g(33, (N, 2, H, W)) * 2).to(DEV)
    mask = (torch.rand(N, H, W, generator=torch.Generator().manual_seed(34)) < 0.8).float().to(DEV)
    for masked in (0, 1):
        o1, o2 = torch.empty_like(a), torch.empty_like(a)
        _rc(_lib, lib.vst_warp_bilinear_fwd(a.data_ptr(), flow.data_ptr(), o1.data_ptr(), N, H, W, 4, 0, masked, s))
        fn = lib.vst_warp_masked_fwd if masked else lib.vst_warp_fwd
        _rc(_lib, fn(a.data_ptr(), flow.data_ptr(), o2.data_ptr(), N, H, W, 4, 0, s))
        assert torch.equal(o1, o2)
    part = torch.empty(lib.vst_loss_part_floats(N * H * W), device=DEV)
    l1, l2 = torch.empty(1, device=DEV), torch.empty(1, device=DEV)
    _rc(_lib, lib.vst_masked_sqdiff_mean_fwd(a.data_ptr(), b.data_ptr(), flow.data_ptr(), mask.data_ptr(),
                                             l1.data_ptr(), part.data_ptr(), N, H, W, 4, 3, 10.0, s))
    _rc(_lib, lib.vst_loss_temporal(a.data_ptr(), b.data_ptr(), flow.data_ptr(), mask.data_ptr(), l2.data_ptr(),
                                    part.data_ptr(), N, H, W, 4, 3, 10.0, s))
    assert torch.equal(l1, l2)
    _rc(_lib, lib.vst_l1_mean_fwd(a.data_ptr(), b.data_ptr(), l1.data_ptr(), part.data_ptr(), N * H * W, 4, 3, 10.0, s))
    ref = (ops.nhwc_to_nchw(a, 3) - ops.nhwc_to_nchw(b, 3)).abs().mean() * 10
    assert abs(l1.item() - ref.item()) <= 1e-5 * abs(ref.item())
    _rc(_lib, lib.vst_mse_const_fwd(a.data_ptr(), 1.0, l1.data_ptr(), part.data_ptr(), N * H * W, 4, 3, 1.0, s))
    ref = ((ops.nhwc_to_nchw(a, 3) - 1.0) ** 2).mean()
    assert abs(l1.item() - ref.item()) <= 1e-5 * abs(ref.item())
    # Adam over two tensors == torch.optim.Adam
    ps = [_g(40 + i, (n,)).to(DEV) for i, n in enumerate((1000, 37))]
    gs = [_g(50 + i, (p.numel(),)).to(DEV) for i, p in enumerate(ps)]
    ms, vs = [torch.zeros_like(p) for p in ps], [torch.zeros_like(p) for p in ps]
    tp = [p.detach().cpu().clone().requires_grad_(True) for p in ps]
    opt = torch.optim.Adam(tp, lr=2e-4, betas=(0.5, 0.999))
    for t, g in zip(tp, gs):
        t.grad = g.cpu()
    opt.step()
    arr = lambda ts: (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])  # noqa: E731
    ns = (ctypes.c_long * 2)(*[p.numel() for p in ps])
    _rc(_lib, lib.vst_adam_multi_tensor(arr(ps), arr(gs), arr(ms), arr(vs), ns, 2, 2e-4, 0.5, 0.999, 1e-8, 1, s))
    for p, t in zip(ps, tp):
        _close(p, t.detach(), tol=1e-6, what="adam")
