"""GPU parity of every libvst_hip kernel family against the fp32 CPU reference (stock torch ops on
the same inputs) and against the reference-generated golden fixtures.  Tolerances are written per
test: convs compare with |err| <= tol * max|ref| + 1e-6 with tol = 2e-5 under VST_MATH_F32 (fp32
MFMA is an exact fp32 fma chain; only the summation order differs from the CPU) and 1e-4 under
VST_MATH_BF16X3 (split-operand bf16 products, <= ~2^-16 relative each); elementwise/flow ops 1e-5
absolute."""
import numpy as np
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


def _close(got, ref, tol=2e-5, what=""):
    got = got.detach().float().cpu()
    ref = ref.detach().float().cpu()
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    scale = ref.abs().max().item() + 1e-12
    err = (got - ref).abs().max().item()
    assert err <= tol * scale + 1e-6, f"{what}: max|err|={err:.3e} scale={scale:.3e}"


def _nhwc(x, ops):
    return ops.nchw_to_nhwc(x.to(DEV).contiguous())


def _nchw(y, c, ops):
    return ops.nhwc_to_nchw(y.contiguous(), c).cpu()


CONV_CASES = [
    # name, N, Ci, H, W, Co, k, stride, pad, mode
    ("c7s1_reflect_img", 2, 3, 20, 18, 16, 7, 1, 3, "reflect"),
    ("d_3x3_s2", 2, 16, 16, 20, 32, 3, 2, 1, "zero"),
    ("res_3x3_reflect", 2, 32, 12, 10, 32, 3, 1, 1, "reflect"),
    ("res_wide", 1, 256, 16, 16, 256, 3, 1, 1, "reflect"),
    ("out_c7s1_3", 2, 16, 14, 14, 3, 7, 1, 3, "reflect"),
    ("D_4x4_s2_img", 2, 3, 32, 32, 16, 4, 2, 1, "zero"),
    ("D_4x4_s1", 2, 32, 9, 11, 64, 4, 1, 1, "zero"),
    ("D_head_1", 2, 64, 7, 7, 1, 4, 1, 1, "zero"),
    ("odd_big_M", 3, 8, 37, 29, 72, 3, 1, 1, "zero"),
    # W_out % 4 == 0 stride-1 shapes take the channel-major wgrad path
    ("c7s1_reflect_w4", 2, 3, 20, 16, 16, 7, 1, 3, "reflect"),
    ("res_reflect_w8", 2, 32, 12, 8, 32, 3, 1, 1, "reflect"),
    ("D_4x4_s1_w12", 2, 32, 9, 13, 64, 4, 1, 1, "zero"),
    ("res_wide_w4", 2, 256, 6, 4, 136, 3, 1, 1, "reflect"),
    # stride 2 with W_out % 4 == 0 and W even: channel-major wgrad over column-phase split rows
    ("d_3x3_s2_w8", 2, 16, 16, 16, 32, 3, 2, 1, "zero"),
    ("s2_reflect_w8", 2, 8, 10, 16, 16, 3, 2, 1, "reflect"),
    ("D_4x4_s2_w8_oddHo", 1, 16, 10, 16, 24, 4, 2, 1, "zero"),
    ("s2_p0_w8", 2, 8, 9, 18, 16, 3, 2, 0, "zero"),
]


# forced GEMM tile kinds (fprop/tconv rk kind, -, wgrad kind): every tiling the planners may pick
TILE_SETS = {"auto": (-1, -1, -1), "t128k64": (4, 4, 4), "t64x128": (1, 1, 1), "t64x64": (3, 3, 3),
             "t128x128": (0, 0, 0), "t256x128": (7, -1, -1), "legacy_wgrad": (-1, -1, 8),
             "legacy_wgrad64": (-1, -1, 11)}


@pytest.mark.parametrize("tiles", list(TILE_SETS), ids=list(TILE_SETS))
@pytest.mark.parametrize("case", CONV_CASES, ids=[c[0] for c in CONV_CASES])
def test_conv_fwd_dgrad_wgrad(ops, case, tiles, conv_math):
    ops.debug_set_tiles(*TILE_SETS[tiles])
    try:
        _conv_case(ops, case, CONV_TOL[conv_math])
    finally:
        ops.debug_set_tiles(-1, -1, -1)


def _conv_case(ops, case, tol):
    name, N, Ci, H, W, Co, k, st, pad, mode = case
    x = _g(1, (N, Ci, H, W))
    w = _g(2, (Co, Ci, k, k), 0.1)
    b = _g(3, (Co,), 0.1)
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    xp = F.pad(xr, (pad,) * 4, mode="reflect") if mode == "reflect" else xr
    yr = F.conv2d(xp, wr, br, stride=st, padding=0 if mode == "reflect" else pad)
    gy = _g(4, tuple(yr.shape))
    yr.backward(gy)
    wd = w.to(DEV)
    kc = ops.weight_pack(wd, ops.PACK_FWD)
    ck = ops.weight_pack(wd, ops.PACK_DGRAD)
    bp = torch.zeros(ops.cpad(Co), device=DEV)
    bp[:Co] = b.to(DEV)
    xn = _nhwc(x, ops)
    y = ops.conv2d_fwd(xn, kc, bp, ops.cpad(Co), k, k, st, pad, mode)
    _close(_nchw(y, Co, ops), yr, tol=tol, what=name + " fwd")
    # dgrad
    gyn = _nhwc(gy, ops)
    if mode == "reflect":
        # two routes: padded-grid transposed conv + fold, and the fused reflect-aware gather
        # (stride 1 only, like the C ABI; a strided reflect conv takes the fold route)
        Hpd, Wpd = H + 2 * pad, W + 2 * pad
        dxp = ops.conv2d_tfwd(gyn, ck, None, Hpd, Wpd, xn.shape[-1], k, k, st, 0)
        _close(_nchw(ops.reflect_fold(dxp, pad), Ci, ops), xr.grad, tol=tol, what=name + " dgrad(fold)")
    if mode == "reflect" and st > 1:
        dx = ops.reflect_fold(dxp, pad)
    elif mode == "reflect":
        add = _nhwc(_g(40, (N, Ci, H, W)), ops)
        dx2 = ops.conv2d_tfwd(gyn, ck, None, H, W, xn.shape[-1], k, k, 1, pad, pad_mode="reflect", addend=add)
        _close(_nchw(dx2, Ci, ops) - _nchw(add, Ci, ops), xr.grad, tol=tol, what=name + " dgrad(reflect+addend)")
        dx = ops.conv2d_tfwd(gyn, ck, None, H, W, xn.shape[-1], k, k, 1, pad, pad_mode="reflect")
    else:
        dx = ops.conv2d_tfwd(gyn, ck, None, H, W, xn.shape[-1], k, k, st, pad)
    _close(_nchw(dx, Ci, ops), xr.grad, tol=tol, what=name + " dgrad")
    # wgrad + bias grad (accumulate into a pre-filled buffer to test accumulation)
    dw = torch.full((Co, Ci, k, k), 0.5, device=DEV)
    db = torch.full((Co,), 0.25, device=DEV)
    ops.conv2d_wgrad(xn, gyn, dw, db, k, k, st, pad, mode, Co, Ci, Ci * k * k, k * k, accumulate=True)
    _close(dw.cpu() - 0.5, wr.grad, tol=tol, what=name + " wgrad")
    _close(db.cpu() - 0.25, br.grad, tol=tol, what=name + " bgrad")


@pytest.mark.parametrize("cfg", [(2, 16, 8, 8, 8), (1, 256, 64, 16, 16), (2, 32, 3, 6, 5)])
def test_conv_transpose(ops, cfg, conv_math):
    """ConvTranspose2d(k3, s2, p1, op1) fwd, dgrad (= strided conv) and weight grad."""
    tol = CONV_TOL[conv_math]
    N, Ci, Co, H, W = cfg
    x = _g(5, (N, Ci, H, W))
    w = _g(6, (Ci, Co, 3, 3), 0.1)
    b = _g(7, (Co,), 0.1)
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    yr = F.conv_transpose2d(xr, wr, br, stride=2, padding=1, output_padding=1)
    gy = _g(8, tuple(yr.shape))
    yr.backward(gy)
    wd = w.to(DEV)
    kc = ops.weight_pack(wd, ops.PACK_FWD)
    ck = ops.weight_pack(wd, ops.PACK_DGRAD)
    bp = torch.zeros(ops.cpad(Co), device=DEV)
    bp[:Co] = b.to(DEV)
    xn = _nhwc(x, ops)
    y = ops.conv2d_tfwd(xn, ck, bp, 2 * H, 2 * W, ops.cpad(Co), 3, 3, 2, 1)
    _close(_nchw(y, Co, ops), yr, tol=tol, what="convT fwd")
    gyn = _nhwc(gy, ops)
    dx = ops.conv2d_fwd(gyn, kc, None, xn.shape[-1], 3, 3, 2, 1, "zero")
    _close(_nchw(dx, Ci, ops), xr.grad, tol=tol, what="convT dgrad")
    dw = torch.zeros((Ci, Co, 3, 3), device=DEV)
    ops.conv2d_wgrad(gyn, xn, dw, None, 3, 3, 2, 1, "zero", Ci, Co, Co * 9, 9)
    _close(dw.cpu(), wr.grad, tol=tol, what="convT wgrad")
    db = torch.zeros(Co, device=DEV)
    ops.channel_sum(gyn, db, Co)
    _close(db.cpu(), br.grad, what="convT bgrad")


@pytest.mark.parametrize("act", ["relu", "lrelu", "none"])
def test_instnorm_act(ops, act):
    N, C, H, W = 2, 64, 24, 20
    x = _g(9, (N, C, H, W), 2.0) + 0.5
    res = _g(10, (N, C, H, W))
    xr = x.clone().requires_grad_(True)
    yr = F.instance_norm(xr, eps=1e-5)
    if act == "relu":
        yr = F.relu(yr)
    elif act == "lrelu":
        yr = F.leaky_relu(yr, 0.2)
    outr = yr + res if act == "none" else yr
    gy = _g(11, (N, C, H, W))
    outr.backward(gy)
    xn = _nhwc(x, ops)
    s = ops.instnorm_stats(xn)
    y = ops.instnorm_act_fwd(xn, s, act, 0.2, residual=_nhwc(res, ops) if act == "none" else None)
    _close(_nchw(y, C, ops), outr, tol=1e-5, what="IN fwd")
    db = torch.full((C,), 0.5, device=DEV)
    dx = ops.instnorm_act_bwd(_nhwc(gy, ops), xn, s, act, 0.2, db=db)
    _close(_nchw(dx, C, ops), xr.grad, tol=1e-5, what="IN bwd")
    # bias gradient of the conv feeding the IN = per-channel sum of dx (exactly 0 in exact math)
    ref_db = xr.grad.sum(dim=(0, 2, 3)).double()
    assert (db.cpu().double() - 0.5 - ref_db).abs().max().item() < 1e-5 * xr.grad.abs().sum().item() / C


def test_warp_golden(ops, golden):
    g = golden("warp")
    for case in ("zero", "int", "frac", "oob", "h1", "w1"):
        x = torch.from_numpy(g[f"{case}_x"])
        flow = torch.from_numpy(g[f"{case}_flow"]).to(DEV)
        C = x.shape[1]
        y = ops.warp_nhwc(_nhwc(x, ops), flow)
        # bit-exact: flow.hip rounds exactly like ATen's CPU grid sampler (fma where it fuses)
        np.testing.assert_array_equal(_nchw(y, C, ops).numpy(), g[f"{case}_y"], err_msg=case)
        gx = ops.warp_bwd_nhwc(_nhwc(torch.from_numpy(g[f"{case}_gout"]), ops), flow)
        np.testing.assert_allclose(_nchw(gx, C, ops).numpy(), g[f"{case}_dx"], atol=1e-5, err_msg=case)


def test_fbcheck_golden(ops, golden):
    """Bit-exact {0,1} mask against the reference's own masks (flow.hip evaluates every weight,
    norm and threshold with the same separately rounded fp32 operations as torch's CPU path)."""
    g = golden("fbc")
    for case in ("cons", "incons"):
        m = ops.fbcheck(torch.from_numpy(g[f"{case}_ff"]).to(DEV), torch.from_numpy(g[f"{case}_bf"]).to(DEV))
        got = m.cpu().numpy()
        assert (got != g[f"{case}_mask"]).sum() == 0, case


def test_fbcheck_exact_vs_oracle(ops):
    """Same exactness on larger random flow pairs (near-consistent, inconsistent, quarter-pixel
    flows that put many sample points on exact pixel positions) against the CPU oracle."""
    from oracle import cpu_ref
    gen = torch.Generator().manual_seed(31)
    for t in range(6):
        ff = torch.randn(2, 2, 96, 128, generator=gen) * 3
        bf = -ff + torch.randn(2, 2, 96, 128, generator=gen) * 0.3 * (t % 3)
        if t >= 3:
            ff, bf = torch.round(ff * 4) / 4, torch.round(bf * 4) / 4
        ref = cpu_ref.fbc_check(ff, bf)
        got = ops.fbcheck(ff.to(DEV).contiguous(), bf.to(DEV).contiguous()).cpu()
        assert int((got != ref).sum()) == 0, t


def test_losses(ops):
    from oracle import cpu_ref
    N, H, W = 2, 16, 24
    a = _g(12, (N, 3, H, W))
    b = _g(13, (N, 3, H, W))
    flow = _g(14, (N, 2, H, W), 3.0)
    mask = (torch.rand(N, 1, H, W, generator=torch.Generator().manual_seed(15)) < 0.8).float()
    ar, br = a.clone().requires_grad_(True), b.clone().requires_grad_(True)
    lt = cpu_ref.temporal_loss(ar, br, flow, mask, 10.0)
    lt.backward()
    an, bn = _nhwc(a, ops), _nhwc(b, ops)
    fl, mk = flow.to(DEV), mask.to(DEV)
    l = ops.loss_temporal(an, bn, fl, mk, 10.0)
    assert abs(l.item() - lt.item()) <= 1e-5 * abs(lt.item())
    one = torch.ones((), device=DEV)
    ga, gb = torch.zeros_like(an), torch.empty_like(bn)
    ops.loss_temporal_bwd(an, bn, fl, mk, one, ga, gb, 10.0)
    _close(_nchw(ga, 3, ops), ar.grad, 1e-5, "temporal d/da")
    _close(_nchw(gb, 3, ops), br.grad, 1e-5, "temporal d/db")
    ar.grad = None
    l1r = (ar - b).abs().mean() * 5.0
    l1r.backward()
    l1 = ops.loss_l1(an, bn, 5.0)
    assert abs(l1.item() - l1r.item()) <= 1e-5 * l1r.item()
    _close(_nchw(ops.loss_l1_bwd(an, bn, one, 5.0), 3, ops), ar.grad, 1e-6, "l1 grad")
    p = _g(16, (N, 1, 7, 7))
    pr = p.clone().requires_grad_(True)
    mr = ((pr - 1.0) ** 2).mean()
    mr.backward()
    pn = _nhwc(p, ops)
    assert abs(ops.loss_mse_const(pn, 1.0).item() - mr.item()) <= 1e-5 * mr.item()
    _close(_nchw(ops.loss_mse_const_bwd(pn, 1.0, one), 1, ops), pr.grad, 1e-6, "mse grad")


def test_adam_matches_torch(ops):
    n = 1000
    p0 = _g(17, (n,))
    grads = [_g(18 + i, (n,)) * 10 ** (-i) for i in range(4)]
    pr = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([pr], lr=2e-4, betas=(0.5, 0.999))
    p, m, v = p0.to(DEV), torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    for i, gr in enumerate(grads):
        pr.grad = gr.clone()
        opt.step()
        ops.adam_step(p, gr.to(DEV), m, v, 2e-4, 0.5, 0.999, 1e-8, i + 1)
    np.testing.assert_allclose(p.cpu().numpy(), pr.detach().numpy(), rtol=0, atol=1e-7)


@pytest.mark.parametrize("case", [
    # name, N, Ci, H, W, Co, k, pad, mode
    ("res_reflect", 2, 32, 12, 10, 32, 3, 1, "reflect"),
    ("res_wide_reflect", 1, 256, 16, 16, 256, 3, 1, "reflect"),
    ("c7_reflect", 2, 16, 14, 12, 16, 7, 3, "reflect"),
    ("D4_s1_zero", 2, 32, 9, 11, 64, 4, 1, "zero"),
    ("k3_zero", 2, 24, 8, 8, 40, 3, 1, "zero"),
    # 3 output channels: the forward conv over a 4-channel dy (the generator's last layer)
    ("out3_c7_reflect", 2, 16, 14, 12, 3, 7, 3, "reflect"),
    ("out3_k3_zero", 1, 8, 9, 7, 3, 3, 1, "zero"),
], ids=lambda c: c[0])
def test_dgrad_as_fprop(ops, case, conv_math):
    """Stride-1 data gradient computed by the forward-conv kernel over the rotated-tap (IKF) pack,
    + reflect fold / addend, against torch autograd."""
    name, N, Ci, H, W, Co, k, pad, mode = case
    x = _g(61, (N, Ci, H, W)).requires_grad_(True)
    w = _g(62, (Co, Ci, k, k), 0.1)
    xp = F.pad(x, (pad,) * 4, mode="reflect") if mode == "reflect" else x
    y = F.conv2d(xp, w, None, padding=0 if mode == "reflect" else pad)
    gy = _g(63, tuple(y.shape))
    y.backward(gy)
    ikf = ops.weight_pack(w.to(DEV), ops.PACK_IKF)
    add = _g(64, (N, Ci, H, W))
    dx = ops.conv2d_dgrad_s1(_nhwc(gy, ops), ikf, H, W, ops.cpad(Ci), k, pad, mode, addend=_nhwc(add, ops))
    _close(_nchw(dx, Ci, ops) - add, x.grad, tol=CONV_TOL[conv_math], what=name)


@pytest.mark.parametrize("nhw,cs,cl", [(37, 2048, 2048), (1000, 1028, 1025), (5000, 64, 61), (3, 4096, 4000)])
def test_channel_sum_wide(ops, nhw, cs, cl):
    """Per-channel sums over NHWC rows, including channel counts above one reduction block (StarGAN's
    2048-channel discriminator layer runs as channel chunks)."""
    x = _g(71, (nhw, cs))
    db = torch.full((cl,), 0.5, device=DEV)
    ops.channel_sum(x.to(DEV), db, cl, accumulate=True)
    _close(db, x[:, :cl].double().sum(0).float() + 0.5, tol=1e-6, what="accumulate")
    ops.channel_sum(x.to(DEV), db, cl, accumulate=False)
    _close(db, x[:, :cl].double().sum(0).float(), tol=1e-6, what="overwrite")


@pytest.mark.parametrize("co,ci,k,mode", [(3, 64, 7, "reflect"), (2, 64, 7, "reflect"), (3, 32, 3, "zero"),
                                          (1, 16, 5, "reflect")])
def test_tap_conv(ops, conv_math, co, ci, k, mode):
    """Tap-GEMM form of a 'same' conv with <= 4 outputs (generator last layer): forward (+bias, tanh)
    and the weight gradient against torch autograd, reflect and zero padding."""
    N, H, W = 2, 11, 75  # W > 64: several row segments in the LDS tap-sum
    pad = (k - 1) // 2
    x = _g(81, (N, ci, H, W)).requires_grad_(True)
    w = (_g(82, (co, ci, k, k), 0.05)).requires_grad_(True)
    b = _g(83, (co,), 0.1)
    xp = F.pad(x, (pad,) * 4, mode="reflect") if mode == "reflect" else F.pad(x, (pad,) * 4)
    y = torch.tanh(F.conv2d(xp, w, b))
    gy = _g(84, tuple(y.shape))
    y.backward(gy)
    ck = ops.weight_pack(w.detach().to(DEV), ops.PACK_CK)
    bp = torch.zeros(4, device=DEV)
    bp[:co] = b.to(DEV)
    xn = _nhwc(x.detach(), ops)
    yt = ops.tap_conv_fwd(xn, ck, bp, k, pad, mode, act="tanh")
    _close(_nchw(yt, co, ops), y, tol=CONV_TOL[conv_math], what="tap fwd")
    sok = ops.weight_pack(w.detach().to(DEV), ops.PACK_SOK, Op=4)
    yh = ops.tap_conv_fwd_h(xn, sok, bp, k, pad, mode, act="tanh")
    _close(_nchw(yh, co, ops), y, tol=CONV_TOL[conv_math], what="tap fwd (k x 1 conv + column taps)")
    g = ops.act_bwd(_nhwc(gy, ops), yt, "tanh")
    dw = torch.full((co, ci, k, k), 0.25, device=DEV)
    ops.tap_conv_wgrad(xn, g, dw, k, pad, mode, accumulate=True)
    _close(dw.cpu() - 0.25, w.grad, tol=CONV_TOL[conv_math], what="tap wgrad")


@pytest.mark.parametrize("N,ci,H,W,k,xt", [(2, 64, 12, 56, 7, False), (2, 64, 12, 56, 7, True), (3, 32, 9, 60, 3, True),
                                          (2, 64, 256, 256, 7, True)])
def test_tap_conv_wgrad_h(ops, N, ci, H, W, k, xt):
    """Weight gradient of a reflect 'same' conv with <= 4 outputs as the k x 1 conv's (vst_tapshift_planes +
    vst_conv2d_wgrad_pre with pad + 1 + vst_tap_wgrad_scatter_h), x6, against torch autograd and the tap-fold
    route; x's padded channel-major image made by the wgrad or by the IN apply (cp=(pad + 1, reflect))."""
    prev = ops.set_conv_math("bf16x6")
    try:
        co, pad = 3, (k - 1) // 2
        x = _g(101, (N, ci, H, W))
        w = (_g(102, (co, ci, k, k), 0.05)).requires_grad_(True)
        y = F.conv2d(F.pad(x, (pad,) * 4, mode="reflect"), w)
        gy = _g(103, tuple(y.shape))
        y.backward(gy)
        xn, g = _nhwc(x, ops), _nhwc(gy, ops)
        assert ops.tap_conv_wgrad_h_ok(xn, k, pad, "reflect")
        x_t = None
        if xt:  # the IN apply's image of x itself: a = IN(z) with z chosen so that a == x (identity stats)
            st = torch.zeros((N, xn.shape[-1], 2), device=DEV)
            st[..., 1] = 1.0
            a, x_t = ops.instnorm_act_fwd(xn, st, "none", cp=(pad + 1, "reflect", 1))
            assert torch.equal(a, xn)
        dw = torch.full((co, ci, k, k), 0.25, device=DEV)
        ops.tap_conv_wgrad_h(xn, g, dw, k, pad, "reflect", accumulate=True, x_t=x_t)
        _close(dw.cpu() - 0.25, w.grad, tol=CONV_TOL["bf16x6"], what="tap wgrad (k x 1 form)")
        dw0 = torch.zeros((co, ci, k, k), device=DEV)
        ops.tap_conv_wgrad(xn, g, dw0, k, pad, "reflect", accumulate=False)
        _close(dw.cpu() - 0.25, dw0.cpu(), tol=CONV_TOL["bf16x6"], what="vs tap fold")
    finally:
        ops.set_conv_math(prev)


@pytest.mark.parametrize("N,ci,H,W,k,xpl,co", [(2, 64, 12, 56, 7, False, 3), (2, 64, 12, 56, 7, True, 3),
                                              (3, 32, 9, 60, 3, True, 3), (2, 16, 10, 50, 7, True, 3),
                                              (1, 64, 40, 17, 5, True, 3), (2, 32, 12, 56, 7, True, 4),
                                              (1, 8, 11, 13, 7, True, 2), (2, 64, 256, 256, 7, True, 3)])
def test_tap_conv_wgrad_swap(ops, N, ci, H, W, k, xpl, co):
    """Weight gradient of a reflect 'same' conv with <= 4 outputs as the swapped GEMM (vst_tap_wgrad_swap: the
    k x k wgrad of the zero-padded dy against x's reflect-padded frame), x6, against torch autograd and the
    k x 1 form; x's frame planes made by the IN apply (vst_instnorm_act_fwd_planes) or inside the op."""
    prev = ops.set_conv_math("bf16x6")
    try:
        pad = (k - 1) // 2
        x = _g(111, (N, ci, H, W))
        w = (_g(112, (co, ci, k, k), 0.05)).requires_grad_(True)
        y = F.conv2d(F.pad(x, (pad,) * 4, mode="reflect"), w)
        gy = _g(113, tuple(y.shape))
        y.backward(gy)
        xn, g = _nhwc(x, ops), _nhwc(gy, ops)
        assert ops.tap_conv_wgrad_swap_ok(xn, k, pad, "reflect")
        x_pl = None
        if xpl:  # the IN apply's planes of x itself (identity stats)
            st = torch.zeros((N, ci, 2), device=DEV)
            st[..., 1] = 1.0
            a, x_pl = ops.instnorm_act_fwd(xn, st, "none", xpl=(pad, "reflect", ops.tap_swap_geom(W, k)[0]))
            assert torch.equal(a, xn)
        dw = torch.full((co, ci, k, k), 0.25, device=DEV)
        db = torch.full((co,), 0.5, device=DEV)  # the bias gradient from the same pass (vst_tap_wgrad_swap_db)
        ops.tap_conv_wgrad_swap(xn, g, dw, k, pad, "reflect", accumulate=True, x_pl=x_pl, db=db)
        _close(dw.cpu() - 0.25, w.grad, tol=CONV_TOL["bf16x6"], what="tap wgrad (swapped form)")
        _close(db.cpu() - 0.5, gy.sum(dim=(0, 2, 3)), tol=1e-5, what="bias gradient (swapped form)")
        if co == 3 and ops.tap_conv_wgrad_h_ok(xn, k, pad, "reflect"):
            dwh = torch.zeros((co, ci, k, k), device=DEV)
            ops.tap_conv_wgrad_h(xn, g, dwh, k, pad, "reflect", accumulate=False)
            _close(dw.cpu() - 0.25, dwh.cpu(), tol=CONV_TOL["bf16x6"], what="vs k x 1 form")
    finally:
        ops.set_conv_math(prev)


@pytest.mark.parametrize("N,C,H,W,pad,wx,act", [(2, 64, 12, 20, 3, 2, "relu"), (1, 8, 9, 7, 1, 5, "none")])
def test_instnorm_act_fwd_planes(ops, N, C, H, W, pad, wx, act):
    """vst_instnorm_act_fwd_planes: a as vst_instnorm_act_fwd gives it, and the three bf16 planes of its
    reflect-padded frame (wx zero columns per row) sum to that frame exactly (hi = RNE bf16 of it)."""
    y = _g(121, (N, H, W, C)).to(DEV)
    st = torch.stack([_g(122, (N, C)) * 0.1, _g(123, (N, C)).abs() + 0.5], -1).to(DEV)
    a0 = ops.instnorm_act_fwd(y, st, act)
    a, pl = ops.instnorm_act_fwd(y, st, act, xpl=(pad, "reflect", wx))
    assert torch.equal(a, a0)
    fr = F.pad(a0.permute(0, 3, 1, 2), (pad,) * 4, mode="reflect")
    fr = F.pad(fr, (0, wx)).permute(1, 0, 2, 3).reshape(C, -1).cpu()
    P = fr.shape[1]
    p = pl[:, :, :P].float().cpu()
    assert torch.equal(p[0], fr.to(torch.bfloat16).float())
    assert torch.allclose(p[0] + p[1] + p[2], fr, rtol=2.0 ** -22, atol=0)


def test_tap_conv_fwd_h_production(ops, conv_math):
    """The generator's last layer (64 -> 3, 7x7 reflect, tanh) at 256x256 through vst_tapconv_h_fwd vs torch
    fp32 and vs the 1x1-conv + full tap-sum route; the SOK pack built by a PackBatch equals the direct one."""
    N, ci, H, W, co, k = 2, 64, 256, 256, 3, 7
    x = _g(85, (N, ci, H, W))
    w = _g(86, (co, ci, k, k), 0.02)
    b = _g(87, (co,), 0.1)
    ref = torch.tanh(F.conv2d(F.pad(x, (3,) * 4, mode="reflect"), w, b))
    wd = w.to(DEV)
    sok = ops.weight_pack(wd, ops.PACK_SOK, Op=4)
    with ops.PackBatch():
        sok_b = ops.weight_pack(wd, ops.PACK_SOK, Op=4)
    assert torch.equal(sok, sok_b) and torch.equal(sok.vst_split, sok_b.vst_split)
    bp = torch.zeros(4, device=DEV)
    bp[:co] = b.to(DEV)
    xn = _nhwc(x, ops)
    yh = ops.tap_conv_fwd_h(xn, sok, bp, k, 3, "reflect", act="tanh")
    _close(_nchw(yh, co, ops), ref, tol=CONV_TOL[conv_math], what="last layer, row conv + column taps")
    yt = ops.tap_conv_fwd(xn, ops.weight_pack(wd, ops.PACK_CK), bp, k, 3, "reflect", act="tanh")
    _close(yh, yt, tol=CONV_TOL[conv_math], what="vs 1x1 conv + full tap sum")
    assert float(yh[..., 3].abs().max()) == float(torch.tanh(torch.zeros(1))[0])


@pytest.mark.parametrize("N,H,W,pad,mode,act", [(2, 12, 256, 3, "reflect", "tanh"), (3, 9, 256, 6, "zero", "none"),
                                                 (1, 7, 1024, 3, "reflect", "tanh"), (2, 20, 256, 6, "zero", "none"),
                                                 (1, 5, 512, 3, "reflect", "none"), (2, 6, 512, 6, "zero", "none"),
                                                 (2, 10, 1024, 6, "zero", "none"), (1, 13, 1024, 3, "reflect", "none")])
def test_tap64_direct(ops, conv_math, N, H, W, pad, mode, act):
    """The direct 64 -> 4 7x7 tap kernel (conv_tap64.hip, inside vst_tapconv_h_fwd when W | 1024): the last
    layer's forward (reflect 3, tanh) and the first layer's full-correlation data-gradient form (zero pad 6,
    (H+6) x (W+6) output), groups of 4 / 2 rows (W = 256 / 512) or of 4 rows x a 256-column segment (W = 1024,
    five segments per row: the 6-column halo, the reflected / zero-padded row ends) with rows past an image's end,
    vs torch fp32 and vs the 1x1-conv + full tap-sum route."""
    ci, co, k = 64, 3, 7
    x = _g(111, (N, ci, H, W))
    w = _g(112, (co, ci, k, k), 0.02)
    b = _g(113, (co,), 0.1) if act == "tanh" else None
    xp = F.pad(x, (pad,) * 4, mode="reflect") if mode == "reflect" else F.pad(x, (pad,) * 4)
    ref = F.conv2d(xp, w, b)
    ref = torch.tanh(ref) if act == "tanh" else ref
    wd = w.to(DEV)
    bp = None
    if b is not None:
        bp = torch.zeros(4, device=DEV)
        bp[:co] = b.to(DEV)
    xn = _nhwc(x, ops)
    yh = ops.tap_conv_fwd_h(xn, ops.weight_pack(wd, ops.PACK_SOK, Op=4), bp, k, pad, mode, act=act)
    assert yh.shape == (N, H + 2 * pad - 6, W + 2 * pad - 6, 4)
    _close(_nchw(yh, co, ops), ref, tol=CONV_TOL[conv_math], what="tap64 direct vs torch")
    assert float(yh[..., 3].abs().max()) == 0.0
    if pad == (k - 1) // 2:   # the tap-sum route takes 'same' convolutions only
        yt = ops.tap_conv_fwd(xn, ops.weight_pack(wd, ops.PACK_CK), bp, k, pad, mode, act=act)
        _close(yh, yt, tol=CONV_TOL[conv_math], what="vs 1x1 conv + full tap sum")


@pytest.mark.parametrize("ci,co,k,mode", [(3, 64, 7, "reflect"), (2, 64, 7, "reflect"), (3, 32, 3, "zero"),
                                          (3, 64, 7, "zero")])
def test_tap_conv_dgrad(ops, conv_math, ci, co, k, mode):
    """Data gradient of a 'same' conv with <= 4 input channels (generator first layer) as a 1x1 conv
    over all taps + the adjoint tap gather, against torch autograd."""
    N, H, W = 2, 12, 70
    pad = (k - 1) // 2
    x = _g(91, (N, ci, H, W)).requires_grad_(True)
    w = _g(92, (co, ci, k, k), 0.05)
    xp = F.pad(x, (pad,) * 4, mode="reflect") if mode == "reflect" else F.pad(x, (pad,) * 4)
    y = F.conv2d(xp, w)
    gy = _g(93, tuple(y.shape))
    y.backward(gy)
    kc = ops.weight_pack(w.to(DEV), ops.PACK_KC)
    dx = ops.tap_conv_dgrad(_nhwc(gy, ops), kc, k, pad, mode)
    _close(_nchw(dx, ci, ops), x.grad, tol=CONV_TOL[conv_math], what="tap dgrad")
    assert float(dx[..., ci:].abs().max()) == 0.0
    # the k x 1 conv + column-tap route over the full-correlation frame (+ reflect fold / interior crop);
    # the PackBatch-built rotated SOK pack equals the direct one
    sokd = ops.dgrad_sok_pack(w.to(DEV))
    with ops.PackBatch():
        sokd_b = ops.dgrad_sok_pack(w.to(DEV))
    assert torch.equal(sokd, sokd_b)
    dxh = ops.tap_conv_dgrad_h(_nhwc(gy, ops), sokd, k, pad, mode)
    _close(_nchw(dxh, ci, ops), x.grad, tol=CONV_TOL[conv_math], what="tap dgrad (k x 1 conv + column taps)")
    assert float(dxh[..., ci:].abs().max()) == 0.0


@pytest.mark.parametrize("ci,co,h,w", [(128, 64, 9, 11), (256, 128, 8, 8), (64, 32, 5, 70),
                                        (256, 128, 64, 64), (128, 64, 128, 128)])  # the generator's u0 / u1
def test_convT_phases(ops, conv_math, ci, co, h, w):
    """ConvTranspose2d(k3, s2, p1, op1) forward as four phase convs vs torch; the phases stored straight
    into the interleaved output (vst_conv2d_fwd_phase, split-bf16 math) equal the phase images +
    interleave route bit for bit (same GEMMs, other store addresses); all four phases in one launch
    (vst_conv2d_convT_s2, Cx % 32 == 0) vs torch and vs the per-phase launches (its 128x128 / 128x64
    tiles walk K as the planned tiles do for the x6 tiles: equal there; within fp32 rounding else)."""
    x = _g(95, (2, ci, h, w))
    wt = _g(96, (ci, co, 3, 3), 0.05)
    b = _g(97, (co,), 0.1)
    ref = F.conv_transpose2d(x, wt, b, stride=2, padding=1, output_padding=1)
    packs = ops.convT3s2_phase_packs(wt.to(DEV))
    xn = _nhwc(x, ops)
    y = ops.convT3s2_fwd(xn, packs, b.to(DEV), co)
    _close(_nchw(y, co, ops), ref, tol=CONV_TOL[conv_math], what="convT phases")
    prev, prev_g, prev_s = ops.CONVT_DIRECT, ops.CONVT_GROUPED, ops.FWD_HW_SPLITK
    try:
        ops.CONVT_GROUPED = False
        y_ph = ops.convT3s2_fwd(xn, packs, b.to(DEV), co)
        ops.CONVT_DIRECT = False
        ops.FWD_HW_SPLITK = False  # the phase images on the same one-launch plans as the phase stores
        y_il = ops.convT3s2_fwd(xn, packs, b.to(DEV), co)
        ops.FWD_HW_SPLITK = True   # ... and on the small grids' split-K plans: within fp32 rounding
        y_sk = ops.convT3s2_fwd(xn, packs, b.to(DEV), co)
    finally:
        ops.CONVT_DIRECT, ops.CONVT_GROUPED, ops.FWD_HW_SPLITK = prev, prev_g, prev_s
    assert torch.equal(y_ph, y_il)
    _close(y_sk, y_il, tol=5e-6, what="phase images on split-K plans")  # fp32 summation order over K = 4 Ci
    _close(y, y_ph, tol=1e-6, what="grouped vs per-phase launches")


@pytest.mark.parametrize("forced", [False, True], ids=["planned", "t256x128"])
def test_production_resnet_conv(ops, conv_math, forced):
    """The train step's dominant shape as the batched G_A calls run it (N=8 frames, ResnetBlock
    3x3 reflect 256->256 at 64x64) — fwd, the stride-1 dgrad as a forward conv over the padded
    frame (+ reflect fold + residual addend) and the weight gradient — with the tiles the planner
    picks in production (bf16x6 fwd: 256x128 channel-slice-major tiles; bf16x3 dgrad: 128x128 +
    the 64x64 wave-quantisation tail launch at m_base != 0), and with 256x128 forced everywhere."""
    N, C, H, W = 8, 256, 64, 64
    if not forced:
        kf, _ = ops.conv_plan_fwd(N, H, W, C, C, 3, 3, 1, 1, 1, conv_math)
        kd, ms = ops.conv_plan_fwd(N, H, W, C, C, 3, 3, 1, 2, 2, conv_math)
        expect = {"bf16x6": (7, 0), "bf16x3": (0, 0)}.get(conv_math)
        if expect:
            assert kf == expect[0]
        if conv_math in ("bf16x3", "bf16x6"):
            assert kd == (0 if conv_math == "bf16x3" else 7) and ms > 0  # the tail split runs below
    x = _g(101, (N, C, H, W))
    w = _g(102, (C, C, 3, 3), 0.03)
    b = _g(103, (C,), 0.1)
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    yr = F.conv2d(F.pad(xr, (1,) * 4, mode="reflect"), wr, br)
    gy = _g(104, tuple(yr.shape))
    yr.backward(gy)
    tol = CONV_TOL[conv_math]
    ops.debug_set_tiles(7 if forced else -1, -1, -1)
    try:
        wd = w.to(DEV)
        kc = ops.weight_pack(wd, ops.PACK_FWD)
        ikf = ops.weight_pack(wd, ops.PACK_IKF)
        xn = _nhwc(x, ops)
        y = ops.conv2d_fwd(xn, kc, b.to(DEV), C, 3, 3, 1, 1, "reflect")
        _close(_nchw(y, C, ops), yr, tol=tol, what="fwd")
        add = _g(105, (N, C, H, W))
        gyn = _nhwc(gy, ops)
        dx = ops.conv2d_dgrad_s1(gyn, ikf, H, W, C, 3, 1, "reflect", addend=_nhwc(add, ops))
        _close(_nchw(dx, C, ops) - add, xr.grad, tol=tol, what="dgrad")
        dw = torch.zeros((C, C, 3, 3), device=DEV)
        ops.conv2d_wgrad(xn, gyn, dw, None, 3, 3, 1, 1, "reflect", C, C, C * 9, 9, accumulate=False)
        _close(dw.cpu(), wr.grad, tol=tol, what="wgrad")
    finally:
        ops.debug_set_tiles(-1, -1, -1)


@pytest.mark.parametrize("case", [
    # N, H, W, Cx, Cop, R, stride, pad, mode      (fused path / fallback noted)
    (2, 64, 64, 256, 256, 3, 1, 1, "reflect"),   # 256x128 tiles, K-slice order: fused
    (12, 64, 64, 256, 256, 3, 1, 1, "reflect"),  # x6 whole rounds + tail launch: fused in both
    (2, 40, 48, 8, 64, 7, 1, 3, "reflect"),      # 8-channel image edge (tap-major K): fused
    (2, 64, 64, 64, 128, 3, 2, 1, "zero"),       # stride 2: fused
    (2, 33, 33, 128, 256, 4, 1, 1, "zero"),      # 32x32 output = 1024 px: fused
    (2, 34, 34, 64, 128, 4, 1, 1, "zero"),       # 33x33 output (not a multiple of 32 px): fallback
])
def test_conv_fwd_in_stats(ops, case, conv_math):
    """vst_conv2d_fwd_in: the conv output equals vst_conv2d_fwd's, and the InstanceNorm statistics
    folded from its epilogue partials equal vst_instnorm_stats of that output (fp64 partial sums in
    another order: mean and rstd to 1e-6 relative)."""
    N, H, W, Cx, Cop, R, st, pad, mode = case
    x = _g(11, (N, H, W, Cx)).to(DEV)
    w = _g(12, (Cop, Cx, R, R), 0.05).to(DEV)
    b = _g(13, (Cop,), 0.1).to(DEV)
    kc = ops.weight_pack(w, ops.PACK_FWD)
    y_ref = ops.conv2d_fwd(x, kc, b, Cop, R, R, st, pad, mode)
    y, s = ops.conv2d_fwd_in(x, kc, b, Cop, R, R, st, pad, mode)
    assert torch.equal(y, y_ref)
    s_ref = ops.instnorm_stats(y_ref)
    rel = ((s - s_ref).abs() / s_ref.abs().clamp_min(1e-6)).max().item()
    assert rel < 1e-6, rel


@pytest.mark.parametrize("ci,co,h,w", [(64, 128, 16, 20), (128, 256, 8, 8), (4, 64, 32, 32), (64, 128, 64, 64),
                                        (128, 256, 32, 32)])  # the last two: D's layers 2 / 3 at 256^2
@pytest.mark.parametrize("batched", [False, True], ids=["single", "packbatch"])
def test_conv4s2_dgrad_phases(ops, conv_math, ci, co, h, w, batched):
    """Data gradient of the PatchGAN Conv2d(k4, s2, p1) as four 2x2 phase convs + interleave vs
    torch's conv_transpose2d (= the conv's input gradient); packs built singly and through a
    PackBatch (tap maps read straight from the weight)."""
    dy = _g(91, (2, co, h, w))
    wd = _g(92, (co, ci, 4, 4), 0.05)
    ref = F.conv_transpose2d(dy, wd, None, stride=2, padding=1)
    if batched:
        with ops.PackBatch():
            packs = ops.conv4s2_dgrad_phase_packs(wd.to(DEV))
    else:
        packs = ops.conv4s2_dgrad_phase_packs(wd.to(DEV))
    g = ops.conv4s2_dgrad(_nhwc(dy, ops), packs, ops.cpad(ci))
    _close(_nchw(g, ci, ops), ref, tol=CONV_TOL[conv_math], what="conv4s2 dgrad phases")
    # the one-launch route (vst_conv4s2_dgrad, split-bf16, Cy % 32 == 0) vs four phase images + interleave
    prev, ops.C4S2_GROUPED = ops.C4S2_GROUPED, False
    try:
        g_il = ops.conv4s2_dgrad(_nhwc(dy, ops), packs, ops.cpad(ci))
    finally:
        ops.C4S2_GROUPED = prev
    # (other tiles than the per-phase launches pick: another K-accumulation order, fp32-rounding apart)
    _close(g, g_il, tol=CONV_TOL[conv_math], what="one launch vs phase images + interleave")


def test_convT3s2_phase_packs_batched_equal_single(ops):
    """ConvTranspose phase packs recorded in a PackBatch (transposed view + tap maps, no copies)
    equal the copy-based single packs bit for bit, planes included."""
    wt = _g(98, (64, 32, 3, 3), 0.05).to(DEV)
    single = ops.convT3s2_phase_packs(wt)
    with ops.PackBatch():
        batched = ops.convT3s2_phase_packs(wt)
    for s_, b_ in zip(single, batched):
        assert torch.equal(s_, b_) and torch.equal(s_.vst_split, b_.vst_split)


@pytest.mark.parametrize("shape", [(64, 32, 3, 3), (3, 64, 7, 7), (1, 512, 4, 4), (130, 70, 3, 3), (128, 64, 3, 3),
                                   (64, 256, 4, 4), (256, 128, 7, 7)])
def test_pack_batch_equals_single_every_mode(ops, shape):
    """vst_weight_pack_batch (4 elements per lane, float4 / 8-byte plane stores; OK / IK / IKF packs with >= 4 taps
    and a 64-multiple inner extent through an LDS transpose tile) equals the per-element vst_weight_pack_split for
    every pack mode, fp32 pack and the three bf16 planes."""
    w = _g(99, shape, 0.05).to(DEV)
    modes = [ops.PACK_FWD, ops.PACK_DGRAD, ops.PACK_IKF]
    single = [ops.weight_pack(w, m) for m in modes]
    with ops.PackBatch():
        batched = [ops.weight_pack(w, m) for m in modes]
    for s_, b_ in zip(single, batched):
        assert torch.equal(s_, b_) and torch.equal(s_.vst_split, b_.vst_split)


# ----------------------------------------------------- fused IN-backward producers (round 2)
def _split3(x):
    hi = x.to(torch.bfloat16)
    r = x - hi.float()
    mid = r.to(torch.bfloat16)
    lo = (r - mid.float()).to(torch.bfloat16)
    return hi, mid, lo


@pytest.mark.parametrize("N", [1, 8, 12])
def test_apre_dgrad_epi_bit_identical(ops, N):
    """instnorm_act_bwd(planes, apre=True) writes dy ONLY as its NHWC planes (exactly the RNE split of the plain pass's
    dy; the fp32 image stays unwritten); the epi data gradient over those planes (interior A by LDS-DMA, the border
    GEMM from the planes, the split-K tail at N = 12) gives g / IN-backward planes / bias gradient bit-identical to
    the plain route, and its own apre output dy_in is the RNE split of the plain route's dy_in."""
    prev = ops.set_conv_math("bf16x6")
    try:
        H, C = 64, 256
        z = _g(171, (N, H, H, C)).to(DEV)
        s = ops.instnorm_stats(z)
        ga = _g(172, (N, H, H, C)).to(DEV)
        dy0, pl0 = ops.instnorm_act_bwd(ga, z, s, "none", planes=True)
        dy1, pl1 = ops.instnorm_act_bwd(ga, z, s, "none", planes=True, apre=True)
        P = N * H * H  # the channel-major plane rows are padded to vst_cp_ld(P): compare the written part
        assert torch.equal(pl0[:, :, :P], pl1[:, :, :P]) and dy1.vst_planes_only
        for p_, ref in zip(dy1.vst_apl.view(3, -1), _split3(dy0.reshape(-1))):
            assert torch.equal(p_, ref)
        dy1.fill_(float("nan"))  # never read
        w = _g(173, (C, C, 3, 3), 0.05)
        ikf = ops.weight_pack(w.to(DEV), ops.PACK_IKF)
        y_in = _g(174, (N, H, H, C)).to(DEV)
        s_in = ops.instnorm_stats(y_in)
        add = _g(175, (N, H, H, C)).to(DEV)
        db0, db1 = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
        r0 = ops.conv2d_dgrad_refl_in(dy0, ikf, H, H, C, y_in, s_in, "relu", addend=add, db=db0, planes=True)
        r1 = ops.conv2d_dgrad_refl_in(dy1, ikf, H, H, C, y_in, s_in, "relu", addend=add, db=db1, planes=True,
                                      apre=True)
        assert r0 is not None and r1 is not None
        assert torch.equal(r0[0], r1[0])
        assert torch.equal(r0[2][:, :, :P], r1[2][:, :, :P])
        assert torch.equal(db0, db1)
        for p_, ref in zip(r1[1].vst_apl.view(3, -1), _split3(r0[1].reshape(-1))):
            assert torch.equal(p_, ref)
    finally:
        ops.set_conv_math(prev)


@pytest.mark.parametrize("N,H,C,act", [(2, 16, 64, "relu"), (3, 12, 128, "none"), (2, 10, 64, "lrelu")])
def test_instnorm_bwd_planes_exact(ops, N, H, C, act):
    """instnorm_act_bwd(planes=True): dy bit-identical to the plain apply pass, and the planes are
    exactly the RNE three-way bf16 split of dy, channel-major [3][C][vst_cp_ld(P)]."""
    y = _g(1, (N, H, H, C)).to(DEV)
    ga = _g(2, (N, H, H, C)).to(DEV)
    st = ops.instnorm_stats(y)
    dy0 = ops.instnorm_act_bwd(ga, y, st, act, 0.2)
    dy1, pl = ops.instnorm_act_bwd(ga, y, st, act, 0.2, planes=True)
    assert torch.equal(dy0, dy1)
    P = N * H * H
    assert pl.shape[2] == ops.lib().vst_cp_ld(P)
    ref = _split3(dy0.reshape(P, C).t())
    for k in range(3):
        assert torch.equal(pl[k, :, :P], ref[k]), k


@pytest.mark.parametrize("st", [1, 2])
def test_wgrad_with_premade_planes_exact(ops, st):
    """vst_conv2d_wgrad_pre with the IN backward's planes == vst_conv2d_wgrad (x6, bit-identical)."""
    prev = ops.set_conv_math("bf16x6")
    try:
        N, H, Ci, Co = 2, 32, 64, 128
        x = _g(3, (N, H, H, Ci)).to(DEV)
        Ho = H // st
        y = _g(4, (N, Ho, Ho, Co)).to(DEV)
        ga = _g(5, (N, Ho, Ho, Co)).to(DEV)
        s = ops.instnorm_stats(y)
        dy, pl = ops.instnorm_act_bwd(ga, y, s, "relu", planes=True)
        path, _, _ = ops.conv_plan_wgrad(N, H, H, Ci, Ho, Ho, Co, 3, 3, st, "bf16x6")
        assert path == 2
        mode, pad = ("reflect", 1) if st == 1 else ("zero", 1)
        dw0 = torch.zeros(Co, Ci, 3, 3, device=DEV)
        dw1 = torch.zeros(Co, Ci, 3, 3, device=DEV)
        ops.conv2d_wgrad(x, dy, dw0, None, 3, 3, st, pad, mode, Co, Ci, Ci * 9, 9)
        ops.conv2d_wgrad(x, dy, dw1, None, 3, 3, st, pad, mode, Co, Ci, Ci * 9, 9, dy_planes=pl)
        assert torch.equal(dw0, dw1)
    finally:
        ops.set_conv_math(prev)


@pytest.mark.parametrize("st,mode,res", [(1, "reflect", False), (1, "reflect", True), (2, "zero", False)])
def test_instnorm_fwd_cp_and_wgrad_exact(ops, st, mode, res):
    """instnorm_act_fwd(cp=...): a bit-identical to the plain apply, and the x6 weight gradient from
    its padded channel-major image (x_t) bit-identical to the one that makes the copy itself."""
    prev = ops.set_conv_math("bf16x6")
    try:
        N, H, C, Co = 2, 32, 64, 128
        y = _g(11, (N, H, H, C)).to(DEV)
        s = ops.instnorm_stats(y)
        r = _g(12, (N, H, H, C)).to(DEV) if res else None
        act = "none" if res else "relu"
        a0 = ops.instnorm_act_fwd(y, s, act, residual=r)
        a1, at = ops.instnorm_act_fwd(y, s, act, residual=r, cp=(1, mode, st))
        assert torch.equal(a0, a1)
        Ho = H // st
        assert ops.conv_plan_wgrad(N, H, H, C, Ho, Ho, Co, 3, 3, st, "bf16x6")[0] == 2
        dy = _g(13, (N, Ho, Ho, Co)).to(DEV)
        dw0 = torch.zeros(Co, C, 3, 3, device=DEV)
        dw1 = torch.zeros(Co, C, 3, 3, device=DEV)
        ops.conv2d_wgrad(a0, dy, dw0, None, 3, 3, st, 1, mode, Co, C, C * 9, 9)
        ops.conv2d_wgrad(a0, dy, dw1, None, 3, 3, st, 1, mode, Co, C, C * 9, 9, x_t=at)
        assert torch.equal(dw0, dw1)
    finally:
        ops.set_conv_math(prev)


@pytest.mark.parametrize("N,pad", [(8, 2), (12, 1), (12, 2)], ids=["n8_dgrad_frame", "n12_fwd", "n12_dgrad_frame"])
def test_splitk_tail_vs_small_tiles_and_torch(ops, N, pad):
    """The x6 split-K wave-quantisation tail (vst_conv2d_fwd_ws: whole rounds of 256x128 tiles, then
    the remaining rows as ks K-range splits of the same tiles + an in-order reduction with bias and
    the IN partials) against the small-tile tail (no workspace) and torch fp32 on the CPU.  Shapes:
    the ResnetBlock conv as the batched train step runs it (N=12 forward; the 66x66-frame data
    gradient, pad 2, at N=8 / 12)."""
    prev = ops.set_conv_math("bf16x6")
    try:
        C, H = 256, 64
        assert ops.conv_plan_fwd_tail(N, H, H, C, C, 3, 3, 1, pad, "bf16x6") >= 2
        x = _g(21, (N, C, H, H))
        w = _g(22, (C, C, 3, 3), 0.03)
        b = _g(23, (C,), 0.1)
        kc = ops.weight_pack(w.to(DEV), ops.PACK_FWD)
        xn = _nhwc(x, ops)
        y, s = ops.conv2d_fwd_in(xn, kc, b.to(DEV), C, 3, 3, 1, pad, "zero")
        ops.FWD_SPLITK = False
        try:
            y0, s0 = ops.conv2d_fwd_in(xn, kc, b.to(DEV), C, 3, 3, 1, pad, "zero")
        finally:
            ops.FWD_SPLITK = True
        _close(y, y0, tol=2e-6, what="split-K vs small tiles")
        # stats [N][C][{mean, rstd}]: mean error in units of the channel's std, rstd relative
        dm = ((s[..., 0] - s0[..., 0]).abs() * s0[..., 1]).max().item()
        dr = ((s[..., 1] - s0[..., 1]).abs() / s0[..., 1]).max().item()
        assert dm < 1e-5 and dr < 1e-5, (dm, dr)
        yr = F.conv2d(x, w, b, padding=pad)
        _close(_nchw(y, C, ops), yr, tol=CONV_TOL["bf16x6"], what="split-K vs torch fp32")
    finally:
        ops.set_conv_math(prev)


@pytest.mark.parametrize("N,H,Ci,Co,k,pad,mode", [(2, 32, 64, 128, 4, 1, "zero"), (2, 30, 64, 96, 3, 1, "reflect"),
                                                  (3, 21, 32, 72, 3, 1, "zero")])
def test_wgrad_wo_padded_rows(ops, N, H, Ci, Co, k, pad, mode):
    """x6 weight gradients of stride-1 convs whose output width is not a multiple of 8 (PatchGAN's
    31-wide layer) on the split-bf16 kernel via Wo-padded rows (VST_WPLAN_BF_PADW) vs torch fp32."""
    prev = ops.set_conv_math("bf16x6")
    try:
        Ho = H + 2 * pad - k + 1
        assert Ho % 8
        assert ops.conv_plan_wgrad(N, H, H, Ci, Ho, Ho, Co, k, k, 1, "bf16x6")[0] == 4
        x = _g(31, (N, Ci, H, H))
        gy = _g(32, (N, Co, Ho, Ho))
        w = _g(33, (Co, Ci, k, k), 0.05).requires_grad_(True)
        xp = F.pad(x, (pad,) * 4, mode="reflect") if mode == "reflect" else F.pad(x, (pad,) * 4)
        F.conv2d(xp, w).backward(gy)
        dw = torch.zeros(Co, Ci, k, k, device=DEV)
        ops.conv2d_wgrad(_nhwc(x, ops), _nhwc(gy, ops), dw, None, k, k, 1, pad, mode, Co, Ci, Ci * k * k, k * k,
                         accumulate=False)
        _close(dw.cpu(), w.grad, tol=CONV_TOL["bf16x6"], what="Wo-padded wgrad")
    finally:
        ops.set_conv_math(prev)


def test_tap_conv_image_chunks(ops):
    """The tap-GEMM convs run in image chunks sized for the Infinity Cache (ops.TAP_CHUNK_BYTES):
    forward and data gradient bit-identical to one pass over the batch, weight gradient within the
    split-K summation-order tolerance."""
    N, H, Ci = 5, 24, 64
    x = _g(41, (N, H, H, Ci)).to(DEV)
    w = _g(42, (3, Ci, 7, 7), 0.05).to(DEV)
    dy4 = _g(43, (N, H, H, 4)).to(DEV)
    ck = ops.weight_pack(w, ops.PACK_CK)
    prev = ops.TAP_CHUNK_BYTES
    try:
        ops.TAP_CHUNK_BYTES = 0
        y0 = ops.tap_conv_fwd(x, ck, None, 7, 3, "reflect")
        dw0 = torch.zeros(3, Ci, 7, 7, device=DEV)
        ops.tap_conv_wgrad(x, dy4, dw0, 7, 3, "reflect", accumulate=False)
        ops.TAP_CHUNK_BYTES = 2 * H * H * 49 * 16  # two images per chunk: 3 chunks
        y1 = ops.tap_conv_fwd(x, ck, None, 7, 3, "reflect")
        dw1 = torch.zeros(3, Ci, 7, 7, device=DEV)
        ops.tap_conv_wgrad(x, dy4, dw1, 7, 3, "reflect", accumulate=False)
    finally:
        ops.TAP_CHUNK_BYTES = prev
    assert torch.equal(y0, y1)
    _close(dw1, dw0, tol=2e-6, what="chunked tap wgrad")


@pytest.mark.parametrize("mode", ["reflect", "zero"])
def test_tapfold_planes_exact(ops, mode):
    """tap_conv_wgrad with the folded dy written as bf16 planes (vst_tapfold_planes) == the fp32 D +
    plane-copy path, bit for bit (same sums, same RNE splits), under bf16x6."""
    prev_m = ops.set_conv_math("bf16x6")
    prev = ops.TAP_PLANES
    try:
        N, H, Ci = 3, 20, 64
        x = _g(61, (N, H, H, Ci)).to(DEV)
        dy4 = _g(62, (N, H, H, 4)).to(DEV)
        out = []
        for flag in (False, True):
            ops.TAP_PLANES = flag
            dw = _g(63, (3, Ci, 7, 7)).to(DEV)
            ops.tap_conv_wgrad(x, dy4, dw, 7, 3, mode, accumulate=True)
            out.append(dw)
        assert torch.equal(out[0], out[1])
    finally:
        ops.TAP_PLANES = prev
        ops.set_conv_math(prev_m)


def test_tap_wgrad_with_forward_x_image(ops):
    """tap_conv_wgrad reading x's channel-major image written by the forward IN apply
    (instnorm_act_fwd(cp=(0, 'zero', 1))) == making that copy itself (bit-identical)."""
    prev_m = ops.set_conv_math("bf16x6")
    try:
        N, H, Ci = 2, 24, 64
        y = _g(71, (N, H, H, Ci)).to(DEV)
        s = ops.instnorm_stats(y)
        a, at = ops.instnorm_act_fwd(y, s, "relu", cp=(0, "zero", 1))
        dy4 = _g(72, (N, H, H, 4)).to(DEV)
        dw0 = torch.zeros(3, Ci, 7, 7, device=DEV)
        dw1 = torch.zeros(3, Ci, 7, 7, device=DEV)
        ops.tap_conv_wgrad(a, dy4, dw0, 7, 3, "reflect")
        ops.tap_conv_wgrad(a, dy4, dw1, 7, 3, "reflect", x_t=at)
        assert torch.equal(dw0, dw1)
    finally:
        ops.set_conv_math(prev_m)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [
    # N, Ci, H (= W), Co, k, pad: the StarGAN discriminator heads at 256^2 (conv1 3x3 -> 1, conv2 4x4 -> c_dim)
    (8, 2048, 4, 1, 3, 1), (4, 2048, 4, 4, 4, 0), (16, 1024, 2, 4, 2, 0), (3, 512, 5, 3, 3, 1)])
def test_conv_fwd_skinny_split(ops, shape):
    """vst_conv2d_fwd on <= 4 output channels with few output pixels and a long K (skinny_split_k: the K range
    split over workgroups, the slabs summed in order) vs torch; the padded channels stay exactly zero."""
    N, Ci, H, Co, k, pad = shape
    x = _g(151, (N, Ci, H, H))
    w = _g(152, (Co, Ci, k, k), 0.05)
    b = _g(153, (Co,), 0.1)
    kc = ops.weight_pack(w.to(DEV), ops.PACK_FWD)
    bp = torch.zeros(ops.cpad(Co), device=DEV)
    bp[:Co] = b.to(DEV)
    y = ops.conv2d_fwd(_nhwc(x, ops), kc, bp, ops.cpad(Co), k, k, 1, pad, "zero", act="lrelu", slope=0.01)
    yr = F.leaky_relu(F.conv2d(x, w, b, padding=pad), 0.01)
    _close(_nchw(y, Co, ops), yr, tol=2e-5, what="skinny split fwd")
    if Co < 4:
        assert torch.count_nonzero(y[..., Co:]).item() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(2, 512, 31, 31, 1, "zero", "none"), (1, 64, 9, 7, 2, "zero", "lrelu"),
                                   (1, 36, 12, 10, 1, "reflect", "tanh")])
def test_conv_fwd_one_real_channel(ops, shape):
    """vst_conv2d_fwd_co with co_real = 1 (the PatchGAN head: one real channel padded to 4): the
    padded channels equal the 4-channel path's exactly, the real one agrees with it to fp32 rounding
    (the compiler contracts the one-channel sum into a different FMA chain) and matches torch."""
    N, Ci, H, W, st, mode, act = shape
    k, pad = 4, 1
    x = _g(61, (N, Ci, H, W))
    w = _g(62, (1, Ci, k, k), 0.05)
    b = _g(63, (1,), 0.1)
    kc = ops.weight_pack(w.to(DEV), ops.PACK_FWD)
    bp = torch.zeros(ops.cpad(1), device=DEV)
    bp[:1] = b.to(DEV)
    xn = _nhwc(x, ops)
    y4 = ops.conv2d_fwd(xn, kc, bp, ops.cpad(1), k, k, st, pad, mode, act=act, slope=0.2)
    y1 = ops.conv2d_fwd(xn, kc, bp, ops.cpad(1), k, k, st, pad, mode, act=act, slope=0.2, co_real=1)
    assert torch.equal(y1[..., 1:], y4[..., 1:])
    d = (y1[..., 0] - y4[..., 0]).abs().max().item()
    assert d <= 1e-6 * (y4[..., 0].abs().max().item() + 1e-12) * Ci ** 0.5, d
    xp = F.pad(x, (pad,) * 4, mode="reflect") if mode == "reflect" else x
    yr = F.conv2d(xp, w, b, stride=st, padding=0 if mode == "reflect" else pad)
    yr = {"none": yr, "lrelu": F.leaky_relu(yr, 0.2), "tanh": torch.tanh(yr)}[act]
    _close(_nchw(y1, 1, ops), yr, tol=1e-4, what="co_real=1 fwd")


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(2, 3, 8, 8, 64, 7, 1, 3, "reflect"), (1, 3, 4, 5, 16, 7, 1, 3, "reflect"),
                                   (3, 3, 16, 12, 64, 4, 2, 1, "zero"), (2, 1, 9, 7, 24, 3, 1, 1, "zero"),
                                   (1, 4, 33, 17, 32, 5, 1, 2, "reflect")])
def test_conv_fwd_four_channel_input(ops, shape):
    """4-channel inputs on the split-bf16 forward (conv_fprop_bf_k<.., false, 3>): K chunks spanning
    two taps, an odd tap count (the last chunk's missing tap reads zeros), reflect at the smallest
    legal frame; output and the epilogue's InstanceNorm statistics vs torch."""
    N, Ci, H, W, Co, k, st, pad, mode = shape
    x = _g(71, (N, Ci, H, W))
    w = _g(72, (Co, Ci, k, k), 0.1)
    b = _g(73, (Co,), 0.1)
    kc = ops.weight_pack(w.to(DEV), ops.PACK_FWD)
    bp = torch.zeros(ops.cpad(Co), device=DEV)
    bp[:Co] = b.to(DEV)
    xn = _nhwc(x, ops)
    assert xn.shape[-1] == 4
    xp = F.pad(x, (pad,) * 4, mode="reflect") if mode == "reflect" else x
    yr = F.conv2d(xp, w, b, stride=st, padding=0 if mode == "reflect" else pad)
    y = ops.conv2d_fwd(xn, kc, bp, ops.cpad(Co), k, k, st, pad, mode)
    _close(_nchw(y, Co, ops), yr, tol=CONV_TOL["bf16x6"], what="c4 fwd")
    y2, s = ops.conv2d_fwd_in(xn, kc, bp, ops.cpad(Co), k, k, st, pad, mode)
    assert torch.equal(y2, y)
    st_ = s.view(N, ops.cpad(Co), 2)[:, :Co].cpu()
    mean = yr.mean(dim=(2, 3))
    rstd = 1.0 / torch.sqrt(yr.var(dim=(2, 3), unbiased=False) + 1e-5)
    assert ((st_[..., 0] - mean).abs() * rstd).max().item() < 1e-5
    assert ((st_[..., 1] - rstd).abs() / rstd).max().item() < 1e-4


@pytest.mark.parametrize("case", [
    # name, N, C_in(=dx), C_out(=dy), H, W
    ("small", 2, 32, 32, 16, 16),
    ("odd_HW_sum", 3, 64, 64, 13, 20),   # H + W odd: padded border rows
    ("minimal", 1, 32, 64, 4, 4),
    ("cx_not_128", 2, 36, 32, 9, 7),
    ("prod_N8", 8, 256, 256, 64, 64),    # the batched G_A calls: the interior is one whole CU round
    ("prod_N12", 12, 256, 256, 64, 64),  # interior with the split-K tail (addend in the reduction)
], ids=lambda c: c[0])
def test_dgrad_reflect_border(ops, conv_math, case):
    """ReflectionPad2d(1) + 3x3 data gradient as the interior zero-pad-1 conv (+ addend in its
    epilogue) + the padded-border GEMM added into rows / columns 1 and H-2 / W-2
    (vst_conv2d_dgrad_refl), against torch autograd and against the padded-frame + fold path."""
    name, N, Ci, Co, H, W = case
    x = _g(111, (N, Ci, H, W)).requires_grad_(True)
    w = _g(112, (Co, Ci, 3, 3), 0.05)
    y = F.conv2d(F.pad(x, (1,) * 4, mode="reflect"), w)
    gy = _g(113, tuple(y.shape))
    y.backward(gy)
    ikf = ops.weight_pack(w.to(DEV), ops.PACK_IKF)
    add = _g(114, (N, Ci, H, W))
    gyn, addn = _nhwc(gy, ops), _nhwc(add, ops)
    cx = ops.cpad(Ci)
    m = ops._math("bwd")
    used = int(ops.lib().vst_conv2d_dgrad_refl_ws_bytes(N, H, W, Co, cx, m)) > 0
    assert used == (conv_math != "fp32")
    dx = ops.conv2d_dgrad_s1(gyn, ikf, H, W, cx, 3, 1, "reflect", addend=addn)
    _close(_nchw(dx, Ci, ops) - add, x.grad, tol=CONV_TOL[conv_math], what=name)
    prev, ops.DGRAD_BORDER = ops.DGRAD_BORDER, False
    try:
        dx_fold = ops.conv2d_dgrad_s1(gyn, ikf, H, W, cx, 3, 1, "reflect", addend=addn)
    finally:
        ops.DGRAD_BORDER = prev
    _close(dx, dx_fold, tol=CONV_TOL[conv_math], what=name + " vs fold path")
    if cx > Ci:
        assert float(dx[..., Ci:].abs().max()) == 0.0


@pytest.mark.parametrize("shape", [
    # N, H, W, pad, mode, act
    (2, 256, 256, 3, "reflect", "none"),   # the generator's c0 at 256^2: one 256-pixel segment per row
    (1, 436, 1024, 3, "reflect", "none"),  # Sintel width: 4 segments per row
    (2, 250, 250, 6, "zero", "none"),      # zero padding 6 (a data-gradient-style frame), 256-wide rows
    (1, 20, 512, 3, "reflect", "relu"),    # two 256-pixel segments per row
    (3, 20, 18, 3, "reflect", "lrelu"),    # a partial 32-row sub-tile
    (2, 64, 64, 3, "reflect", "tanh"),
    # row-ring runs (conv_c4_ring_k: a block owns per = ceil(T / CUs) consecutive row segments):
    (3, 175, 256, 3, "reflect", "none"),   # per 3, runs crossing image boundaries (a restage mid-run)
    (12, 256, 256, 3, "reflect", "none"),  # per 12: the train step's N=12 c0
], ids=lambda s: "x".join(str(v) for v in s))
def test_conv_c4_direct(ops, shape, conv_math):
    """The patch-staged direct kernel for 4-channel inputs with 64 outputs (conv_c4.hip; the generator's
    7x7 image convs): output vs torch fp32, vs the implicit-GEMM 4-channel route (forced tile), and —
    where Wo % 32 == 0 — the epilogue's InstanceNorm statistics vs torch."""
    if conv_math == "fp32":
        pytest.skip("the direct kernel is a split-bf16 kernel (fp32 runs the [row][k] path)")
    N, H, W, pad, mode, act = shape
    Ci, Co, k = 3, 64, 7
    x = _g(81, (N, Ci, H, W))
    w = _g(82, (Co, Ci, k, k), 0.05)
    b = _g(83, (Co,), 0.1)
    kc = ops.weight_pack(w.to(DEV), ops.PACK_FWD)
    bp = b.to(DEV).contiguous()
    xn = _nhwc(x, ops)
    assert ops.conv_plan_fwd(N, H, W, 4, Co, k, k, 1, pad, pad, conv_math)[0] == ops.PLAN_C4_DIRECT
    xp = F.pad(x, (pad,) * 4, mode="reflect") if mode == "reflect" else x
    yr = F.conv2d(xp, w, b, padding=0 if mode == "reflect" else pad)
    yr = {"none": yr, "relu": F.relu(yr), "lrelu": F.leaky_relu(yr, 0.2), "tanh": torch.tanh(yr)}[act]
    y = ops.conv2d_fwd(xn, kc, bp, Co, k, k, 1, pad, mode, act=act, slope=0.2)
    tol = CONV_TOL[conv_math]
    _close(_nchw(y, Co, ops), yr, tol=tol, what="c4 direct vs torch")
    ops.debug_set_tiles(1, -1, -1)  # the implicit-GEMM 4-channel route (128x64 tiles)
    try:
        y_ig = ops.conv2d_fwd(xn, kc, bp, Co, k, k, 1, pad, mode, act=act, slope=0.2)
    finally:
        ops.debug_set_tiles(-1, -1, -1)
    _close(y, y_ig, tol=tol, what="c4 direct vs implicit GEMM")
    Ho, Wo = y.shape[1], y.shape[2]
    if act == "none" and (Ho * Wo) % 32 == 0:
        y2, s = ops.conv2d_fwd_in(xn, kc, bp, Co, k, k, 1, pad, mode)
        assert torch.equal(y2, y)
        st_ = s.view(N, Co, 2).cpu()
        mean = yr.mean(dim=(2, 3))
        rstd = 1.0 / torch.sqrt(yr.var(dim=(2, 3), unbiased=False) + 1e-5)
        assert ((st_[..., 0] - mean).abs() * rstd).max().item() < 1e-5
        assert ((st_[..., 1] - rstd).abs() / rstd).max().item() < 1e-4


@pytest.mark.parametrize("case", [
    # name, N, C_in (= dx = IN channels), C_out (= dy), H, W, act, addend
    ("small_relu", 2, 256, 256, 16, 16, "relu", True),      # all split-K tiles
    ("all_split_N1", 1, 256, 256, 64, 64, "relu", False),  # the whole conv as split-K tiles (B=1)
    ("prod_N8", 8, 256, 256, 64, 64, "relu", False),       # whole 256x128 rounds
    ("prod_N8_add", 8, 256, 256, 64, 64, "none", True),
    ("prod_N12", 12, 256, 256, 64, 64, "none", True),      # a round + the split-K tail
    ("c3_436x1024", 1, 256, 256, 109, 256, "relu", True),  # one partial round of 256x128 tiles (218 blocks)
], ids=lambda c: c[0])
def test_dgrad_refl_in_epi(ops, case):
    """ops.conv2d_dgrad_refl_in / vst_conv2d_dgrad_refl_in_epi (the IN backward partials taken by the data gradient's GEMM epilogue /
    split-K reduce and the border add's correction slices) vs the separate passes (vst_conv2d_dgrad_refl +
    vst_instnorm_act_bwd_planes): g bit-identical; the IN input gradient, its planes and the bias gradient
    equal up to the partials' fp64 summation order (1e-6 of max); and vs torch autograd."""
    name, N, Ci, Co, H, W, act, with_add = case
    prev = ops.set_conv_math("bf16x6")
    try:
        w = _g(131, (Co, Ci, 3, 3), 0.05)
        ikf = ops.weight_pack(w.to(DEV), ops.PACK_IKF)
        dy = _nhwc(_g(132, (N, Co, H, W)), ops)
        add = _nhwc(_g(133, (N, Ci, H, W)), ops) if with_add else None
        y_in = _nhwc(_g(134, (N, Ci, H, W)), ops)
        s = ops.instnorm_stats(y_in)
        db0 = torch.zeros(Ci, device=DEV)
        db1 = torch.zeros(Ci, device=DEV)
        r = ops.conv2d_dgrad_refl_in(dy, ikf, H, W, Ci, y_in, s, act, addend=add, db=db1, planes=True)
        assert r is not None, name
        g1, dx1, pl1 = r
        g0 = ops.conv2d_dgrad_s1(dy, ikf, H, W, Ci, 3, 1, "reflect", addend=add)
        dx0, pl0 = ops.instnorm_act_bwd(g0, y_in, s, act, db=db0, planes=True)
        assert torch.equal(g1, g0), name
        sc = dx0.abs().max().item()
        assert (dx1 - dx0).abs().max().item() <= 1e-6 * sc, name
        P = N * H * W
        assert (pl1[:, :, :P].float().sum(0) - pl0[:, :, :P].float().sum(0)).abs().max().item() <= 1e-6 * sc, name
        assert (db1 - db0).abs().max().item() <= 1e-6 * max(db0.abs().max().item(), 1e-30), name
        x = _g(135, (N, Ci, H, W)).requires_grad_(True)
        yy = F.conv2d(F.pad(x, (1,) * 4, mode="reflect"), w)
        yy.backward(_nchw(dy, Co, ops))
        gref = x.grad + (_nchw(add, Ci, ops) if with_add else 0)
        _close(_nchw(g1, Ci, ops), gref, tol=CONV_TOL["bf16x6"], what=name + " g")
        yt = _nchw(y_in, Ci, ops).requires_grad_(True)
        a = F.instance_norm(yt, eps=1e-5)
        a = F.relu(a) if act == "relu" else a
        a.backward(_nchw(g1, Ci, ops))
        _close(_nchw(dx1, Ci, ops), yt.grad, tol=1e-4, what=name + " IN bwd")
    finally:
        ops.set_conv_math(prev)


def test_dgrad_refl_in_epi_unsupported(ops):
    """H W not a multiple of 32, or a plan that is neither 256x128 rounds (+ a split-K tail) nor all split-K
    (N = 4 at 64 x 64: one round of 128x128 tiles): the epi route declines (None), the caller keeps the separate
    passes."""
    prev = ops.set_conv_math("bf16x6")
    try:
        for (N, C, H, W) in ((2, 64, 13, 20), (4, 256, 64, 64)):
            w = _g(141, (C, C, 3, 3), 0.05)
            ikf = ops.weight_pack(w.to(DEV), ops.PACK_IKF)
            dy = _nhwc(_g(142, (N, C, H, W)), ops)
            y_in = _nhwc(_g(143, (N, C, H, W)), ops)
            s = ops.instnorm_stats(y_in)
            assert ops.conv2d_dgrad_refl_in(dy, ikf, H, W, C, y_in, s, "relu") is None
    finally:
        ops.set_conv_math(prev)


@pytest.mark.parametrize("N,H,W", [(2, 256, 256), (1, 20, 256), (3, 64, 64), (1, 436, 1024), (12, 256, 256)])
def test_c4_dgrad_reflect(ops, N, H, W, conv_math):
    """The last layer's data gradient (ReflectionPad2d(3) + Conv2d(64 -> 3, 7x7), networks.py:365-366)
    as the direct-kernel interior conv + vst_c4_dgrad_frame, vs torch autograd and vs the padded-frame
    conv + reflect fold route (same products; the frame terms are fp32 FMAs)."""
    if conv_math == "fp32":
        pytest.skip("the direct kernel is a split-bf16 kernel")
    Ci, Co, R, pad = 64, 3, 7, 3
    x = _g(101, (N, Ci, H, W)).to(DEV).requires_grad_(True)
    w = _g(102, (Co, Ci, R, R), 0.05).to(DEV)
    gy = _g(103, (N, Co, H, W)).to(DEV)
    F.conv2d(F.pad(x, (pad,) * 4, mode="reflect"), w).backward(gy)
    ikf = ops.weight_pack(w, ops.PACK_IKF)
    g4 = _nhwc(gy.cpu(), ops)
    assert ops.c4_dgrad_reflect_ok(g4, Ci, R, pad)
    dx = ops.c4_dgrad_reflect(g4, ikf, H, W, Ci, R, pad)
    _close(_nchw(dx, Ci, ops), x.grad, tol=CONV_TOL[conv_math], what="c4 dgrad vs torch")
    ref = ops.conv2d_dgrad_s1(g4, ikf, H, W, Ci, R, pad, "reflect")
    _close(dx, ref, tol=CONV_TOL[conv_math], what="c4 dgrad vs frame + fold")
