"""Deterministic warp backward (the atomic-free debug path of the warp's input
gradient, csrc/flow_det.hip) against the fp32-atomic product scatter and against the ordered CPU
restatement (oracle/flow_ref.warp_bwd_ordered, pinned to the reference's grid_sample gradients in
tests/test_oracle_golden.py).  Reference: utils/flowtools.py:18-32, CycleGANCon cycle_gan_model.py:191-204.

Bars: deterministic vs ordered oracle BIT-EXACT (same order, same roundings); deterministic run twice
bit-identical; deterministic vs atomic within 1e-5 x max|gx| (summation order only); a full C2 train
step under the switch bit-identical run to run (every other kernel of the step is atomic-free)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def gb():
    import gbvst
    gbvst._lib.load()
    return gbvst


@pytest.fixture
def det(gb):
    from gbvst import ops
    prev = ops.set_deterministic(True)
    yield ops
    ops.set_deterministic(prev)


def _flow(kind, N, H, W, seed):
    g = torch.Generator().manual_seed(seed)
    if kind == "iid":
        return torch.randn(N, 2, H, W, generator=g) * 3.0
    if kind == "converge":   # everything pulled toward a 6x6 patch: targets receive hundreds of contributions
        ys, xs = torch.meshgrid(torch.arange(H).float(), torch.arange(W).float(), indexing="ij")
        f = torch.stack([W / 2 - xs, H / 2 - ys])[None].repeat(N, 1, 1, 1)
        return f + torch.rand(N, 2, H, W, generator=g) * 6 - 3
    if kind == "oob":
        return (torch.rand(N, 2, H, W, generator=g) * 2 - 1) * 100.0
    return torch.zeros(N, 2, H, W)


@pytest.mark.parametrize("kind", ["iid", "converge", "oob", "zero"])
@pytest.mark.parametrize("C", [4, 64])
@pytest.mark.parametrize("align,masked", [(False, False), (True, False), (False, True)])
def test_warp_bwd_det(det, kind, C, align, masked):
    from oracle import flow_ref
    ops = det
    N, H, W = 2, 37, 53
    g = torch.Generator().manual_seed(11)
    gout = (torch.rand(N, H, W, C, generator=g) * 2 - 1)
    flow = _flow(kind, N, H, W, 12).contiguous()
    gd, fd = gout.to(DEV), flow.to(DEV)
    bwd = ops.warp_masked_bwd_nhwc if masked else ops.warp_bwd_nhwc
    a = bwd(gd, fd, align)
    b = bwd(gd, fd, align)
    assert torch.equal(a, b)
    ref = flow_ref.warp_bwd_ordered(gout.numpy(), flow.numpy(), align=align, masked=masked)
    np.testing.assert_array_equal(a.cpu().numpy(), ref)
    ops.set_deterministic(False)
    at = bwd(gd, fd, align)
    ops.set_deterministic(True)
    scale = max(at.abs().max().item(), 1e-6)
    assert (a - at).abs().max().item() <= 1e-5 * scale


def test_temporal_bwd_det(det):
    """The temporal loss's fake_B gradient: -(ordered scatter of gb), gb unchanged by the switch."""
    from oracle import flow_ref
    ops = det
    N, H, W = 2, 48, 64
    g = torch.Generator().manual_seed(5)
    a = (torch.rand(N, H, W, 4, generator=g) * 2 - 1)
    a[..., 3] = 0
    b = (torch.rand(N, H, W, 4, generator=g) * 2 - 1)
    b[..., 3] = 0
    mask = (torch.rand(N, 1, H, W, generator=g) < 0.8).float()
    flow = _flow("iid", N, H, W, 6).contiguous()
    gout = torch.tensor([1.7])
    A, B, M, Fl, G = (t.to(DEV).contiguous() for t in (a, b, mask, flow, gout))

    def run():
        ga, gbt = torch.zeros_like(A), torch.empty_like(B)
        ops.loss_temporal_bwd(A, B, Fl, M, G, ga, gbt, 10.0, 3)
        return ga, gbt
    ga1, gb1 = run()
    ga2, gb2 = run()
    assert torch.equal(ga1, ga2) and torch.equal(gb1, gb2)
    ref = flow_ref.warp_bwd_ordered(gb1.cpu().numpy(), flow.numpy(), cl=3, negate=True)
    np.testing.assert_array_equal(ga1.cpu().numpy(), ref)
    ops.set_deterministic(False)
    ga3, gb3 = run()
    ops.set_deterministic(True)
    assert torch.equal(gb3, gb1)
    assert (ga3 - ga1).abs().max().item() <= 1e-5 * ga3.abs().max().item()


@pytest.mark.timeout(300)
def test_train_step_bit_identical_under_switch(det):
    """Two C2 optimize_parameters() runs (ngf=ndf=64, 128x128, B=2, pool 0, two steps each) from the
    same weights and batch: every parameter bit-identical under the deterministic switch."""
    from gbvst.cycle_gan_model import CycleGANModel
    from gbvst.options import default_opt
    from oracle import cpu_ref

    data = cpu_ref.synthetic_batch(2, 128, 128, gen=torch.Generator().manual_seed(77))
    init = None
    finals = []
    for _ in range(2):
        torch.manual_seed(0)
        m = CycleGANModel(default_opt(True, pool_size=0, gpu_ids=[0]))
        nets = [m.netG_A, m.netG_B, m.netD_A, m.netD_B]
        if init is None:
            init = [n.flat_param.clone() for n in nets]
        else:
            for n, p in zip(nets, init):
                n.flat_param.copy_(p)
                n.bump_version()
        for _ in range(2):
            m.set_input_fc2((data[0], data[1], data[2], None, data[3], data[4]))
            m.optimize_parameters()
        torch.cuda.synchronize()
        finals.append([n.flat_param.clone() for n in nets])
    for p, q in zip(*finals):
        assert torch.equal(p, q)
