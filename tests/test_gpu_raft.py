"""GPU parity of RAFT inference (SURVEY §8 A19 + §8f rank 3): gbvst.raft against the reference RAFT's
own outputs (tests/golden/raft_small.npz) and the pinned CPU oracle (oracle/raft_ref.py), plus
its glue kernels against stock torch on the CPU.

Tolerances (relative to max|ref|): glue kernels 1e-6 (element-wise; sigmoid/tanh/exp differ from
ATen's by a few ulp), separable-padding convs 2e-5 (bf16x6 / fp32 arithmetic); encoder features
1e-4; flows after 3-6 GRU iterations 1e-3 (the iteration feeds flow back into the bilinear
correlation lookup, so per-conv rounding compounds; north_star's 1e-3 bound)."""
import argparse

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import prng, raft_ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def gb():
    import gbvst
    gbvst._lib.load()
    return gbvst


def _rel(got, ref):
    got = got.detach().double().cpu().numpy() if torch.is_tensor(got) else np.asarray(got, np.float64)
    ref = ref.detach().double().cpu().numpy() if torch.is_tensor(ref) else np.asarray(ref, np.float64)
    assert got.shape == ref.shape, (got.shape, ref.shape)
    return float(np.abs(got - ref).max() / (np.abs(ref).max() + 1e-30))


def _model(base=1300):
    from gbvst import raft
    m = raft.RAFT(argparse.Namespace(small=False))
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    sd = raft_ref.raft_weights(shapes, base)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    return m.to(DEV).eval(), {k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}


@pytest.mark.parametrize("k,pad", [((1, 5), (0, 2)), ((5, 1), (2, 0)), ((3, 3), (1, 1))])
def test_conv_separate_padding(gb, conv_math, k, pad):
    from gbvst import ops
    x = torch.randn(2, 64, 9, 13)
    w = torch.randn(48, 64, *k) * 0.1
    b = torch.randn(48) * 0.1
    ref = F.conv2d(x, w, b, padding=pad)
    xp = ops.nchw_to_nhwc(x.to(DEV))
    wp = ops.weight_pack(w.to(DEV), ops.PACK_FWD)
    y = ops.conv2d_fwd_hw(xp, wp, b.to(DEV), 48, k[0], k[1], 1, pad[0], pad[1])
    from conftest import CONV_TOL
    assert _rel(ops.nhwc_to_nchw(y, 48), ref) < CONV_TOL[conv_math]


def test_glue_kernels(gb):
    from gbvst import ops
    # prep: replicate pad + 2*(x/255)-1
    img = torch.rand(2, 3, 13, 21) * 255
    pads = (1, 2, 0, 3)
    got = ops.raft_prep(img.to(DEV), pads).cpu()
    ref = 2 * (raft_ref.pad_replicate(img, pads) / 255.0) - 1.0
    assert torch.equal(got[..., :3].permute(0, 3, 1, 2), ref) and bool((got[..., 3] == 0).all())
    # add_relu / copy_channels
    a, b = torch.randn(3, 5, 7, 8), torch.randn(3, 5, 7, 8)
    assert torch.equal(ops.add_relu(a.to(DEV), b.to(DEV)).cpu(), torch.relu(a + b))
    dst = torch.zeros(3, 5, 7, 12, device=DEV)
    ops.copy_channels(a.to(DEV), 2, dst, 5, 6)
    ref = torch.zeros(3, 5, 7, 12)
    ref[..., 5:11] = a[..., 2:8]
    assert torch.equal(dst.cpu(), ref)
    # GRU halves
    P, hd = 37, 8
    zr, h, q = torch.randn(P, 2 * hd), torch.randn(P, hd), torch.tanh(torch.randn(P, hd))
    rhx = torch.zeros(P, 3 * hd, device=DEV)
    hx = torch.zeros(P, 3 * hd, device=DEV)
    ops.gru_reset(zr.to(DEV), h.to(DEV), rhx)
    assert _rel(rhx[:, :hd], torch.sigmoid(zr[:, hd:]) * h) < 1e-6
    hd_ = h.to(DEV).clone()
    ops.gru_update(zr.to(DEV), q.to(DEV), hd_, hx)
    z = torch.sigmoid(zr[:, :hd])
    assert _rel(hd_, (1 - z) * h + z * q) < 1e-6 and torch.equal(hx[:, :hd], hd_)
    # convex upsampling
    B, h8, w8 = 2, 5, 6
    coords1 = raft_ref.coords_grid(B, h8, w8) + torch.randn(B, 2, h8, w8) * 2
    mask = torch.randn(B, 576, h8, w8)
    ref = raft_ref.upsample_flow(coords1 - raft_ref.coords_grid(B, h8, w8), mask)
    got = ops.raft_upsample(coords1.to(DEV).contiguous(), ops.nchw_to_nhwc(mask.to(DEV)))
    assert _rel(got, ref) < 1e-6


def test_raft_vs_reference_golden(gb, golden):
    from gbvst import raft
    g = golden("raft_small")
    m, _ = _model()
    pads = tuple(int(v) for v in g["pads"])
    assert raft.InputPadder(g["img1"].shape).pads == pads
    i1, i2 = torch.from_numpy(g["img1"]).to(DEV), torch.from_numpy(g["img2"]).to(DEV)
    with torch.no_grad():
        low, up = m(i1, i2, iters=6, test_mode=True, pads=pads)
        preds = m(i1, i2, iters=3, test_mode=False, pads=pads)
        up_c = raft.compute_raft(m, i1, i2, it=6)
    assert _rel(low, g["low6"]) < 1e-3
    assert _rel(up, g["up6"]) < 1e-3
    assert _rel(torch.stack(preds), g["preds3"]) < 1e-3
    assert torch.equal(up_c, up)


def test_raft_vs_oracle_larger(gb):
    """Non-divisible frame size (pads on all sides), batch 2, 8 iterations, flow_init."""
    from gbvst import raft
    m, sd = _model(1400)
    img1 = prng.uniform_f32(1401, (2, 3, 131, 170), 0.0, 255.0)
    img2 = np.clip(np.roll(img1, (3, 2), axis=(2, 3)) + prng.normal(1402, img1.shape, std=3.0), 0, 255)
    img2 = img2.astype(np.float32)
    pads = raft.InputPadder(img1.shape).pads
    i1 = raft_ref.pad_replicate(torch.from_numpy(img1), pads)
    i2 = raft_ref.pad_replicate(torch.from_numpy(img2), pads)
    h8, w8 = i1.shape[-2] // 8, i1.shape[-1] // 8
    finit = torch.from_numpy(prng.normal(1403, (2, 2, h8, w8), std=0.5))
    with torch.no_grad():
        low_r, up_r = raft_ref.raft_forward(sd, i1, i2, iters=8, flow_init=finit, test_mode=True)
        low, up = m(torch.from_numpy(img1).to(DEV), torch.from_numpy(img2).to(DEV), iters=8,
                    flow_init=finit.to(DEV), test_mode=True, pads=pads)
    assert _rel(low, low_r) < 1e-3
    assert _rel(up, up_r) < 1e-3


def test_raft_graph_replay_matches_eager(gb):
    """compute_raft's captured-graph replay gives the eager result bit for bit, across replays with
    new inputs and after a weight reload (which must drop the stale graph)."""
    from gbvst import raft
    m, _ = _model(1500)
    x = [torch.from_numpy(prng.uniform_f32(1501 + i, (2, 3, 128, 160), 0.0, 255.0)).to(DEV) for i in range(4)]
    with torch.no_grad():
        for a, b in ((x[0], x[1]), (x[2], x[3])):
            m.use_graphs = False
            ref = raft.compute_raft(m, a, b, it=5)
            m.use_graphs = True
            got = raft.compute_raft(m, a, b, it=5)
            assert torch.equal(got, ref)
        assert len(m._graphs) == 1
        m2, _ = _model(1600)
        m.load_state_dict(m2.state_dict())
        got = raft.compute_raft(m, x[0], x[1], it=5)
        m.use_graphs = False
        assert torch.equal(got, raft.compute_raft(m, x[0], x[1], it=5))


def test_sintel_harness_with_raft_flows(gb):
    """utils/sintel_eval.py harness on the HIP RAFT: computeRAFT (InputPadder + the reference's
    flow_up[:, :, :H, :] cut) and computeTCL on a non-divisible frame size, vs the CPU oracle."""
    from gbvst import networks, raft, sintel_eval
    from oracle import cpu_ref
    m, sd = _model(1700)
    m.use_graphs = True
    H, W = 132, 160  # H % 8 != 0 (padded rows), H % 4 == 0 (shape-preserving G), W % 8 == 0 as on Sintel
    img1 = torch.from_numpy(prng.uniform_f32(1701, (1, 3, H, W), -1.0, 1.0))
    img2 = torch.from_numpy(np.clip(np.roll(img1.numpy(), (1, 2), axis=(2, 3)), -1, 1))
    with torch.no_grad():
        pads = raft_ref.input_pads(img1.shape)
        _, up_r = raft_ref.raft_forward(sd, raft_ref.pad_replicate(img1, pads), raft_ref.pad_replicate(img2, pads),
                                        iters=6, test_mode=True)
        flow = sintel_eval.computeRAFT(m, img1.to(DEV), img2.to(DEV), it=6)
    assert flow.shape == (1, 2, H, W)
    assert _rel(flow, up_r[:, :, :H, :]) < 1e-3
    G = networks.define_G(3, 3, 8, "resnet_9blocks", "instance", False, "normal", 0.02, [0])
    Gr = cpu_ref.RefResnetGenerator(3, 3, 8, 9)
    sdg = prng.init_state_dict(cpu_ref.state_shapes(Gr), base_seed=1702)
    cpu_ref.load_np_state(Gr, sdg)
    G.load_state_dict({k: torch.from_numpy(v) for k, v in sdg.items()})

    class _Net:
        def forward_eval(self, x):
            return G(x)

    fake = torch.from_numpy(prng.uniform_f32(1703, (1, 3, H, W), -1.0, 1.0))
    flow_fn = lambda a, b: sintel_eval.computeRAFT(m, a, b, it=6)  # noqa: E731
    tcl = float(sintel_eval.computeTCL(_Net(), flow_fn, fake.to(DEV), img1.to(DEV), img2.to(DEV)))
    with torch.no_grad():
        ff = raft_ref.raft_forward(sd, raft_ref.pad_replicate(img2, pads), raft_ref.pad_replicate(img1, pads), iters=6,
                                   test_mode=True)[1][:, :, :H, :]
        bf = up_r[:, :, :H, :]
        tcl_ref = float(cpu_ref.tcl(fake, Gr(img2), bf, cpu_ref.fbc_check(ff, bf)))
    assert abs(tcl - tcl_ref) <= 1e-3 * abs(tcl_ref) + 1e-6, (tcl, tcl_ref)
