"""Config C3 on the GPU: the CycleGANCon step + VGG-19 content / Gram loss on fake_B2
(gbvst.cycle_gan_vgg_model), against
  * tests/golden/c3_small.npz — the REFERENCE CycleGANCon model with the reference network.Vgg19
    composed in (oracle/gen_golden_c3.py), ngf=ndf=8, 64x64, B=2, two optimize_parameters steps;
  * the CPU oracle (oracle/c3_ref.py, pinned to that fixture by tests/test_oracle_c3.py) at the
    C3 frame size 1x3x436x1024: generator forward, flow-warp temporal loss, VGG-19 slices, Grams and
    the composed content / style loss terms.
Tolerances: north_star's 1e-3 relative on losses / stylised frames; later steps within max(1e-3,
3x the deviation the reference's own result shows under an fp64 run of the same algorithm or a 1e-6
relative weight perturbation — Adam's early steps are ~lr*sign(g), so rounding-level gradient
differences move near-zero parameters by 2*lr)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
SEEDS = {"G_A": 1300, "G_B": 1400, "D_A": 1500, "D_B": 1600}


@pytest.fixture(scope="module")
def gb():
    import gbvst
    gbvst._lib.load()
    return gbvst


def _oracle(g, dtype, perturb=0.0):
    """The C3 oracle run of the fixture; perturb: scale every G/D weight by (1 + perturb * N(0,1)) —
    a change of the size any other fp32 summation order makes to the forward."""
    from oracle import c3_ref, cpu_ref, prng, style_ref
    m = c3_ref.RefCycleGANConVGG(ngf=8, ndf=8)
    style_ref.load_np(m.vgg, style_ref.vgg_weights(m.vgg, 530))
    m.vgg.to(dtype)
    for name, seed in SEEDS.items():
        net = m.nets()[name]
        sd = prng.init_state_dict(cpu_ref.state_shapes(net), base_seed=seed)
        if perturb:
            sd = {k: (v * (1 + perturb * prng.normal(seed + 17, v.shape))).astype(np.float32) for k, v in sd.items()}
        cpu_ref.load_np_state(net, sd)
        net.to(dtype)
    m.opt_G = torch.optim.Adam(list(m.G_A.parameters()) + list(m.G_B.parameters()), lr=2e-4, betas=(0.5, 0.999))
    m.opt_D = torch.optim.Adam(list(m.D_A.parameters()) + list(m.D_B.parameters()), lr=2e-4, betas=(0.5, 0.999))
    m.set_input_fc2(*(torch.from_numpy(g[k]).to(dtype) for k in ("real_A", "real_A2", "real_B", "mask", "flow")))
    names = [str(n) for n in g["loss_names"]]
    out = []
    for _ in range(g["losses"].shape[0]):
        m.optimize_parameters()
        cur = m.get_current_losses()
        out.append([cur[n] for n in names])
    with torch.no_grad():
        probe = m.G_A(torch.from_numpy(g["probe"]).to(dtype)).double().numpy()
    return np.array(out), probe


def c3_lambdas():
    from oracle import c3_ref
    return c3_ref.LAMBDA_C, c3_ref.LAMBDA_S


def _hip_model(gb, ngf, ndf, pool=0):
    from gbvst.cycle_gan_vgg_model import CycleGANVGGModel
    from gbvst.options import default_opt
    from oracle import cpu_ref, prng, style_ref
    # the golden's composition weights (oracle/c3_ref.LAMBDA_*), not the model's calibrated defaults
    m = CycleGANVGGModel(default_opt(True, model="cycle_gan_vgg", ngf=ngf, ndf=ndf, pool_size=pool, gpu_ids=[0],
                                     lambda_content=c3_lambdas()[0], lambda_style=c3_lambdas()[1]))
    m.netVGG.load_state_dict({k: torch.from_numpy(v) for k, v in style_ref.vgg_weights(m.netVGG, 530).items()})
    for name, seed in SEEDS.items():
        net = getattr(m, "net" + name)
        net.load_state_dict({k: torch.from_numpy(v) for k, v in
                             prng.init_state_dict(cpu_ref.state_shapes(net), base_seed=seed).items()})
    return m


def test_c3_step_vs_reference_golden(gb, golden, train_math):
    g = golden("c3_small")
    m = _hip_model(gb, 8, 8)
    names = [str(n) for n in g["loss_names"]]
    assert names == m.loss_names
    ref = g["losses"]
    l64, p64 = _oracle(g, torch.float64)
    lp, pp = _oracle(g, torch.float32, perturb=1e-6)
    band = np.maximum(np.abs(l64 - ref), np.abs(lp - ref)).__truediv__(np.abs(ref)).max(axis=1)
    data = tuple(torch.from_numpy(g[k]) for k in ("real_A", "real_A2", "real_B"))
    data = data + (None, torch.from_numpy(g["mask"]), torch.from_numpy(g["flow"]))
    for s in range(ref.shape[0]):
        m.set_input_fc2(data)
        m.optimize_parameters()
        cur = m.get_current_losses()
        rel = np.abs(np.array([cur[n] for n in names]) - ref[s]) / np.abs(ref[s])
        tol = 1e-3 if s == 0 else max(1e-3, 3 * band[s])
        assert rel.max() <= tol, (s, dict(zip(names, rel)), band[s])
    with torch.no_grad():
        out = m.forward_eval(torch.from_numpy(g["probe"])).double().cpu().numpy()
    # after two Adam steps (~lr * sign(g) each) the reference's own output moves this much under an
    # fp64 run or a 1e-6 weight perturbation; the HIP run must stay within 3x that band
    dev = max(np.abs(p64 - g["probe_out"]).max(), np.abs(pp - g["probe_out"]).max())
    assert np.abs(out - g["probe_out"]).max() <= max(1e-3, 3 * dev), (np.abs(out - g["probe_out"]).max(), dev)


@pytest.mark.timeout(600)
def test_c3_sintel_size_vs_oracle(gb, infer_math):
    """1x3x436x1024 (the Sintel frame size of C3): G forward, temporal warp loss, VGG-19 slices /
    Grams and the composed C3 loss terms against the CPU oracle on the same inputs and weights."""
    from gbvst import ops, perceptual
    from gbvst.cycle_gan_model import temporal_loss
    from oracle import c3_ref, cpu_ref, prng, style_ref
    H, W = 436, 1024
    m = _hip_model(gb, 64, 64)
    G = cpu_ref.RefResnetGenerator(3, 3, 64, 9)
    cpu_ref.load_np_state(G, prng.init_state_dict(cpu_ref.state_shapes(G), base_seed=SEEDS["G_A"]))
    vgg = style_ref.RefVGG("vgg19")
    style_ref.load_np(vgg, style_ref.vgg_weights(vgg, 530))
    gen = torch.Generator().manual_seed(436)
    a, a2, b, mask, flow = cpu_ref.synthetic_batch(1, H, W, gen=gen)
    flow = flow * 4.0  # the same flow generator scaled x4
    # generator forward (the stylised frames)
    with torch.no_grad():
        fa_ref, fa2_ref = G(a), G(a2)
        fa = m.netG_A(a.to(DEV)).cpu()
    assert (fa - fa_ref).abs().max().item() < 1e-3
    # temporal loss on the reference's stylised frames (isolates the warp kernel at this size)
    lt_ref = cpu_ref.temporal_loss(fa_ref, fa2_ref, flow, mask, 10.0).item()
    lt = temporal_loss(ops.nchw_to_nhwc(fa_ref.to(DEV)), ops.nchw_to_nhwc(fa2_ref.to(DEV)), flow.to(DEV),
                       mask.to(DEV), 10.0).item()
    assert abs(lt - lt_ref) <= 1e-4 * abs(lt_ref), (lt, lt_ref)
    # VGG-19 slices + Grams of the stylised frame and the composed loss terms
    with torch.no_grad():
        f_ref = vgg(c3_ref.vgg_in(fa2_ref))
        c_ref, s_ref = c3_ref.c3_terms(vgg, fa2_ref, a2, b)
        x = ops.nchw_to_nhwc(fa2_ref.to(DEV))
        f = m.vgg_features(x)
        for i, (fi, ri) in enumerate(zip(f, f_ref)):
            got = ops.nhwc_to_nchw(fi.contiguous(), fi.shape[-1]).cpu()
            assert (got - ri).abs().max().item() <= 1e-3 * ri.abs().max().item(), i
            gi = perceptual.gram_nhwc(fi).cpu()
            gr = style_ref.gram_matrix(ri)
            assert (gi - gr).abs().max().item() <= 1e-3 * gr.abs().max().item(), i
        m.fake_B2 = x
        m.real_A2 = ops.nchw_to_nhwc(a2.to(DEV))
        m.real_B = ops.nchw_to_nhwc(b.to(DEV))
        m.extra_G_loss()
    assert abs(m.loss_G_C.item() - c_ref.item()) <= 1e-3 * abs(c_ref.item())
    assert abs(m.loss_G_S.item() - s_ref.item()) <= 1e-3 * abs(s_ref.item())
