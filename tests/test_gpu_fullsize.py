"""Full-size parity of the secondary paths bench.py times, at the sizes its lines report, against the
CPU oracle on identical counter-PRNG weights and inputs (the cases: oracle/fullsize_cases.py):

* StarGAN C4 (bench ``stargan_train``): one solver.py:315-363 iteration at 256x256, B=4 — D losses
  incl. the WGAN-GP term and every D gradient, then the G step on the SAME D (d_lr = 0).
* RAFT (bench ``raft_sintel``): 1x3x436x1024 frames (InputPadder -> 440 rows), 20 GRU iterations,
  low-res and up-sampled flow, eager and captured-graph replay.
* MoGAN (bench ``mogan_train``, 256x256 B=2, and ``mogan_train_c5``, 1x3x436x1024): an E-step then
  an M-step, ngf = ndf = 64: every loss and every G / D / M gradient, on seeded flows / masks
  (fullsize_cases.mg_flows) injected into both sides; the model's RAFT flows and fb-check mask on one
  real frame pair are checked live against the oracle's.
* C3 (bench ``c3_train``): one CycleGANCon + VGG-19 content / Gram optimize_parameters at
  1x3x436x1024: every loss, every G / D gradient and G_A(probe) after the Adam update.

Reference and bar.  Every quantity is compared with the oracle run in fp64 (the reference's
arithmetic carried exactly, `ref64`), not with its fp32 run: the reference's OWN fp32 result sits
0.2-3 % (norm-wise) from the exact gradients at these sizes, because fp32 rounding flips a few
ReLU / LeakyReLU decisions, each of which moves a whole gradient by ~0.1 %.  No fp32-class
implementation can therefore sit within 2e-3 of another; the HIP path is held to the exact result,
as tightly as the reference itself reaches it:
    losses              |HIP - ref64| <= 1e-3 relative                                 (north_star)
    gradients, tensors  ||HIP - ref64|| <= max(2e-3 / 1e-3, MARGIN * ||ref32 - ref64||)  norm-wise
MARGIN = 3: the HIP forward carries each fp32-equivalent MAC as six MFMA-accumulated split products;
its distance to the exact gradients measured 1.5-2.4x the CPU fp32 path's (StarGAN 1.5, C3 1.9,
MoGAN 2.4) — the forward's rounding decides which ReLU / LeakyReLU elements flip.

The fp64 and fp32 oracle runs take minutes per case on a CPU, so they are made once, here, by
oracle/gen_fullsize_refs.py and committed as tests/golden/fullsize_<case>.npz: per loss both values;
per gradient / tensor ||ref64||, ||ref32 - ref64|| / ||ref64|| and ref64 itself — whole up to 2048
elements, else as a 1024-bucket CountSketch (oracle/sketch.py), from which ||HIP - ref64|| is
estimated to ~2 % (one sigma; SKETCH_SLACK covers 4.5 sigma).  IN-preceded conv biases (exact
gradient 0, rounding noise on every side) are checked for magnitude only.  VST_PARITY_LOG=<dir>
writes every compared quantity's deviations and tolerance as JSON.
"""
import argparse
import os

import numpy as np
import pytest
import torch

from oracle import fullsize_cases as fc

pytestmark = pytest.mark.gpu
DEV = "cuda"
MARGIN = 3.0
# A gradient is ALSO held to its own fp32 deviation: <= max(floor, OWN_MARGIN x ||ref32 - ref64|| of that parameter),
# so a layer-local regression cannot hide under its network's largest fp32 deviation.  Measured (round 5, every case,
# both policies: tools/parity_ratios.py over VST_PARITY_LOG): the largest HIP / own-fp32 ratio above the floor is 12.1
# (C5 MoGAN e_grad|D_B|model.2.weight: 2.26e-3 vs 1.87e-4).
OWN_MARGIN = 20.0
SKETCH_SLACK = 1.1
F64 = torch.float64
FLOORS = {"loss": 1e-3, "grad": 2e-3, "tensor": 1e-3}
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _mrel(a, b):
    a, b = torch.as_tensor(a).double(), torch.as_tensor(b).double()
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


def _fixture(case):
    path = os.path.join(GOLDEN, "fullsize_%s.npz" % case)
    assert os.path.exists(path), "missing %s: run oracle/gen_fullsize_refs.py %s" % (path, case)
    return np.load(path, allow_pickle=False)


def _in_biases():
    """Parameter keys of biases that feed an InstanceNorm in the CycleGAN G / D (magnitude-checked)."""
    keys = ["|model.%d.bias" % i for i in (1, 4, 7, 19, 22, 2, 5, 8)]
    keys += ["|model.%d.conv_block.%d.bias" % (i, j) for i in range(10, 19) for j in (1, 5)]
    return tuple(keys)


def _log_deviations(name, rows):
    import json
    d = os.environ.get("VST_PARITY_LOG")
    if not d:
        return
    from gbvst import ops
    os.makedirs(d, exist_ok=True)
    json.dump({k: {"dev_hip_vs_ref64": h, "dev_ref32_vs_ref64": r, "tol": t} for k, h, r, t in rows},
              open(os.path.join(d, "fullsize_%s_%s.json" % (name, ops.get_conv_math())), "w"), indent=0,
              sort_keys=True)


def _net_of(key):
    """'<phase>grad|<net>|<param>' -> '<phase>grad|<net>' (the network-and-phase group of a gradient)."""
    return key.rsplit("|", 1)[0] if fc.kind(key) == "grad" else key


def _check(name, got, fixture, skip=()):
    """Every quantity of the fixture (the exact reference) against got (HIP).  A gradient's reference
    error scale is the largest fp32 deviation among its network's weights in that phase: the flips that
    move the gradients happen in the network's activations and reach all of its layers, so one
    parameter's own fp32 deviation is a noisy estimate of it (the C5 D_B layers read 1.3-1.9e-4 in the
    fp32 run beside 9e-4 at its first layer, while D alone at that size — test_discriminator_sintel_
    size_vs_fp64 — puts HIP at 1.6-1.9x the fp32 deviation on every layer).  Each gradient is in addition
    held to OWN_MARGIN x its own fp32 deviation (above the floor)."""
    sketched = {n.split(":", 1)[1] for n in fixture.files if n.startswith("S:")}
    devs = fc.deviations(got, fixture)
    scale = {}
    for key, (_, dref) in devs.items():
        if fc.kind(key) == "grad" and not any(key.endswith(s) for s in skip):
            scale[_net_of(key)] = max(scale.get(_net_of(key), 0.0), dref)
    bad, rows = [], []
    for key, (dev, dref) in devs.items():
        if any(key.endswith(s) for s in skip):
            continue
        kind = fc.kind(key)
        ref_err = scale.get(_net_of(key), dref) if kind == "grad" else dref
        tol = FLOORS[kind] if kind == "loss" else max(FLOORS[kind], MARGIN * ref_err)
        if kind == "grad":  # the layer-local bound (OWN_MARGIN)
            tol = min(tol, max(FLOORS[kind], OWN_MARGIN * dref))
        if key in sketched:
            tol *= SKETCH_SLACK
        rows.append((key, dev, dref, tol))
        if not dev <= tol:
            bad.append((key, dev, dref, tol))
    _log_deviations(name, rows)
    assert rows and not bad, bad[:12]


def _check_in_biases(grads):
    for name, d in grads.items():
        for k, g in d.items():
            if any(("|" + k).endswith(s) for s in _in_biases()):
                assert g.abs().max().item() < 1e-3, (name, k)


@pytest.fixture(scope="module")
def gb():
    import gbvst
    gbvst._lib.load()
    return gbvst


# ------------------------------------------------------------------------- StarGAN (config C4)
@pytest.mark.timeout(300)
def test_stargan_full_size_iteration_vs_oracle(gb, prod_math):
    from gbvst import stargan
    from oracle import stargan_ref
    SG = fc.SG
    grads = {}
    sol = stargan.StarGANSolver(image_size=SG["image_size"], c_dim=SG["c_dim"], g_conv_dim=SG["conv_dim"],
                                d_conv_dim=SG["conv_dim"], g_repeat_num=SG["g_repeat"], d_repeat_num=SG["d_repeat"],
                                n_critic=1, d_lr=0.0, device=DEV)
    sol.grad_hook = fc.grab(grads, {id(sol.G): "G", id(sol.D): "D"})
    fc.load(sol.G, stargan_ref.sg_weights(sol.G, fc.SG_SEEDS[0]))
    fc.load(sol.D, stargan_ref.sg_weights(sol.D, fc.SG_SEEDS[1]))
    x, lo, lt, alpha = fc.sg_inputs()
    losses = {k: float(v) for k, v in sol.train_step(x, lo, lt, alpha=alpha).items()}
    torch.cuda.synchronize()
    _check("sg", fc.flatten(losses, grads, {}), _fixture("sg"))


# ---------------------------------------------------------------------------- RAFT at Sintel size
RAFT_HW, RAFT_ITERS, RAFT_SEED = (436, 1024), 20, 1410


def _raft_shapes():
    from gbvst import raft
    return {k: tuple(v.shape) for k, v in raft.RAFT(argparse.Namespace(small=False)).state_dict().items()}


def raft_inputs():
    from oracle import prng
    H, W = RAFT_HW
    img1 = prng.uniform_f32(RAFT_SEED + 1, (1, 3, H, W), 0.0, 255.0)
    img2 = np.clip(np.roll(img1, (3, 2), axis=(2, 3)) + prng.normal(RAFT_SEED + 2, img1.shape, std=3.0), 0, 255)
    return torch.from_numpy(img1), torch.from_numpy(img2.astype(np.float32))


def raft_oracle(dtype=torch.float32):
    from oracle import raft_ref
    sd = {k: torch.from_numpy(np.asarray(v)).to(dtype)
          for k, v in raft_ref.raft_weights(_raft_shapes(), RAFT_SEED).items()}
    i1, i2 = (t.to(dtype) for t in raft_inputs())
    pads = raft_ref.input_pads(i1.shape)
    with torch.no_grad():
        low, up = raft_ref.raft_forward(sd, raft_ref.pad_replicate(i1, pads), raft_ref.pad_replicate(i2, pads),
                                        iters=RAFT_ITERS, test_mode=True)
    return {"low": low.double(), "up": up.double()}


@pytest.mark.timeout(300)
def test_raft_sintel_size_vs_oracle(gb):
    """Live oracle (fp32 and fp64 RAFT forwards take seconds): max-abs deviation relative to max|ref64|
    within max(1e-3, MARGIN x the fp32 reference's own)."""
    from gbvst import raft
    from oracle import raft_ref
    r32, r64 = raft_oracle(torch.float32), raft_oracle(F64)
    m = raft.RAFT(argparse.Namespace(small=False))
    fc.load(m, raft_ref.raft_weights(_raft_shapes(), RAFT_SEED))
    m = m.to(DEV).eval()
    i1, i2 = (t.to(DEV) for t in raft_inputs())
    pads = raft.InputPadder(i1.shape).pads
    assert pads == raft_ref.input_pads(i1.shape) == (0, 0, 2, 2)
    with torch.no_grad():
        low, up = m(i1, i2, iters=RAFT_ITERS, test_mode=True, pads=pads)
        m.use_graphs = True
        up_g = raft.compute_raft(m, i1, i2, it=RAFT_ITERS)   # the bench's captured-graph path
    assert torch.equal(up_g, up)
    rows = []
    for k, got in (("low", low.cpu()), ("up", up.cpu())):
        dev, dref = _mrel(got, r64[k]), _mrel(r32[k], r64[k])
        rows.append(("tensor|" + k, dev, dref, max(FLOORS["tensor"], MARGIN * dref)))
    _log_deviations("raft", rows)
    assert all(d <= t for _, d, _, t in rows), rows


# ---------------------------------------------------------------------------------- MoGAN steps
def _mg_hip(cfg):
    from gbvst import mogan_model, raft
    from gbvst.options import default_opt
    from oracle import prng, raft_ref
    r = raft.RAFT(argparse.Namespace(small=False))
    fc.load(r, raft_ref.raft_weights(_raft_shapes(), *fc.MG_RAFT))
    opt = default_opt(True, model="mogan", ngf=64, ndf=64, pool_size=0, gpu_ids=[0])
    m = mogan_model.MoGANModel(opt, raft_model=r.to(DEV).eval())
    names = {}
    for name, seed in fc.MG_SEEDS.items():
        net = getattr(m, "net" + name)
        names[id(net)] = name
        shapes = {k: tuple(v.shape) for k, v in net.state_dict().items()}
        fc.load(net, prng.init_state_dict(shapes, base_seed=seed))
    m.set_input_fc2(fc.mg_inputs(cfg))
    return m, names


def _mogan_case(which, name):
    from gbvst import ops
    from oracle import cpu_ref, mogan_ref, raft_ref
    cfg = fc.MG_CFG[which]
    fixture = _fixture("mg" + which)
    m, names = _mg_hip(cfg)
    # (1) the model's RAFT flows (computeRAFT: padded RAFT, unpadded flow) and fb-check mask on the
    #     real frame pair, against the oracle's fp32 RAFT / fbcCheck
    ff = ops.nhwc_to_nchw(m.computeRAFT(m.real_A, m.real_A2), 2)
    bf = ops.nhwc_to_nchw(m.computeRAFT(m.real_A2, m.real_A), 2)
    mask = ops.fbcheck(ff, bf)
    torch.cuda.synchronize()
    rsd = {k: torch.from_numpy(np.asarray(v)) for k, v in raft_ref.raft_weights(_raft_shapes(), *fc.MG_RAFT).items()}
    ref = mogan_ref.RefMoGAN(rsd, ngf=4, ndf=4)
    a, a2 = fc.mg_inputs(cfg)[:2]
    rff, rbf = ref.raft(a, a2), ref.raft(a2, a)
    assert _mrel(ff.cpu(), rff) <= 1e-3 and _mrel(bf.cpu(), rbf) <= 1e-3, (_mrel(ff.cpu(), rff), _mrel(bf.cpu(), rbf))
    rmask = cpu_ref.fbc_check(rff, rbf)
    flips = float((mask.reshape(rmask.shape).cpu() != rmask).double().mean())
    assert flips <= 1e-4, flips
    # (2) the E- and M-step on the injected flows / masks: every loss and gradient
    m.flow_inject = fc.mg_flows(cfg)
    ge, gm = {}, {}
    m.optimize_parameters(fc.grab(ge, names), fc.grab(ge, names), fc.grab(ge, names))
    torch.cuda.synchronize()
    le = {k: float(getattr(m, "loss_" + k)) for k in m.loss_names if hasattr(m, "loss_" + k)}
    m.optimize_parameters(fc.grab(gm, names), fc.grab(gm, names), fc.grab(gm, names))
    torch.cuda.synchronize()
    lm = {k: float(getattr(m, "loss_" + k)) for k in ("AM_A", "AM_B")}
    got = fc.flatten(le, ge, {}, "e_")
    got.update(fc.flatten(lm, gm, {}, "m_"))
    _check(name, got, fixture, skip=_in_biases())
    _check_in_biases(ge)
    _check_in_biases(gm)


@pytest.mark.timeout(300)
def test_mogan_full_size_steps_vs_oracle(gb, prod_math):
    _mogan_case("256", "mogan")


@pytest.mark.timeout(300)
def test_mogan_c5_size_steps_vs_oracle(gb, prod_math):
    """The C5 MoGAN step at its stated 1x3x436x1024 (bench ``mogan_train_c5``)."""
    _mogan_case("c5", "mogan_c5")


# ------------------------------------------------------------------------------------ C3 step
@pytest.mark.timeout(300)
def test_c3_full_size_step_vs_oracle(gb, prod_math):
    from gbvst.cycle_gan_vgg_model import CycleGANVGGModel
    from gbvst.options import default_opt
    from oracle import cpu_ref, prng, style_ref
    m = CycleGANVGGModel(default_opt(True, model="cycle_gan_vgg", pool_size=0, gpu_ids=[0]))
    assert (m.opt.lambda_content, m.opt.lambda_style) == fc.C3_LAMBDA   # the model's defaults (bench)
    m.netVGG.load_state_dict({k: torch.from_numpy(v) for k, v in
                              style_ref.vgg_weights(m.netVGG, fc.C3_VGG, init="fan_out").items()})
    names = {}
    for name, seed in fc.C3_SEEDS.items():
        net = getattr(m, "net" + name)
        names[id(net)] = name
        fc.load(net, prng.init_state_dict(cpu_ref.state_shapes(net), base_seed=seed))
    data, probe = fc.c3_inputs()
    m.set_input_fc2((data[0], data[1], data[2], None, data[3], data[4]))
    grads = {}
    m.optimize_parameters(fc.grab(grads, names), fc.grab(grads, names))
    torch.cuda.synchronize()
    losses = m.get_current_losses()
    # the style term is live at this size (it was 0.0 with the golden's weights)
    assert losses["G_S"] > 0.05 and losses["G_C"] > 0.01, losses
    with torch.no_grad():
        out = m.forward_eval(probe).cpu()
    _check("c3", fc.flatten(losses, grads, {"probe_after_adam": out}), _fixture("c3"), skip=_in_biases())
    _check_in_biases(grads)


# ------------------------------------------------------------ PatchGAN D alone at the Sintel size
@pytest.mark.timeout(300)
def test_discriminator_sintel_size_vs_fp64(gb, prod_math):
    """The PatchGAN discriminator alone (networks.py:538-583) at 2x3x436x1024 — the C3 / C5 D inputs,
    odd intermediate sizes (218 x 512 -> 109 x 256 -> 108 x 255 -> 107 x 254): LSGAN loss against 1,
    every parameter gradient vs the oracle run in fp64 (on the GPU) and in fp32 (CPU);
    no generator in front, so only D's own LeakyReLU decisions can flip."""
    from gbvst import networks
    from oracle import cpu_ref, prng
    sd = prng.init_state_dict(cpu_ref.state_shapes(cpu_ref.RefNLayerDiscriminator(3, 64)), base_seed=1700)
    x = torch.from_numpy(prng.uniform_f32(1701, (2, 3, 436, 1024), -1.0, 1.0))

    def oracle(dtype, dev):
        D = cpu_ref.RefNLayerDiscriminator(3, 64)
        fc.load(D, sd)
        D = D.to(device=dev, dtype=dtype)
        xi = x.to(device=dev, dtype=dtype).requires_grad_(True)
        loss = ((D(xi) - 1.0) ** 2).mean()
        loss.backward()
        g = {k: p.grad.detach().double().cpu() for k, p in D.named_parameters()}
        return float(loss), g, xi.grad.detach().double().cpu()

    l64, g64, x64 = oracle(F64, DEV)
    l32, g32, x32 = oracle(torch.float32, "cpu")
    D = networks.define_D(3, 64, "basic", 3, "instance", "normal", 0.02, [0])
    fc.load(D, sd)
    xi = x.to(DEV).requires_grad_(True)
    loss = ((D(xi) - 1.0) ** 2).mean()
    loss.backward()
    torch.cuda.synchronize()

    def nrel(a, b):
        return float((a.double().cpu() - b).norm() / (b.norm() + 1e-30))
    rows = [("loss", abs(float(loss) - l64) / abs(l64), abs(l32 - l64) / abs(l64), FLOORS["loss"])]
    off = 0
    for k, p in D.named_parameters():   # the HIP nets keep their gradients in one flat buffer
        g = D.flat_grad[off:off + p.numel()].view_as(p)
        off += p.numel()
        if any(("|" + k).endswith(s) for s in _in_biases()):   # exact gradient 0: magnitude only
            assert g.abs().max().item() < 1e-3, k
            continue
        d32 = nrel(g32[k], g64[k])
        rows.append(("grad|" + k, nrel(g, g64[k]), d32, max(FLOORS["grad"], MARGIN * d32)))
    _log_deviations("d_sintel", rows)
    assert all(d <= t for _, d, _, t in rows), [r for r in rows if r[1] > r[3]]
