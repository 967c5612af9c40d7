"""TEST INFRASTRUCTURE ONLY: the full-size parity cases of tests/test_gpu_fullsize.py — their seeded
inputs and weights, and the oracle runs (fp32 and fp64) whose compact summaries
oracle/gen_fullsize_refs.py commits as tests/golden/fullsize_*.npz.

* StarGAN C4: one solver.py:315-363 iteration at 256x256, c_dim 4, conv_dim 64, 6 / 6 repeats, B=4:
  D losses (WGAN-GP double backward included) and every D gradient, then the G step on the SAME D.
* MoGAN at 256x256 B=2 and at the C5 size 1x3x436x1024: an E-step then an M-step
  (MoGAN/models/cycle_gan_model.py:160-195, 297-331), ngf = ndf = 64, conditioned on seeded flows and
  fb-check masks (mg_flows) so the E / M arithmetic is compared without RAFT's discrete, amplified
  parts (RAFT has its own full-size test; the MoGAN RAFT plumbing is checked live on one pair).
* C3: one CycleGANCon + VGG-19 content / Gram optimize_parameters at 1x3x436x1024 with the model's
  loss weights: every loss, every G / D gradient (before Adam) and G_A(probe) after the Adam update.

A run is flattened to {key: value}: 'loss|name', 'grad|net|param', 'tensor|name' (MoGAN keys carry an
'e_' / 'm_' phase prefix on the kind).
"""
import numpy as np
import torch
import torch.nn.functional as F

from oracle import sketch

F64 = torch.float64
RAW_MAX = 2048            # quantities up to this many elements are stored whole, larger ones as a sketch


def load(net, sd):
    net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    return net


def grab(store, names):
    """grad hook: per network name (names: id(net) -> name), every parameter gradient (fp64, CPU)."""
    def hook(nets):
        for net in nets:
            d = store.setdefault(names[id(net)], {})
            for k, p in net.named_parameters():
                if p.grad is not None:
                    d[k] = p.grad.detach().double().cpu().clone()
    return hook


def flatten(losses, grads, tensors, prefix=""):
    out = {prefix + "loss|" + k: float(v) for k, v in losses.items()}
    for n, d in grads.items():
        for k, g in d.items():
            out[prefix + "grad|%s|%s" % (n, k)] = g
    for k, t in tensors.items():
        out[prefix + "tensor|" + k] = t
    return out


def kind(key):
    return key.split("|", 1)[0].split("_")[-1]


# ------------------------------------------------------------------------- StarGAN (config C4)
SG = dict(image_size=256, c_dim=4, conv_dim=64, g_repeat=6, d_repeat=6, B=4)
SG_SEEDS = (920, 930)


def sg_inputs():
    from oracle import prng
    S, B = SG["image_size"], SG["B"]
    x = torch.from_numpy(prng.uniform_f32(921, (B, 3, S, S), -1.0, 1.0))
    alpha = torch.from_numpy(prng.uniform_f32(922, (B, 1, 1, 1)))
    return x, torch.tensor([0, 1, 2, 3]), torch.tensor([2, 3, 0, 1]), alpha


def sg_oracle(dtype):
    from oracle import stargan_ref
    G = stargan_ref.RefGenerator(SG["conv_dim"], SG["c_dim"], SG["g_repeat"])
    D = stargan_ref.RefDiscriminator(SG["image_size"], SG["conv_dim"], SG["c_dim"], SG["d_repeat"])
    load(G, stargan_ref.sg_weights(G, SG_SEEDS[0])).to(dtype)
    load(D, stargan_ref.sg_weights(D, SG_SEEDS[1])).to(dtype)
    x, lo, lt, alpha = sg_inputs()
    x, alpha = x.to(dtype), alpha.to(dtype)
    d_loss, losses = stargan_ref.d_losses(G, D, x, lo, lt, alpha, SG["c_dim"])
    gd = torch.autograd.grad(d_loss, list(D.parameters()))
    g_loss, parts = stargan_ref.g_losses(G, D, x, lo, lt, SG["c_dim"])
    gg = torch.autograd.grad(g_loss, list(G.parameters()))
    losses.update(parts)
    grads = {"D": {k: g.double() for (k, _), g in zip(D.named_parameters(), gd)},
             "G": {k: g.double() for (k, _), g in zip(G.named_parameters(), gg)}}
    return flatten(losses, grads, {})


# ---------------------------------------------------------------------------------- MoGAN steps
MG_SEEDS = {"G_A": 1530, "G_B": 1531, "D_A": 1532, "D_B": 1533, "M_A": 1534, "M_B": 1535}
MG_RAFT = (1300, 1e-3)
MG_CFG = {"256": dict(B=2, H=256, W=256, seed=1540), "c5": dict(B=1, H=436, W=1024, seed=1560)}
FLOW_KEYS = ("ff_real_A", "bf_real_A", "bf_fake_B", "bf_rec_A", "ff_real_B", "bf_real_B", "bf_fake_A", "bf_rec_B")


def mg_inputs(cfg):
    from oracle import prng
    return [torch.from_numpy(prng.uniform_f32(cfg["seed"] + i, (cfg["B"], 3, cfg["H"], cfg["W"]), -1.0, 1.0))
            for i in range(4)]


def mg_flows(cfg):
    """The conditioning of both forwards (E, M): per FLOW_KEYS entry a smooth field (bicubic upsample of
    a seeded N(0, 2^2) 9x9 grid, SURVEY §8d's generator), per direction a Bernoulli(0.85) mask on a
    32x32 grid (nearest upsample: exact on every machine)."""
    from oracle import prng
    B, H, W, s0 = cfg["B"], cfg["H"], cfg["W"], cfg["seed"] + 100
    out = []
    for ph in range(2):
        d = {}
        for j, k in enumerate(FLOW_KEYS):
            coarse = torch.from_numpy(prng.normal(s0 + 20 * ph + j, (B, 2, 9, 9), std=2.0).astype(np.float32))
            d[k] = F.interpolate(coarse, size=(H, W), mode="bicubic", align_corners=True).contiguous()
        for j, k in enumerate(("mask_A", "mask_B")):
            m = torch.from_numpy((prng.uniform_f32(s0 + 20 * ph + 10 + j, (B, 1, 32, 32)) < 0.85).astype(np.float32))
            d[k] = F.interpolate(m, size=(H, W), mode="nearest").contiguous()
        out.append(d)
    return out


def mg_oracle(cfg, dtype, device="cpu"):
    """E-step then M-step of oracle/mogan_ref.py on mg_flows(cfg): losses and every gradient of each phase
    (device: where torch runs the restatement — the C5 size's fp64 run needs more than this container's
    64 GB, so oracle/gen_fullsize_refs.py runs it on a GPU in fp64)."""
    from oracle import cpu_ref, mogan_ref, prng
    m = mogan_ref.RefMoGAN(None, ngf=64, ndf=64)
    for name, net in m.nets().items():
        cpu_ref.load_np_state(net, prng.init_state_dict(cpu_ref.state_shapes(net), base_seed=MG_SEEDS[name]))
        net.to(device=device, dtype=dtype)
    adam = lambda nets: torch.optim.Adam([p for n in nets for p in n.parameters()], lr=2e-4,  # noqa: E731
                                         betas=(0.5, 0.999))
    m.opt_G, m.opt_D, m.opt_M = adam([m.G_A, m.G_B]), adam([m.D_A, m.D_B]), adam([m.M_A, m.M_B])
    m.inject = [{k: v.to(device=device, dtype=dtype) for k, v in d.items()} for d in mg_flows(cfg)]
    m.set_input_fc2(*(t.to(device=device, dtype=dtype) for t in mg_inputs(cfg)))
    names = {id(n): k for k, n in m.nets().items()}
    ge, gm = {}, {}
    m.optimize_parameters(grab(ge, names), grab(ge, names), grab(ge, names))
    le = m.get_current_losses()
    m.optimize_parameters(grab(gm, names), grab(gm, names), grab(gm, names))
    lm = m.get_current_losses()
    out = flatten(le, ge, {}, "e_")
    out.update(flatten({k: lm[k] for k in ("AM_A", "AM_B")}, gm, {}, "m_"))
    return out


# ------------------------------------------------------------------------------------ C3 step
C3_HW, C3_LAMBDA = (436, 1024), (100.0, 500.0)
C3_SEEDS = {"G_A": 1600, "G_B": 1601, "D_A": 1602, "D_B": 1603}
C3_VGG = 1610


def c3_inputs():
    from oracle import cpu_ref, prng
    H, W = C3_HW
    a, a2, b, mask, flow = cpu_ref.synthetic_batch(1, H, W, gen=torch.Generator().manual_seed(4360))
    probe = torch.from_numpy(prng.uniform_f32(4361, (1, 3, H, W), -1.0, 1.0))
    return (a, a2, b, mask, flow * 4.0), probe   # the flow generator scaled x4


def c3_oracle(dtype):
    from oracle import c3_ref, cpu_ref, prng, style_ref
    m = c3_ref.RefCycleGANConVGG(ngf=64, ndf=64, lambda_c=C3_LAMBDA[0], lambda_s=C3_LAMBDA[1])
    style_ref.load_np(m.vgg, style_ref.vgg_weights(m.vgg, C3_VGG, init="fan_out"))
    m.vgg.to(dtype)
    for name, net in m.nets().items():
        cpu_ref.load_np_state(net, prng.init_state_dict(cpu_ref.state_shapes(net), base_seed=C3_SEEDS[name]))
        net.to(dtype)
    m.opt_G = torch.optim.Adam(list(m.G_A.parameters()) + list(m.G_B.parameters()), lr=2e-4, betas=(0.5, 0.999))
    m.opt_D = torch.optim.Adam(list(m.D_A.parameters()) + list(m.D_B.parameters()), lr=2e-4, betas=(0.5, 0.999))
    data, probe = c3_inputs()
    m.set_input_fc2(*(t.to(dtype) for t in data))
    names = {id(n): k for k, n in m.nets().items()}
    grads = {}
    m.optimize_parameters(grab(grads, names), grab(grads, names))
    losses = m.get_current_losses()
    with torch.no_grad():
        out = m.G_A(probe.to(dtype)).double()
    return flatten(losses, grads, {"probe_after_adam": out})


ORACLES = {"sg": lambda dt, dev: sg_oracle(dt), "mg256": lambda dt, dev: mg_oracle(MG_CFG["256"], dt, dev),
           "mgc5": lambda dt, dev: mg_oracle(MG_CFG["c5"], dt, dev), "c3": lambda dt, dev: c3_oracle(dt)}
# where each case's fp64 run was made (the fp32 run, the reference's own arithmetic, is always the CPU's)
R64_DEVICE = {"sg": "cpu", "mg256": "cpu", "mgc5": "cuda", "c3": "cpu"}


# ------------------------------------------------------------------------------ fixture summary
def summarize(r32, r64):
    """The committed form of one case: per loss (v64, v32); per gradient / tensor its exact ||ref64||,
    the reference's own fp32 deviation ||ref32 - ref64|| / ||ref64||, and ref64 itself (whole when
    small, else its CountSketch)."""
    out = {}
    for key, r in r64.items():
        if kind(key) == "loss":
            out["L:" + key] = np.array([r, r32[key]], np.float64)
            continue
        r, g = torch.as_tensor(r).double(), torch.as_tensor(r32[key]).double()
        n64 = float(r.norm())
        out["N:" + key] = np.array([n64, float((g - r).norm()) / (n64 + 1e-300), r.numel()], np.float64)
        out[("V:" if r.numel() <= RAW_MAX else "S:") + key] = (
            r.reshape(-1).numpy() if r.numel() <= RAW_MAX else sketch.count_sketch(r).numpy())
    return out


def deviations(got, fixture):
    """{key: (dev HIP vs ref64, dev ref32 vs ref64)} for every quantity of a fixture; losses relative,
    gradients / tensors norm-wise (exact for whole-stored ones, from the sketch for the rest)."""
    rows = {}
    for name in fixture.files:
        tag, key = name.split(":", 1)
        if tag == "L":
            v64, v32 = fixture[name]
            rows[key] = (abs(float(got[key]) - v64) / (abs(v64) + 1e-30), abs(v32 - v64) / (abs(v64) + 1e-30))
        elif tag in ("V", "S"):
            n64, d32, numel = fixture["N:" + key]
            g = torch.as_tensor(got[key]).double().cpu().reshape(-1)
            assert g.numel() == int(numel), (key, g.numel(), numel)
            ref = torch.from_numpy(fixture[name])
            dev = (float((g - ref).norm()) / (n64 + 1e-300) if tag == "V"
                   else sketch.sketch_dev(sketch.count_sketch(g), ref, n64))
            rows[key] = (dev, float(d32))
    return rows
