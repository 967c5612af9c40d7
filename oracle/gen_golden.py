"""Generate the golden fixtures under tests/golden/ by importing the READ-ONLY reference.

TEST INFRASTRUCTURE ONLY.  Runs in the build container (where /root/reference exists); the GPU box
never runs this.  The outputs are data (inputs + the reference's own outputs), committed as small
.npz files; no reference source travels.

    cd /tmp && PYTHONDONTWRITEBYTECODE=1 python /root/repo/oracle/gen_golden.py

What is imported:
  methods/GAN-based/CycleGANCon/models/cycle_gan_model.py  CycleGANModel (networks, base_model, image_pool)
  methods/GAN-based/CycleGAN/models/networks.py            define_G / define_D
  utils/flowtools.py                                       warp, fbcCheckTorch
Shim (oracle side only): torch.Tensor.cuda is made the identity because flowtools.warp and
CycleGANCon.backward_G hard-code .cuda() (utils/flowtools.py:25, cycle_gan_model.py:197).
Weights come from oracle/prng.py (counter-based), loaded into the reference modules by name.
"""
import argparse
import os
import sys

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REPO)
from oracle import prng  # noqa: E402

torch.Tensor.cuda = lambda self, *a, **k: self          # oracle-side shim (see docstring)
torch.set_num_threads(8)


def _import_flowtools():
    sys.path.insert(0, os.path.join(REF, "utils"))
    import flowtools  # noqa
    sys.path.pop(0)
    return flowtools


def _import_cyclegancon():
    d = os.path.join(REF, "methods", "GAN-based", "CycleGANCon")
    sys.path.insert(0, d)
    cwd = os.getcwd()
    os.chdir(d)
    from models.cycle_gan_model import CycleGANModel  # noqa
    from models import networks  # noqa
    os.chdir(cwd)
    return CycleGANModel, networks


def _np(t):
    return t.detach().cpu().numpy().astype(np.float32)


def gen_warp(ft):
    """Fixture 1: warp fwd + d/dx for several flow kinds, non-square, plus W=1/H=1 cases."""
    out = {}
    cases = []
    B, C, H, W = 2, 3, 20, 24
    x = prng.normal(11, (B, C, H, W))
    g = prng.normal(12, (B, C, H, W))
    cases.append(("zero", x, np.zeros((B, 2, H, W), np.float32), g))
    cases.append(("int", x, np.round(prng.normal(13, (B, 2, H, W), std=3.0)), g))
    cases.append(("frac", x, prng.normal(14, (B, 2, H, W), std=2.5), g))
    cases.append(("oob", x, prng.normal(15, (B, 2, H, W), std=40.0), g))
    x1 = prng.normal(16, (1, 2, 1, 7))
    cases.append(("h1", x1, prng.normal(17, (1, 2, 1, 7), std=1.5), prng.normal(18, (1, 2, 1, 7))))
    x2 = prng.normal(19, (1, 2, 6, 1))
    cases.append(("w1", x2, prng.normal(20, (1, 2, 6, 1), std=1.5), prng.normal(21, (1, 2, 6, 1))))
    for name, xv, fv, gv in cases:
        xt = torch.from_numpy(xv).requires_grad_(True)
        ftt = torch.from_numpy(fv.astype(np.float32))
        y = ft.warp(xt, ftt)
        y.backward(torch.from_numpy(gv))
        out[f"{name}_x"], out[f"{name}_flow"], out[f"{name}_gout"] = xv, fv.astype(np.float32), gv
        out[f"{name}_y"], out[f"{name}_dx"] = _np(y), _np(xt.grad)
    np.savez_compressed(os.path.join(OUT, "warp.npz"), **out)


def gen_fbc(ft):
    """Fixture 2: fbcCheckTorch on consistent and inconsistent flow pairs (2x2x40x48)."""
    B, H, W = 2, 40, 48
    base = prng.normal(30, (B, 2, H, W), std=2.0)
    out = {}
    # consistent-ish: bf ≈ -ff (smooth), inconsistent: independent noise with a jump
    yy, xx = np.meshgrid(np.linspace(-1, 1, H), np.linspace(-1, 1, W), indexing="ij")
    smooth = np.stack([3 * np.sin(2 * xx) + yy, 2 * np.cos(3 * yy) - xx]).astype(np.float32)
    ff1 = np.broadcast_to(smooth, (B, 2, H, W)).copy()
    bf1 = -ff1 + 0.05 * base
    ff2 = 0.5 * ff1
    bf2 = -ff2 + 0.02 * prng.normal(31, (B, 2, H, W))
    bf2[:, :, 10:25, 20:40] += 3.0          # an occluded block: occ and motion-boundary both fire
    for name, ff, bf in (("cons", ff1, bf1), ("incons", ff2, bf2)):
        m = ft.fbcCheckTorch(torch.from_numpy(ff), torch.from_numpy(bf.astype(np.float32)), device="cpu")
        out[f"{name}_ff"], out[f"{name}_bf"], out[f"{name}_mask"] = ff, bf.astype(np.float32), _np(m)
    np.savez_compressed(os.path.join(OUT, "fbc.npz"), **out)


def _opt(ngf, ndf, pool):
    return argparse.Namespace(
        gpu_ids=[], isTrain=True, checkpoints_dir="/tmp/ck", name="golden", preprocess="none",
        input_nc=3, output_nc=3, ngf=ngf, ndf=ndf, netG="resnet_9blocks", netD="basic",
        n_layers_D=3, norm="instance", no_dropout=True, init_type="normal", init_gain=0.02,
        lambda_identity=0.5, lambda_A=10.0, lambda_B=10.0, lambda_T=10.0, pool_size=pool,
        gan_mode="lsgan", lr=2e-4, beta1=0.5, direction="AtoB")


def _shapes(net):
    return {k: tuple(v.shape) for k, v in net.state_dict().items()}


def gen_nets(networks):
    """Fixture 6: ResnetGenerator(ngf=8, 9 blocks) and NLayerDiscriminator(ndf=8) at 64x64, B=2:
    outputs, input grads and every parameter grad for a fixed upstream gradient."""
    out = {}
    G = networks.define_G(3, 3, 8, "resnet_9blocks", "instance", False, "normal", 0.02, [])
    D = networks.define_D(3, 8, "basic", 3, "instance", "normal", 0.02, [])
    for tag, net, seed in (("G", G, 100), ("D", D, 200)):
        sd = prng.init_state_dict(_shapes(net), base_seed=seed)
        net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
        x = prng.uniform_f32(seed + 1, (2, 3, 64, 64), -1.0, 1.0)
        xt = torch.from_numpy(x).requires_grad_(True)
        y = net(xt)
        gy = prng.normal(seed + 2, tuple(y.shape))
        y.backward(torch.from_numpy(gy))
        out[f"{tag}_x"], out[f"{tag}_y"], out[f"{tag}_gy"], out[f"{tag}_dx"] = x, _np(y), gy, _np(xt.grad)
        for k, p in net.named_parameters():
            out[f"{tag}_w_{k}"] = sd[k]
            out[f"{tag}_g_{k}"] = _np(p.grad)
    np.savez_compressed(os.path.join(OUT, "nets_small.npz"), **out)


def gen_step(CycleGANModel, ngf=8, ndf=8, H=64, W=64, B=2, steps=3):
    """Fixture 7: 3 CycleGANCon optimize_parameters() steps, pool_size=0 (deterministic):
    per-step loss dict, and G_A(probe) after the last step."""
    m = CycleGANModel(_opt(ngf, ndf, 0))
    out = {}
    for name, seed in (("G_A", 300), ("G_B", 400), ("D_A", 500), ("D_B", 600)):
        net = getattr(m, "net" + name)
        sd = prng.init_state_dict(_shapes(net), base_seed=seed)
        net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
        for k, v in sd.items():
            out[f"w_{name}_{k}"] = v
    a = prng.uniform_f32(701, (B, 3, H, W), -1, 1)
    a2 = np.clip(a + 0.05 * prng.normal(702, (B, 3, H, W)), -1, 1).astype(np.float32)
    b = prng.uniform_f32(703, (B, 3, H, W), -1, 1)
    mask = (prng.uniform_f32(704, (B, 1, H, W)) < 0.8).astype(np.float32)
    flow = prng.normal(705, (B, 2, H, W), std=2.0)
    probe = prng.uniform_f32(706, (1, 3, H, W), -1, 1)
    for k, v in (("real_A", a), ("real_A2", a2), ("real_B", b), ("mask", mask), ("flow", flow), ("probe", probe)):
        out[k] = v
    data = (torch.from_numpy(a), torch.from_numpy(a2), torch.from_numpy(b), None,
            torch.from_numpy(mask), torch.from_numpy(flow))
    names = m.loss_names
    losses = np.zeros((steps, len(names)), np.float64)
    for s in range(steps):
        m.set_input_fc2(data)
        m.optimize_parameters()
        cur = m.get_current_losses()
        losses[s] = [cur[n] for n in names]
    out["loss_names"] = np.array(names)
    out["losses"] = losses
    with torch.no_grad():
        out["probe_out"] = _np(m.netG_A(torch.from_numpy(probe)))
    for name in ("G_A", "D_A"):
        for k, v in getattr(m, "net" + name).state_dict().items():
            if k.endswith("weight"):
                out[f"after_{name}_{k}"] = _np(v)
    np.savez_compressed(os.path.join(OUT, "step_small.npz"), **out)


def gen_prng():
    """Fixture 0: PRNG known-answer vector (pins oracle/prng.py and the C++/HIP restatement)."""
    np.savez_compressed(os.path.join(OUT, "prng.npz"), u=prng.uniform(7, 16), n=prng.normal(7, (17,)))


def main():
    os.makedirs(OUT, exist_ok=True)
    only = sys.argv[1:]
    if only:
        ft = _import_flowtools()
        for name in only:
            globals()['gen_' + name](ft)
        return
    gen_prng()
    ft = _import_flowtools()
    gen_warp(ft)
    gen_fbc(ft)
    CycleGANModel, networks = _import_cyclegancon()
    gen_nets(networks)
    gen_step(CycleGANModel)
    for f in sorted(os.listdir(OUT)):
        print(f, os.path.getsize(os.path.join(OUT, f)))


if __name__ == "__main__":
    main()
