"""Generate tests/golden/mogan_small.npz by running the READ-ONLY reference MoGAN model.

TEST INFRASTRUCTURE ONLY — build container only (the GPU box never runs this); outputs are data.

    cd /tmp && PYTHONDONTWRITEBYTECODE=1 python /root/repo/oracle/gen_golden_mogan.py

Imported from /root/reference: methods/GAN-based/MoGAN/models/cycle_gan_model.py
(+ its networks.py, base_model.py, flowtools.py, raft/ package).  Oracle-side shims: torch.Tensor.cuda
= identity (flowtools.warp calls .cuda()), fbcCheckTorch(..., device='cpu'); ``initRaftModel`` is replaced by a RAFT with counter-PRNG
weights (oracle/raft_ref.raft_weights base 1300, flow head scaled by 1e-3) in eval mode, because raft/models/raft-chairs.pth is
not shipped.  G/D/M weights: prng.init_state_dict by name (bases 1500-1505, std 0.02).  Config:
ngf = ndf = 8, resnet_9blocks, basic D, 1x3x128x128 frames in [-1, 1], pool_size 0, two
optimize_parameters calls (E-step then M-step); the per-step loss dicts plus the step-1 RAFT flow /
fb-check mask / motion-net output are stored.
"""
import argparse
import os
import sys

import numpy as np
import torch

REF = "/root/reference/methods/GAN-based/MoGAN"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REPO)
from oracle import prng, raft_ref  # noqa: E402

torch.set_num_threads(8)
LOSS_NAMES = ['D_A', 'G_A', 'cycle_A', 'idt_A', 'D_B', 'G_B', 'cycle_B', 'idt_B', 'MC_A', 'AM_A', 'MT_A', 'MC_B',
              'AM_B', 'MT_B']
RAFT_FLOW_SCALE = 1e-3  # flows of ~1e-2 px: fbcCheck keeps most pixels, so MC / MT are exercised
SEEDS = {"G_A": 1500, "G_B": 1501, "D_A": 1502, "D_B": 1503, "M_A": 1504, "M_B": 1505}


def _np(t):
    return t.detach().cpu().numpy().astype(np.float32)


def main():
    cwd = os.getcwd()
    os.chdir(REF)
    sys.path.insert(0, REF)
    torch.Tensor.cuda = lambda self, *a, **k: self
    from models import cycle_gan_model as cgm  # noqa
    from raft.raft import RAFT  # noqa

    def init_raft(self, opt):
        m = RAFT(argparse.Namespace(small=False, mixed_precision=False, alternate_corr=False, dropout=0))
        shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
        m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in raft_ref.raft_weights(shapes, 1300, RAFT_FLOW_SCALE).items()})
        return m.eval()

    cgm.CycleGANModel.initRaftModel = init_raft
    fbc = cgm.fbcCheckTorch
    cgm.fbcCheckTorch = lambda ff, bf, device="cpu": fbc(ff, bf, device="cpu")
    opt = argparse.Namespace(isTrain=True, gpu_ids=[], checkpoints_dir="/tmp/mogan_ckpt", name="golden",
                             preprocess="none", input_nc=3, output_nc=3, ngf=8, ndf=8, netG="resnet_9blocks",
                             netD="basic", n_layers_D=3, norm="instance", no_dropout=True, init_type="normal",
                             init_gain=0.02, pool_size=0, gan_mode="lsgan", lr=2e-4, beta1=0.5, lambda_A=10.0,
                             lambda_B=10.0, lambda_MC=10.0, lambda_AM=1.0, lambda_MT=10.0, lambda_identity=0.5,
                             direction="AtoB", small=False, mixed_precision=False, alternate_corr=False)
    model = cgm.CycleGANModel(opt)
    for name, seed in SEEDS.items():
        net = getattr(model, "net" + name)
        shapes = {k: tuple(v.shape) for k, v in net.state_dict().items()}
        net.load_state_dict({k: torch.from_numpy(v) for k, v in prng.init_state_dict(shapes, base_seed=seed).items()})
    imgs = [prng.uniform_f32(1510 + i, (1, 3, 128, 128), -1.0, 1.0) for i in range(4)]
    imgs[1] = np.clip(np.roll(imgs[0], (2, 3), axis=(2, 3)) + prng.normal(1520, imgs[0].shape, std=0.05), -1, 1)
    imgs[3] = np.clip(np.roll(imgs[2], (-1, 2), axis=(2, 3)) + prng.normal(1521, imgs[0].shape, std=0.05), -1, 1)
    imgs = [i.astype(np.float32) for i in imgs]
    out = {"img%d" % i: im for i, im in enumerate(imgs)}
    losses = []
    for step in range(2):
        model.set_input_fc2([torch.from_numpy(i) for i in imgs])
        model.optimize_parameters()
        # (get_current_losses raises before the first M-step defines loss_AM_*: read what exists)
        losses.append([float(getattr(model, "loss_" + n)) if hasattr(model, "loss_" + n) else np.nan
                       for n in LOSS_NAMES])
        if step == 0:
            out.update(bf_real_A=_np(model.bf_real_A), mask_A=_np(model.mask_A), bf_M_A=_np(model.bf_M_A),
                       fake_B=_np(model.fake_B), bf_fake_B=_np(model.bf_fake_B))
    out["losses"] = np.array(losses, np.float64)
    out["loss_names"] = np.array(LOSS_NAMES)
    os.chdir(cwd)
    np.savez_compressed(os.path.join(OUT, "mogan_small.npz"), **out)


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    main()
    print("mogan_small.npz", os.path.getsize(os.path.join(OUT, "mogan_small.npz")))
