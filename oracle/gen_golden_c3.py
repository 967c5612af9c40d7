"""Generate tests/golden/c3_small.npz by importing the READ-ONLY reference (config C3 composition).

TEST INFRASTRUCTURE ONLY — build container only; the output is data.

    cd /tmp && PYTHONDONTWRITEBYTECODE=1 python /root/repo/oracle/gen_golden_c3.py

Runs the reference's own CycleGANCon CycleGANModel (methods/GAN-based/CycleGANCon/models/
cycle_gan_model.py, with its networks / image_pool / base_model) and adds the C3 VGG term
(oracle/c3_ref.py docstring) computed with the reference's methods/learning-based/network.Vgg19:
the composed term is attached where the reference forms its total G loss — a ``loss_G`` property
on a subclass adds it when backward_G assigns the total (cycle_gan_model.py:204-215), so the
reference's forward / backward_G / optimize_parameters code runs unmodified.  gram_matrix /
normalize come from the oracle restatement (fast_style_transfer.py needs cv2 / imageio / skimage).
Shims (oracle side only): torch.Tensor.cuda = identity; a torchvision stub returning seeded VGG-19
features (no pretrained weights offline).  Weights: counter PRNG by name (never stored).
ngf = ndf = 8, 64x64, B = 2, pool_size 0, 2 steps: per-step losses + G_A(probe) after the steps.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
from oracle import c3_ref, gen_golden, gen_golden_style, prng, style_ref  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden", "c3_small.npz")
VGG_SEED = 530


def main():
    gen_golden_style._stub_torchvision()
    sys.path.insert(0, os.path.join(gen_golden.REF, "methods", "learning-based"))
    import network  # noqa: reference Vgg19
    CycleGANModel, _ = gen_golden._import_cyclegancon()

    class C3Model(CycleGANModel):
        """Reference CycleGANCon step with the C3 VGG term composed into its total G loss."""

        @property
        def loss_G(self):
            return self._loss_G

        @loss_G.setter
        def loss_G(self, v):
            if torch.is_tensor(v) and v.requires_grad:
                self.loss_G_C, self.loss_G_S = c3_ref.c3_terms(self.vgg19, self.fake_B2, self.real_A2, self.real_B)
                v = v + self.loss_G_C + self.loss_G_S
            self._loss_G = v

    m = C3Model(gen_golden._opt(8, 8, 0))
    m.loss_names = list(m.loss_names) + ["G_C", "G_S"]
    m.vgg19 = network.Vgg19()
    style_ref.load_np(m.vgg19, style_ref.vgg_weights(m.vgg19, VGG_SEED))
    out = {}
    for name, seed in (("G_A", 1300), ("G_B", 1400), ("D_A", 1500), ("D_B", 1600)):
        net = getattr(m, "net" + name)
        net.load_state_dict({k: torch.from_numpy(v) for k, v in
                             prng.init_state_dict(gen_golden._shapes(net), base_seed=seed).items()})
    B, H, W = 2, 64, 64
    a = prng.uniform_f32(1701, (B, 3, H, W), -1, 1)
    a2 = np.clip(a + 0.05 * prng.normal(1702, (B, 3, H, W)), -1, 1).astype(np.float32)
    b = prng.uniform_f32(1703, (B, 3, H, W), -1, 1)
    mask = (prng.uniform_f32(1704, (B, 1, H, W)) < 0.8).astype(np.float32)
    flow = prng.normal(1705, (B, 2, H, W), std=2.0)
    probe = prng.uniform_f32(1706, (1, 3, H, W), -1, 1)
    for k, v in (("real_A", a), ("real_A2", a2), ("real_B", b), ("mask", mask), ("flow", flow), ("probe", probe)):
        out[k] = v
    data = (torch.from_numpy(a), torch.from_numpy(a2), torch.from_numpy(b), None, torch.from_numpy(mask),
            torch.from_numpy(flow))
    names = m.loss_names
    steps = 2
    losses = np.zeros((steps, len(names)))
    for s in range(steps):
        m.set_input_fc2(data)
        m.optimize_parameters()
        cur = m.get_current_losses()
        losses[s] = [cur[n] for n in names]
    out["loss_names"] = np.array(names)
    out["losses"] = losses
    with torch.no_grad():
        out["probe_out"] = m.netG_A(torch.from_numpy(probe)).numpy().astype(np.float32)
    np.savez_compressed(OUT, **out)
    print(dict(zip(names, losses[0])), os.path.getsize(OUT))


if __name__ == "__main__":
    main()
