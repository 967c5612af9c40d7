"""Fused Adam over the flat parameter buffers of HIP networks.

Drop-in for the ``torch.optim.Adam(itertools.chain(netG_A.parameters(), netG_B.parameters()),
lr=opt.lr, betas=(opt.beta1, 0.999))`` built at methods/GAN-based/CycleGANCon/models/
cycle_gan_model.py:97-98: same update rule (bias-corrected, eps outside the sqrt, no weight decay),
one vst_adam_step launch per network instead of one kernel per parameter tensor.  It is a
torch.optim.Optimizer, so lr schedulers (networks.get_scheduler) drive ``param_groups[0]['lr']``.
"""
import torch

from . import ops


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, nets, lr=2e-4, betas=(0.9, 0.999), eps=1e-8):
        self.nets = list(nets)
        flats = [n.flat_param for n in self.nets]
        super().__init__(flats, dict(lr=lr, betas=betas, eps=eps))
        self.moments = [(torch.zeros_like(f), torch.zeros_like(f)) for f in flats]
        self.step_count = 0

    def zero_grad(self, set_to_none=False):
        for n in self.nets:
            n.flat_grad.zero_()

    @torch.no_grad()
    def step(self, closure=None):
        self.step_count += 1
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        for n, (m, v) in zip(self.nets, self.moments):
            ops.adam_step(n.flat_param, n.flat_grad, m, v, g["lr"], b1, b2, g["eps"], self.step_count)
            n.bump_version()
        return None
