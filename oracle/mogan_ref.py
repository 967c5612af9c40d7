"""CPU oracle for the MoGAN train step.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): restatement of
methods/GAN-based/MoGAN/models/cycle_gan_model.py:160-352 (forward_train, backward_G, backward_D_*,
backward_M, the E-step / M-step alternation) over the restated CycleGAN networks (oracle/cpu_ref.py),
RAFT (oracle/raft_ref.py), warp and fbcCheckTorch (oracle/cpu_ref.py); pool_size 0 (ImagePool is
the identity).  Pinned by tests/golden/mogan_small.npz, which oracle/gen_golden_mogan.py wrote by
running the reference MoGAN model itself.
"""
import torch

from oracle import cpu_ref, raft_ref


class RefMoGAN:
    loss_names = ['D_A', 'G_A', 'cycle_A', 'idt_A', 'D_B', 'G_B', 'cycle_B', 'idt_B', 'MC_A', 'AM_A', 'MT_A',
                  'MC_B', 'AM_B', 'MT_B']

    def __init__(self, raft_sd, ngf=8, ndf=8, n_blocks=9, lr=2e-4, beta1=0.5, lambda_A=10.0, lambda_B=10.0,
                 lambda_MC=10.0, lambda_AM=1.0, lambda_MT=10.0, lambda_idt=0.5, raft_iters=20):
        self.G_A = cpu_ref.RefResnetGenerator(3, 3, ngf, n_blocks)
        self.G_B = cpu_ref.RefResnetGenerator(3, 3, ngf, n_blocks)
        self.D_A = cpu_ref.RefNLayerDiscriminator(3, ndf)
        self.D_B = cpu_ref.RefNLayerDiscriminator(3, ndf)
        self.M_A = cpu_ref.RefResnetGenerator(2, 2, ngf, n_blocks)
        self.M_B = cpu_ref.RefResnetGenerator(2, 2, ngf, n_blocks)
        self.raft_sd, self.raft_iters = raft_sd, raft_iters
        self.lA, self.lB, self.lMC, self.lAM, self.lMT, self.lI = lambda_A, lambda_B, lambda_MC, lambda_AM, lambda_MT, \
            lambda_idt
        adam = lambda nets: torch.optim.Adam([p for n in nets for p in n.parameters()], lr=lr,  # noqa: E731
                                             betas=(beta1, 0.999))
        self.opt_G, self.opt_D, self.opt_M = adam([self.G_A, self.G_B]), adam([self.D_A, self.D_B]), \
            adam([self.M_A, self.M_B])
        self._req([self.M_A, self.M_B], False)
        self.e_step = True
        # conditioning hooks of the parity tests: every forward_train's 8 RAFT flows + 2 fb-check masks
        # are appended to `record`; with `inject` (a list of such dicts, consumed in order) they are
        # taken from there instead of computed (the discrete / RAFT-amplified parts held equal)
        self.record, self.inject = [], None

    def nets(self):
        return {"G_A": self.G_A, "G_B": self.G_B, "D_A": self.D_A, "D_B": self.D_B, "M_A": self.M_A, "M_B": self.M_B}

    @staticmethod
    def _req(nets, flag):
        for n in nets:
            for p in n.parameters():
                p.requires_grad_(flag)

    def raft(self, a, b):
        """computeRAFT (:128-134).  The reference returns flow_up at the padded size, which its warp /
        motion losses cannot take for frames that are not multiples of 8 (1024x436 pads to 440 rows);
        the flow is cut back to the frame (InputPadder.unpad), the build's defined behaviour there."""
        with torch.no_grad():
            pads = raft_ref.input_pads(a.shape)
            _, up = raft_ref.raft_forward(self.raft_sd, raft_ref.pad_replicate(a, pads),
                                          raft_ref.pad_replicate(b, pads), iters=self.raft_iters, test_mode=True)
        l, r, t, bt = pads
        return up[..., t:up.shape[-2] - bt, l:up.shape[-1] - r]

    def set_input_fc2(self, img1, img2, simg1, simg2):
        self.real_A, self.real_A2, self.real_B, self.real_B2 = img1, img2, simg1, simg2

    def forward_train(self):
        self.fake_B = self.G_A(self.real_A)
        self.rec_A = self.G_B(self.fake_B)
        self.fake_A = self.G_B(self.real_B)
        self.rec_B = self.G_A(self.fake_A)
        self.fake_B2 = self.G_A(self.real_A2)
        self.rec_A2 = self.G_B(self.fake_B2)
        self.fake_A2 = self.G_B(self.real_B2)
        self.rec_B2 = self.G_A(self.fake_A2)
        rec = {}
        src = self.inject.pop(0) if self.inject else None
        for d, (r, r2, f, f2, rc, rc2, M) in (("A", (self.real_A, self.real_A2, self.fake_B, self.fake_B2, self.rec_A,
                                                     self.rec_A2, self.M_A)),
                                              ("B", (self.real_B, self.real_B2, self.fake_A, self.fake_A2, self.rec_B,
                                                     self.rec_B2, self.M_B))):
            other = "B" if d == "A" else "A"
            names = ("ff_real_" + d, "bf_real_" + d, "bf_fake_" + other, "bf_rec_" + d)
            if src is not None:
                ff_real, bf_real, bf_fake, bf_rec = (src[k].clone() for k in names)
            else:
                ff_real = self.raft(r, r2)
                bf_real = self.raft(r2, r)
                bf_fake = self.raft(f2, f)
                bf_rec = self.raft(rc2, rc)
            bf_M = M(bf_real)
            warp = cpu_ref.warp(f, bf_M)
            mask = src["mask_" + d].clone() if src is not None else cpu_ref.fbc_check(ff_real, bf_real)
            rec.update(zip(names, (ff_real, bf_real, bf_fake, bf_rec)))
            rec["mask_" + d] = mask
            setattr(self, "bf_real_" + d, bf_real)
            setattr(self, "bf_fake_" + other, bf_fake)
            setattr(self, "bf_rec_" + d, bf_rec)
            setattr(self, "bf_M_" + d, bf_M)
            setattr(self, "warp_" + other, warp)
            setattr(self, "mask_" + d, mask)
        self.record.append({k: v.detach().clone() for k, v in rec.items()})

    def optimize_parameters(self, grad_hook_G=None, grad_hook_D=None, grad_hook_M=None):
        """grad_hook_*(nets): called between each phase's backward and its Adam step (the tests read
        the gradients there, as the HIP model's DP hooks do)."""
        self.forward_train()
        if self.e_step:
            self._req([self.D_A, self.D_B], False)
            self.opt_G.zero_grad()
            self.loss_idt_A = (self.G_A(self.real_B) - self.real_B).abs().mean() * self.lB * self.lI
            self.loss_idt_B = (self.G_B(self.real_A) - self.real_A).abs().mean() * self.lA * self.lI
            self.loss_G_A = cpu_ref.gan_loss(self.D_A(self.fake_B), True)
            self.loss_G_B = cpu_ref.gan_loss(self.D_B(self.fake_A), True)
            self.loss_cycle_A = (self.rec_A - self.real_A).abs().mean() * self.lA
            self.loss_cycle_B = (self.rec_B - self.real_B).abs().mean() * self.lB
            self.loss_MC_A = (self.mask_A * torch.abs(self.bf_rec_A - self.bf_real_A)).mean() * self.lMC
            self.loss_MC_B = (self.mask_B * torch.abs(self.bf_rec_B - self.bf_real_B)).mean() * self.lMC
            self.loss_MT_A = (self.mask_A * torch.abs(self.warp_B - self.fake_B2)).mean() * self.lMT
            self.loss_MT_B = (self.mask_B * torch.abs(self.warp_A - self.fake_A2)).mean() * self.lMT
            loss = (self.loss_G_A + self.loss_G_B + self.loss_cycle_A + self.loss_cycle_B + self.loss_idt_A
                    + self.loss_idt_B + self.loss_MC_A + self.loss_MC_B + self.loss_MT_A + self.loss_MT_B)
            loss.backward()
            if grad_hook_G is not None:
                grad_hook_G([self.G_A, self.G_B])
            self.opt_G.step()
            self._req([self.D_A, self.D_B], True)
            self.opt_D.zero_grad()
            self.loss_D_A = cpu_ref.RefCycleGANCon._backward_D(self.D_A, self.real_B, self.fake_B)
            self.loss_D_B = cpu_ref.RefCycleGANCon._backward_D(self.D_B, self.real_A, self.fake_A)
            if grad_hook_D is not None:
                grad_hook_D([self.D_A, self.D_B])
            self.opt_D.step()
            self._req([self.M_A, self.M_B], True)
            self._req([self.G_A, self.G_B], False)
            self._req([self.D_A, self.D_B], False)
            self.e_step = False
        else:
            self.opt_M.zero_grad()
            self.loss_AM_A = torch.abs(self.bf_M_A - self.bf_fake_B).mean() * self.lAM
            self.loss_AM_B = torch.abs(self.bf_M_B - self.bf_fake_A).mean() * self.lAM
            (self.loss_AM_A + self.loss_AM_B).backward()
            if grad_hook_M is not None:
                grad_hook_M([self.M_A, self.M_B])
            self.opt_M.step()
            self._req([self.M_A, self.M_B], False)
            self._req([self.G_A, self.G_B], True)
            self.e_step = True

    def get_current_losses(self):
        return {n: float(getattr(self, "loss_" + n)) for n in self.loss_names if hasattr(self, "loss_" + n)}
