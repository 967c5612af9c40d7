"""CPU oracle — stock-PyTorch (NCHW, fp32) restatement of the reference hot path.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  This module restates, with stock torch
operators on the CPU, exactly the arithmetic the reference runs, so the HIP path can be checked
against it on identical seeded inputs, and so it can be timed as the host-CPU baseline.

Reference files restated (paths relative to the reference root):
  methods/GAN-based/CycleGAN/models/networks.py           ResnetGenerator 315-373, ResnetBlock 376-433,
                                                          NLayerDiscriminator 538-583, GANLoss 209-275
  methods/GAN-based/CycleGANCon/models/cycle_gan_model.py forward 133-139, backward_D_basic 141-161,
                                                          backward_G 173-216, optimize_parameters 218-232
  methods/GAN-based/CycleGAN/models/cycle_gan_model.py    forward_eval 164-171
  utils/flowtools.py                                      gradient 12-16, warp 18-32, fbcCheckTorch 34-58
  methods/GAN-based/CycleGANCon/util/image_pool.py        ImagePool.query 23-54 (pool_size 0 here)
The modules keep the reference's nn.Sequential indices so state_dict keys are identical
(e.g. model.10.conv_block.1.weight) and fixtures/weights load by name.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F


# ----------------------------------------------------------------------------- networks
class RefResnetBlock(nn.Module):
    """networks.py:376-433 with padding_type='reflect', norm=instance, no dropout."""

    def __init__(self, dim):
        super().__init__()
        self.conv_block = nn.Sequential(
            nn.ReflectionPad2d(1), nn.Conv2d(dim, dim, 3, padding=0, bias=True),
            nn.InstanceNorm2d(dim), nn.ReLU(True),
            nn.ReflectionPad2d(1), nn.Conv2d(dim, dim, 3, padding=0, bias=True),
            nn.InstanceNorm2d(dim))

    def forward(self, x):
        return x + self.conv_block(x)          # networks.py:432


class RefResnetGenerator(nn.Module):
    """networks.py:315-373 (resnet_{n}blocks, ngf, instance norm ⇒ conv bias on, 335-338)."""

    def __init__(self, input_nc=3, output_nc=3, ngf=64, n_blocks=9):
        super().__init__()
        L = [nn.ReflectionPad2d(3), nn.Conv2d(input_nc, ngf, 7, padding=0, bias=True),
             nn.InstanceNorm2d(ngf), nn.ReLU(True)]
        for i in range(2):
            m = 2 ** i
            L += [nn.Conv2d(ngf * m, ngf * m * 2, 3, stride=2, padding=1, bias=True),
                  nn.InstanceNorm2d(ngf * m * 2), nn.ReLU(True)]
        for _ in range(n_blocks):
            L += [RefResnetBlock(ngf * 4)]
        for i in range(2):
            m = 2 ** (2 - i)
            L += [nn.ConvTranspose2d(ngf * m, ngf * m // 2, 3, stride=2, padding=1,
                                     output_padding=1, bias=True),
                  nn.InstanceNorm2d(ngf * m // 2), nn.ReLU(True)]
        L += [nn.ReflectionPad2d(3), nn.Conv2d(ngf, output_nc, 7, padding=0), nn.Tanh()]
        self.model = nn.Sequential(*L)

    def forward(self, x):
        return self.model(x)


class RefNLayerDiscriminator(nn.Module):
    """networks.py:538-583 (netD='basic' ⇒ n_layers=3, instance norm ⇒ bias on, LeakyReLU 0.2)."""

    def __init__(self, input_nc=3, ndf=64, n_layers=3):
        super().__init__()
        L = [nn.Conv2d(input_nc, ndf, 4, stride=2, padding=1), nn.LeakyReLU(0.2, True)]
        mult = 1
        for n in range(1, n_layers):
            prev, mult = mult, min(2 ** n, 8)
            L += [nn.Conv2d(ndf * prev, ndf * mult, 4, stride=2, padding=1, bias=True),
                  nn.InstanceNorm2d(ndf * mult), nn.LeakyReLU(0.2, True)]
        prev, mult = mult, min(2 ** n_layers, 8)
        L += [nn.Conv2d(ndf * prev, ndf * mult, 4, stride=1, padding=1, bias=True),
              nn.InstanceNorm2d(ndf * mult), nn.LeakyReLU(0.2, True)]
        L += [nn.Conv2d(ndf * mult, 1, 4, stride=1, padding=1)]
        self.model = nn.Sequential(*L)

    def forward(self, x):
        return self.model(x)


def state_shapes(net):
    return {k: tuple(v.shape) for k, v in net.state_dict().items()}


def load_np_state(net, sd):
    net.load_state_dict({k: torch.from_numpy(v).clone() for k, v in sd.items()})
    return net


# ----------------------------------------------------------------------------- flow ops
def warp(x, flow, align_corners=False):
    """utils/flowtools.py:18-32 — backward bilinear warp, zeros padding.  Normalises the pixel
    grid with max(W-1,1)/max(H-1,1) but samples with align_corners=False (quirk);
    CycleGANCon's inline copy (cycle_gan_model.py:191-203) uses the torch default (False) too."""
    B, C, H, W = x.shape
    xx = torch.arange(W, dtype=torch.float32, device=x.device).view(1, 1, 1, W).expand(B, 1, H, W)
    yy = torch.arange(H, dtype=torch.float32, device=x.device).view(1, 1, H, 1).expand(B, 1, H, W)
    g = torch.cat([xx, yy], 1) + flow
    gx = 2.0 * g[:, 0] / max(W - 1, 1) - 1.0
    gy = 2.0 * g[:, 1] / max(H - 1, 1) - 1.0
    grid = torch.stack([gx, gy], -1)
    return F.grid_sample(x, grid, mode="bilinear", padding_mode="zeros",
                         align_corners=align_corners)


def gradient(x):
    """utils/flowtools.py:12-16 — zero-padded central differences / 2 on a [B,H,W] field."""
    dx = (F.pad(x, (0, 1, 0, 0))[:, :, 1:] - F.pad(x, (1, 0, 0, 0))[:, :, :-1]) / 2
    dy = (F.pad(x, (0, 0, 0, 1))[:, 1:, :] - F.pad(x, (0, 0, 1, 0))[:, :-1, :]) / 2
    return torch.stack([dx, dy])


def fbc_check(ff, bf):
    """utils/flowtools.py:34-58 — forward/backward consistency mask [B,1,H,W] in {0,1}."""
    wf = warp(ff, bf)
    nwb = torch.norm(wf + bf, dim=1) ** 2
    nw = torch.norm(wf, dim=1) ** 2
    nb = torch.norm(bf, dim=1) ** 2
    occ = nwb > 0.01 * (nw + nb) + 0.5
    nu = torch.norm(gradient(bf[:, 0]), dim=0) ** 2.0
    nv = torch.norm(gradient(bf[:, 1]), dim=0) ** 2.0
    mob = nu + nv > 0.01 * nb + 0.002
    mask = torch.ones_like(nb)
    mask = torch.where(occ | mob, torch.zeros_like(mask), mask)
    return mask.unsqueeze(1)


def temporal_loss(fake_b, fake_b2, flow, mask, lambda_t=10.0):
    """CycleGANCon/models/cycle_gan_model.py:191-204."""
    w = warp(fake_b, flow)
    return ((mask * (fake_b2 - w)) ** 2).mean() * lambda_t


def tcl(x_fake, x_prev_fake, bf, mask):
    """utils/sintel_eval.py:104-110 — sqrt(mean((mask*(x - warp(prev, bf)))^2))."""
    return torch.sqrt(((mask * (x_fake - warp(x_prev_fake, bf))) ** 2).mean())


def gan_loss(pred, real):
    """networks.py:257-275 with gan_mode='lsgan' ⇒ MSE against a constant 1/0 target."""
    return ((pred - (1.0 if real else 0.0)) ** 2).mean()


# ----------------------------------------------------------------------------- train step
class RefCycleGANCon:
    """CycleGANCon/models/cycle_gan_model.py:10-232 restated (pool_size=0 ⇒ ImagePool is identity,
    image_pool.py:35-36).  Adam(lr, betas=(beta1, 0.999)) over G_A∪G_B and D_A∪D_B (:97-98)."""

    loss_names = ['D_A', 'G_A', 'cycle_A', 'idt_A', 'D_B', 'G_B', 'cycle_B', 'idt_B', 'G_T']

    def __init__(self, ngf=64, ndf=64, n_blocks=9, lr=2e-4, beta1=0.5, lambda_A=10.0,
                 lambda_B=10.0, lambda_T=10.0, lambda_idt=0.5, device="cpu"):
        self.G_A = RefResnetGenerator(3, 3, ngf, n_blocks).to(device)
        self.G_B = RefResnetGenerator(3, 3, ngf, n_blocks).to(device)
        self.D_A = RefNLayerDiscriminator(3, ndf).to(device)
        self.D_B = RefNLayerDiscriminator(3, ndf).to(device)
        self.lA, self.lB, self.lT, self.lI = lambda_A, lambda_B, lambda_T, lambda_idt
        self.opt_G = torch.optim.Adam(list(self.G_A.parameters()) + list(self.G_B.parameters()),
                                      lr=lr, betas=(beta1, 0.999))
        self.opt_D = torch.optim.Adam(list(self.D_A.parameters()) + list(self.D_B.parameters()),
                                      lr=lr, betas=(beta1, 0.999))

    def nets(self):
        return {"G_A": self.G_A, "G_B": self.G_B, "D_A": self.D_A, "D_B": self.D_B}

    def set_input_fc2(self, real_A, real_A2, real_B, mask, flow):
        self.real_A, self.real_A2, self.real_B, self.mask, self.flow = (
            real_A, real_A2, real_B, mask, flow)

    def optimize_parameters(self, grad_hook_G=None, grad_hook_D=None):
        """grad_hook_*(nets): called between backward and the optimizer step (parity tests read the
        accumulated gradients there, like CycleGANModel.optimize_parameters' hooks)."""
        # forward (:133-139)
        self.fake_B = self.G_A(self.real_A)
        self.fake_B2 = self.G_A(self.real_A2)
        self.rec_A = self.G_B(self.fake_B)
        self.fake_A = self.G_B(self.real_B)
        self.rec_B = self.G_A(self.fake_A)
        for p in list(self.D_A.parameters()) + list(self.D_B.parameters()):
            p.requires_grad_(False)
        self.opt_G.zero_grad()
        # backward_G (:173-216)
        self.idt_A = self.G_A(self.real_B)
        self.loss_idt_A = (self.idt_A - self.real_B).abs().mean() * self.lB * self.lI
        self.idt_B = self.G_B(self.real_A)
        self.loss_idt_B = (self.idt_B - self.real_A).abs().mean() * self.lA * self.lI
        self.loss_G_T = temporal_loss(self.fake_B, self.fake_B2, self.flow, self.mask, self.lT)
        self.loss_G_A = gan_loss(self.D_A(self.fake_B), True)
        self.loss_G_B = gan_loss(self.D_B(self.fake_A), True)
        self.loss_cycle_A = (self.rec_A - self.real_A).abs().mean() * self.lA
        self.loss_cycle_B = (self.rec_B - self.real_B).abs().mean() * self.lB
        self.loss_G = (self.loss_G_A + self.loss_G_B + self.loss_cycle_A + self.loss_cycle_B
                       + self.loss_idt_A + self.loss_idt_B + self.loss_G_T)
        extra = self.extra_G_loss()
        if extra is not None:
            self.loss_G = self.loss_G + extra
        self.loss_G.backward()
        if grad_hook_G is not None:
            grad_hook_G([self.G_A, self.G_B])
        self.opt_G.step()
        # D step (:141-166, 226-232)
        for p in list(self.D_A.parameters()) + list(self.D_B.parameters()):
            p.requires_grad_(True)
        self.opt_D.zero_grad()
        self.loss_D_A = self._backward_D(self.D_A, self.real_B, self.fake_B)
        self.loss_D_B = self._backward_D(self.D_B, self.real_A, self.fake_A)
        if grad_hook_D is not None:
            grad_hook_D([self.D_A, self.D_B])
        self.opt_D.step()

    def extra_G_loss(self):
        """Hook for composed steps (oracle/c3_ref.py): a term added to loss_G before backward."""
        return None

    @staticmethod
    def _backward_D(D, real, fake):
        loss = (gan_loss(D(real), True) + gan_loss(D(fake.detach()), False)) * 0.5
        loss.backward()
        return loss

    def get_current_losses(self):
        return {n: float(getattr(self, "loss_" + n)) for n in self.loss_names}


def forward_eval(G, img):
    """CycleGAN/models/cycle_gan_model.py:164-171 — no-grad generator inference."""
    with torch.no_grad():
        return G(img)


# ----------------------------------------------------------------------------- synthetic data
def synthetic_batch(B, H, W, seed=1234, gen=None):
    """SURVEY §8d synthetic C2 inputs: images (u8/255-0.5)/0.5 (truncating u8 as fc2_dataset.py:38),
    smooth flow (bicubic upsample of an N(0,4^2) 9x9 grid), Bernoulli(0.8) mask on a 32x32 grid."""
    g = gen or torch.Generator().manual_seed(seed)
    imgs = [((torch.randint(0, 256, (B, 3, H, W), generator=g).float() / 255.0) - 0.5) / 0.5
            for _ in range(3)]
    coarse = torch.randn(B, 2, 9, 9, generator=g) * 4.0
    flow = F.interpolate(coarse, size=(H, W), mode="bicubic", align_corners=True)
    mcoarse = (torch.rand(B, 1, 32, 32, generator=g) < 0.8).float()
    mask = F.interpolate(mcoarse, size=(H, W), mode="nearest")
    return imgs[0], imgs[1], imgs[2], mask.contiguous(), flow.contiguous()
