"""CycleGANModel — the metric's train step, HIP-backed.

Mirror of methods/GAN-based/CycleGANCon/models/cycle_gan_model.py:10-232 (CycleGAN + optical-flow
warped temporal loss, 'G_T') with the generator-only inference entry ``forward_eval`` of
methods/GAN-based/CycleGAN/models/cycle_gan_model.py:164-171.  With ``lambda_T == 0`` the step is
the plain CycleGAN step of methods/GAN-based/CycleGAN/models/cycle_gan_model.py:150-252
(4 + 2 generator passes, no temporal term).

Same method names, loss names, option names/defaults and update order:
  forward (5 G passes) -> G step [D frozen: dgrad only] (2 identity passes, temporal warp loss,
  LSGAN + cycle + identity losses, one backward, Adam) -> D step (pool query, 4 D passes, Adam).
Internally every image is NHWC4 on the GPU; networks run as single autograd nodes over
libvst_hip kernels (see networks.py); the losses are HIP reduction kernels.
"""
import os

import torch

from . import networks, ops
from .base_model import BaseModel
from .image_pool import ImagePool
from .optim import FusedAdam


# Group the step's generator passes per network into batched calls (and real+fake per D);
# False runs them one by one as the reference does.
BATCH_PASSES = True


class _TemporalFn(torch.autograd.Function):
    """loss_G_T = mean((mask * (fake_B2 - warp(fake_B, flow)))^2) * lambda_T  (:191-204)."""

    @staticmethod
    def forward(ctx, fake_b, fake_b2, flow, mask, lam):
        ctx.save_for_backward(fake_b, fake_b2, flow, mask)
        ctx.lam = lam
        return ops.loss_temporal(fake_b, fake_b2, flow, mask, lam)

    @staticmethod
    def backward(ctx, g):
        fake_b, fake_b2, flow, mask = ctx.saved_tensors
        ga = torch.zeros_like(fake_b) if ctx.needs_input_grad[0] else None
        gb = torch.empty_like(fake_b2) if ctx.needs_input_grad[1] else None
        ops.loss_temporal_bwd(fake_b, fake_b2, flow, mask, g.contiguous(), ga, gb, ctx.lam)
        return ga, gb, None, None, None


def temporal_loss(fake_b, fake_b2, flow, mask, lambda_T):
    return _TemporalFn.apply(fake_b, fake_b2, flow.contiguous(), mask.contiguous(), float(lambda_T))


class CycleGANModel(BaseModel):
    @staticmethod
    def modify_commandline_options(parser, is_train=True):
        """cycle_gan_model.py:21-48 (same flags and defaults)."""
        parser.set_defaults(no_dropout=True)
        if is_train:
            parser.add_argument('--lambda_A', type=float, default=10.0, help='weight for cycle loss (A -> B -> A)')
            parser.add_argument('--lambda_B', type=float, default=10.0, help='weight for cycle loss (B -> A -> B)')
            parser.add_argument('--lambda_T', type=float, default=10.0, help='weight for temporal loss')
            parser.add_argument('--lambda_identity', type=float, default=0.5, help='use identity mapping.')
        return parser

    def __init__(self, opt):
        BaseModel.__init__(self, opt)
        self.temporal = self.isTrain and getattr(opt, 'lambda_T', 0.0) > 0.0
        self.loss_names = ['D_A', 'G_A', 'cycle_A', 'idt_A', 'D_B', 'G_B', 'cycle_B', 'idt_B']
        if self.temporal:
            self.loss_names.append('G_T')
        visual_names_A = ['real_A', 'fake_B', 'rec_A']
        visual_names_B = ['real_B', 'fake_A', 'rec_B']
        if self.isTrain and self.opt.lambda_identity > 0.0:
            visual_names_A.append('idt_B')
            visual_names_B.append('idt_A')
        self.visual_names = visual_names_A + visual_names_B
        self.model_names = ['G_A', 'G_B', 'D_A', 'D_B'] if self.isTrain else ['G_A', 'G_B']

        self.netG_A = networks.define_G(opt.input_nc, opt.output_nc, opt.ngf, opt.netG, opt.norm,
                                        not opt.no_dropout, opt.init_type, opt.init_gain, self.gpu_ids)
        self.netG_B = networks.define_G(opt.output_nc, opt.input_nc, opt.ngf, opt.netG, opt.norm,
                                        not opt.no_dropout, opt.init_type, opt.init_gain, self.gpu_ids)
        if self.isTrain:
            self.netD_A = networks.define_D(opt.output_nc, opt.ndf, opt.netD, opt.n_layers_D, opt.norm,
                                            opt.init_type, opt.init_gain, self.gpu_ids)
            self.netD_B = networks.define_D(opt.input_nc, opt.ndf, opt.netD, opt.n_layers_D, opt.norm,
                                            opt.init_type, opt.init_gain, self.gpu_ids)
            if opt.lambda_identity > 0.0:
                assert opt.input_nc == opt.output_nc
            self.fake_A_pool = ImagePool(opt.pool_size)
            self.fake_B_pool = ImagePool(opt.pool_size)
            self.criterionGAN = networks.GANLoss(opt.gan_mode).to(self.device)
            self.optimizer_G = FusedAdam([self.netG_A, self.netG_B], lr=opt.lr, betas=(opt.beta1, 0.999))
            self.optimizer_D = FusedAdam([self.netD_A, self.netD_B], lr=opt.lr, betas=(opt.beta1, 0.999))
            self.optimizers = [self.optimizer_G, self.optimizer_D]

    # ------------------------------------------------------------------------------- inputs
    def _img(self, x):
        x = x.to(self.device, non_blocking=True).float().contiguous()
        return ops.nchw_to_nhwc(x) if x.shape[1] == self.opt.input_nc else x

    def set_input(self, inp):
        AtoB = self.opt.direction == 'AtoB'
        self.real_A = self._img(inp['A' if AtoB else 'B'])
        self.real_B = self._img(inp['B' if AtoB else 'A'])
        self.image_paths = inp.get('A_paths' if AtoB else 'B_paths', [])

    def set_input_fc2(self, data):
        """cycle_gan_model.py:124-131: (img1, img2, styled, label, mask, flow), NCHW from the loader."""
        img1, img2, simg, _, mask, flow = data
        self.real_A = self._img(img1)
        self.real_A2 = self._img(img2)
        self.real_B = self._img(simg)
        self.mask = mask.to(self.device).float().contiguous()
        self.flow = flow.to(self.device).float().contiguous()

    def set_input_nhwc(self, real_A, real_A2, real_B, mask, flow):
        """Zero-copy entry for device-resident NHWC4 batches (bench / DP loaders)."""
        self.real_A, self.real_A2, self.real_B, self.mask, self.flow = real_A, real_A2, real_B, mask, flow

    # ------------------------------------------------------------------------------ forward
    def forward(self):
        """CycleGANCon :133-139 (fake_B2 only with the temporal term; CycleGAN :150-155 otherwise)."""
        if BATCH_PASSES and self.isTrain:
            return self._forward_batched()
        self.fake_B = self.netG_A.forward_nhwc(self.real_A)
        if self.temporal:
            self.fake_B2 = self.netG_A.forward_nhwc(self.real_A2)
        self.rec_A = self.netG_B.forward_nhwc(self.fake_B)
        self.fake_A = self.netG_B.forward_nhwc(self.real_B)
        self.rec_B = self.netG_A.forward_nhwc(self.fake_A)

    def _forward_batched(self):
        """The same generator passes, grouped by network into three batched calls (InstanceNorm is
        per sample, so every sample's result is the unbatched one): G_A[real_A, real_A2],
        G_B[fake_B, real_B, (real_A)], G_A[fake_A, (real_B)] — the identity passes of backward_G
        (:180-189) ride along.  Larger GEMMs use the chip better (G fwd+bwd at B=8 measured 9 %
        below two B=4 passes)."""
        B = self.real_A.shape[0]
        idt = self.opt.lambda_identity > 0
        xa = torch.cat([self.real_A, self.real_A2]) if self.temporal else self.real_A
        ya = self.netG_A.forward_nhwc(xa)
        self.fake_B = ya[:B]
        if self.temporal:
            self.fake_B2 = ya[B:]
        yb = self.netG_B.forward_nhwc(torch.cat([self.fake_B, self.real_B] + ([self.real_A] if idt else [])))
        self.rec_A, self.fake_A = yb[:B], yb[B:2 * B]
        yc = self.netG_A.forward_nhwc(torch.cat([self.fake_A, self.real_B]) if idt else self.fake_A)
        self.rec_B = yc[:B]
        self._idt_pre = (yc[B:], yb[2 * B:]) if idt else None

    def forward_eval(self, inp, AtoB=True):
        """CycleGAN/models/cycle_gan_model.py:164-171: no-grad generator inference (NCHW in/out)."""
        img = inp.to(self.device).float().contiguous()
        with torch.no_grad():
            net = self.netG_A if AtoB else self.netG_B
            return net(img)

    # ---------------------------------------------------------------------------- backward
    def backward_D_basic(self, netD, real, fake):
        """:141-161 (real and fake through D as one batch when BATCH_PASSES: per-sample layers)."""
        if BATCH_PASSES and real.shape == fake.shape:
            B = real.shape[0]
            pred = netD.forward_nhwc(torch.cat([real, fake.detach()]))
            pred_real, pred_fake = pred[:B], pred[B:]
        else:
            pred_real = netD.forward_nhwc(real)
            pred_fake = netD.forward_nhwc(fake.detach())
        loss_D_real = self.criterionGAN(pred_real, True, nhwc=True)
        loss_D_fake = self.criterionGAN(pred_fake, False, nhwc=True)
        loss_D = (loss_D_real + loss_D_fake) * 0.5
        loss_D.backward()
        return loss_D

    def backward_D_A(self):
        fake_B = self.fake_B_pool.query(self.fake_B)
        self.loss_D_A = self.backward_D_basic(self.netD_A, self.real_B, fake_B)

    def backward_D_B(self):
        fake_A = self.fake_A_pool.query(self.fake_A)
        self.loss_D_B = self.backward_D_basic(self.netD_B, self.real_A, fake_A)

    def backward_G(self):
        """CycleGANCon :173-216."""
        lambda_idt = self.opt.lambda_identity
        lambda_A, lambda_B = self.opt.lambda_A, self.opt.lambda_B
        if lambda_idt > 0:
            pre = getattr(self, "_idt_pre", None)
            self._idt_pre = None
            self.idt_A = pre[0] if pre is not None else self.netG_A.forward_nhwc(self.real_B)
            self.loss_idt_A = networks.l1_loss(self.idt_A, self.real_B, lambda_B * lambda_idt)
            self.idt_B = pre[1] if pre is not None else self.netG_B.forward_nhwc(self.real_A)
            self.loss_idt_B = networks.l1_loss(self.idt_B, self.real_A, lambda_A * lambda_idt)
        else:
            self.loss_idt_A = 0
            self.loss_idt_B = 0
        if self.temporal:
            self.loss_G_T = temporal_loss(self.fake_B, self.fake_B2, self.flow, self.mask, self.opt.lambda_T)
        else:
            self.loss_G_T = 0
        self.loss_G_A = self.criterionGAN(self.netD_A.forward_nhwc(self.fake_B), True, nhwc=True)
        self.loss_G_B = self.criterionGAN(self.netD_B.forward_nhwc(self.fake_A), True, nhwc=True)
        self.loss_cycle_A = networks.l1_loss(self.rec_A, self.real_A, lambda_A)
        self.loss_cycle_B = networks.l1_loss(self.rec_B, self.real_B, lambda_B)
        self.loss_G = (self.loss_G_A + self.loss_G_B + self.loss_cycle_A + self.loss_cycle_B
                       + self.loss_idt_A + self.loss_idt_B + self.loss_G_T)
        extra = self.extra_G_loss()
        if extra is not None:
            self.loss_G = self.loss_G + extra
        self.loss_G.backward()

    def extra_G_loss(self):
        """Hook for composed steps (cycle_gan_vgg_model.py, config C3): a term added to the total G
        loss before its backward.  None for the CycleGANCon step itself."""
        return None

    def optimize_parameters(self, grad_hook_G=None, grad_hook_D=None):
        """:218-232.  ``grad_hook_*`` (used by dp.py) run between backward and the optimizer step."""
        self.forward()
        self.set_requires_grad([self.netD_A, self.netD_B], False)
        self.optimizer_G.zero_grad()
        self.backward_G()
        if grad_hook_G is not None:
            grad_hook_G([self.netG_A, self.netG_B])
        self.optimizer_G.step()
        self.set_requires_grad([self.netD_A, self.netD_B], True)
        self.optimizer_D.zero_grad()
        self.backward_D_A()
        self.backward_D_B()
        if grad_hook_D is not None:
            grad_hook_D([self.netD_A, self.netD_B])
        self.optimizer_D.step()

    def _visual(self, t):
        if torch.is_tensor(t) and t.dim() == 4 and t.shape[-1] == ops.cpad(self.opt.input_nc):
            return ops.nhwc_to_nchw(t.detach().contiguous(), self.opt.input_nc)
        return t


from . import _lib as _lib_routes  # noqa: E402
_lib_routes.apply_route_overrides(__name__, globals())
