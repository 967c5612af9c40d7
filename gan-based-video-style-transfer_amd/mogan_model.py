"""MoGAN (motion-consistent CycleGAN) train step, HIP-backed ("the RAFT
encoders/GRU via the conv kernels; MoGAN step").

Mirror of methods/GAN-based/MoGAN/models/cycle_gan_model.py:13-331 (class ``CycleGANModel`` in the
reference's MoGAN tree; exported here as ``MoGANModel`` and registered as model 'mogan'):
  * forward_train (:160-196): 8 generator passes over two frames of both domains, 8 RAFT calls
    (20 iterations, no_grad, InputPadder), motion nets M_A / M_B (ResNet generators on 2-channel
    flows), warp of the fakes by the predicted motion, fbcCheckTorch masks;
  * alternating steps (:313-331): E-step = G update (GAN + cycle + identity + motion-cycle MC +
    motion-translation MT losses) then D update; M-step = M update (auxiliary motion AM loss);
  * same loss / option names and defaults (lambda_MC 10, lambda_AM 1, lambda_MT 10).
Internally images and motion fields are NHWC4 on the device; G/D/M are the HIP ResNet/PatchGAN
networks (networks.py), RAFT is raft.py (inference only, as the reference's torch.no_grad), the
masked L1 motion losses are HIP reductions, warp / fb-check are the flow kernels.  Note the
reference quirks kept: RAFT sees [-1, 1] images although it rescales as if [0, 255]
(SURVEY App. A.5), and the MC loss has no gradient (both flows come from no_grad RAFT).
"""
import argparse

import torch

from . import networks, ops
from .base_model import BaseModel
from .cycle_gan_model import BATCH_PASSES
from .flowtools import warp_nhwc
from .image_pool import ImagePool
from .optim import FusedAdam
from .raft import RAFT, InputPadder


class _MaskedL1Fn(torch.autograd.Function):
    """scale * mean(mask * |a - b|) over NHWC a, b (cl logical channels), mask [B,1,H,W] or None."""

    @staticmethod
    def forward(ctx, a, b, mask, scale, cl):
        ctx.save_for_backward(a, b, mask)
        ctx.scale, ctx.cl = scale, cl
        return ops.loss_masked_l1(a, b, mask, scale, cl)

    @staticmethod
    def backward(ctx, g):
        a, b, mask = ctx.saved_tensors
        g = g.contiguous()
        ga = ops.loss_masked_l1_bwd(a, b, mask, g, ctx.scale, ctx.cl) if ctx.needs_input_grad[0] else None
        gb = ops.loss_masked_l1_bwd(b, a, mask, g, ctx.scale, ctx.cl) if ctx.needs_input_grad[1] else None
        return ga, gb, None, None, None


def masked_l1(a, b, mask, scale, cl):
    return _MaskedL1Fn.apply(a, b, mask, float(scale), int(cl))


class CycleGANModel(BaseModel):
    @staticmethod
    def modify_commandline_options(parser, is_train=True):
        """MoGAN cycle_gan_model.py:29-54 + the RAFT flags of MoGAN/options/base_options.py:30-32."""
        parser.set_defaults(no_dropout=True)
        if is_train:
            parser.add_argument('--lambda_A', type=float, default=10.0, help='weight for cycle loss (A -> B -> A)')
            parser.add_argument('--lambda_B', type=float, default=10.0, help='weight for cycle loss (B -> A -> B)')
            parser.add_argument('--lambda_MC', type=float, default=10.0, help='weight for motion cycle loss')
            parser.add_argument('--lambda_AM', type=float, default=1.0, help='weight for auxiliary motion loss')
            parser.add_argument('--lambda_MT', type=float, default=10.0, help='weight for motion translation loss')
            parser.add_argument('--lambda_identity', type=float, default=0.5, help='use identity mapping.')
        for flag in ('--small', '--mixed_precision', '--alternate_corr'):
            try:
                parser.add_argument(flag, action='store_true')
            except argparse.ArgumentError:
                pass
        return parser

    def __init__(self, opt, raft_model=None, raft_iters=20):
        BaseModel.__init__(self, opt)
        self.e_step = True
        self.raft_iters = raft_iters
        self.loss_names = ['D_A', 'G_A', 'cycle_A', 'idt_A', 'D_B', 'G_B', 'cycle_B', 'idt_B', 'MC_A', 'AM_A',
                           'MT_A', 'MC_B', 'AM_B', 'MT_B']
        visual_names_A = ['real_A', 'fake_B', 'rec_A', 'real_A2', 'fake_B2', 'rec_A2', 'warp_B', 'mask_A']
        visual_names_B = ['real_B', 'fake_A', 'rec_B', 'real_B2', 'fake_A2', 'rec_B2', 'warp_A', 'mask_B']
        if self.isTrain and self.opt.lambda_identity > 0.0:
            visual_names_A.append('idt_B')
            visual_names_B.append('idt_A')
        self.visual_names = visual_names_A + visual_names_B
        self.model_names = ['G_A', 'G_B', 'D_A', 'D_B', 'M_A', 'M_B'] if self.isTrain else ['G_A', 'G_B']
        mk_g = lambda i, o: networks.define_G(i, o, opt.ngf, opt.netG, opt.norm, not opt.no_dropout,  # noqa: E731
                                              opt.init_type, opt.init_gain, self.gpu_ids)
        self.netG_A = mk_g(opt.input_nc, opt.output_nc)
        self.netG_B = mk_g(opt.output_nc, opt.input_nc)
        if self.isTrain:
            self.netD_A = networks.define_D(opt.output_nc, opt.ndf, opt.netD, opt.n_layers_D, opt.norm,
                                            opt.init_type, opt.init_gain, self.gpu_ids)
            self.netD_B = networks.define_D(opt.input_nc, opt.ndf, opt.netD, opt.n_layers_D, opt.norm,
                                            opt.init_type, opt.init_gain, self.gpu_ids)
            self.netM_A = mk_g(2, 2)
            self.netM_B = mk_g(2, 2)
            self.raftModel = raft_model if raft_model is not None else self.initRaftModel(opt)
            if opt.lambda_identity > 0.0:
                assert opt.input_nc == opt.output_nc
            self.fake_A_pool = ImagePool(opt.pool_size)
            self.fake_B_pool = ImagePool(opt.pool_size)
            self.criterionGAN = networks.GANLoss(opt.gan_mode).to(self.device)
            self.optimizer_G = FusedAdam([self.netG_A, self.netG_B], lr=opt.lr, betas=(opt.beta1, 0.999))
            self.optimizer_D = FusedAdam([self.netD_A, self.netD_B], lr=opt.lr, betas=(opt.beta1, 0.999))
            self.optimizer_M = FusedAdam([self.netM_A, self.netM_B], lr=opt.lr, betas=(opt.beta1, 0.999))
            self.optimizers = [self.optimizer_G, self.optimizer_D, self.optimizer_M]
            self.set_requires_grad([self.netM_A, self.netM_B], False)
        # test conditioning hook (parity tests only): a list of dicts of NCHW flows / masks, one per
        # forward_train, used instead of the RAFT calls and fb-check masks (FLOW_KEYS + mask_A / mask_B)
        self.flow_inject = None

    FLOW_KEYS = ("ff_real_A", "bf_real_A", "bf_fake_B", "bf_rec_A", "ff_real_B", "bf_real_B", "bf_fake_A", "bf_rec_B")

    def _injected(self):
        if not self.flow_inject:
            return None
        src = self.flow_inject.pop(0)
        return {k: (ops.nchw_to_nhwc(v.to(self.device).float().contiguous()) if k in self.FLOW_KEYS
                    else v.to(self.device).float().contiguous()) for k, v in src.items()}

    def initRaftModel(self, opt):
        """:119-126 — the reference loads raft/models/raft-chairs.pth, which is not shipped; the
        caller passes a loaded RAFT (``raft_model=``) or gets random-init weights here."""
        m = RAFT(argparse.Namespace(small=getattr(opt, 'small', False), mixed_precision=False,
                                    alternate_corr=getattr(opt, 'alternate_corr', False), dropout=0))
        return m.to(self.device).eval()

    def computeRAFT(self, img1, img2, it=None):
        """:128-134: no_grad RAFT on NHWC4 images -> flow_up as NHWC4 [B,H,W,4] (2 logical)."""
        it = self.raft_iters if it is None else it
        with torch.no_grad():
            B, H, W, _ = img1.shape
            padder = InputPadder((B, 3, H, W))
            if getattr(self.raftModel, "use_graphs", False):
                flow_up = self.raftModel.graphed(img1.detach(), img2.detach(), it, padder.pads, nhwc=True)[1]
            else:
                _, flow_up = self.raftModel(img1.detach(), img2.detach(), iters=it, test_mode=True, pads=padder.pads,
                                            nhwc=True)
            l, r, t, b = padder.pads
            if l or r or t or b:
                # the reference returns the padded flow_up (:128-134) and then warps / compares it with the
                # unpadded frames, which fails for frames that are not multiples of 8 (1024x436: 440 rows);
                # the flow is cut back to the frame here (InputPadder.unpad), as the oracle does
                flow_up = flow_up[:, t:flow_up.shape[1] - b, l:flow_up.shape[2] - r].contiguous()
        return flow_up

    # ------------------------------------------------------------------------------- inputs
    def _img(self, x):
        x = x.to(self.device, non_blocking=True).float().contiguous()
        return ops.nchw_to_nhwc(x) if x.dim() == 4 and x.shape[1] == self.opt.input_nc else x

    def set_input_fc2(self, data):
        """:136-142: (img1, img2, simg1, simg2) NCHW."""
        img1, img2, simg1, simg2 = data
        self.real_A, self.real_A2 = self._img(img1), self._img(img2)
        self.real_B, self.real_B2 = self._img(simg1), self._img(simg2)

    def set_input_nhwc(self, real_A, real_A2, real_B, real_B2):
        self.real_A, self.real_A2, self.real_B, self.real_B2 = real_A, real_A2, real_B, real_B2

    # ------------------------------------------------------------------------------ forward
    def forward_train(self):
        """:160-196."""
        if BATCH_PASSES:
            return self._forward_train_batched()
        G_A, G_B = self.netG_A.forward_nhwc, self.netG_B.forward_nhwc
        self.fake_B = G_A(self.real_A)
        self.rec_A = G_B(self.fake_B)
        self.fake_A = G_B(self.real_B)
        self.rec_B = G_A(self.fake_A)
        self.fake_B2 = G_A(self.real_A2)
        self.rec_A2 = G_B(self.fake_B2)
        self.fake_A2 = G_B(self.real_B2)
        self.rec_B2 = G_A(self.fake_A2)

        self.ff_real_A = self.computeRAFT(self.real_A, self.real_A2)
        self.bf_real_A = self.computeRAFT(self.real_A2, self.real_A)
        self.bf_fake_B = self.computeRAFT(self.fake_B2, self.fake_B)
        self.bf_rec_A = self.computeRAFT(self.rec_A2, self.rec_A)
        self.bf_M_A = self.netM_A.forward_nhwc(self.bf_real_A)
        self.warp_B = warp_nhwc(self.fake_B, ops.nhwc_to_nchw(self.bf_M_A.detach(), 2))
        self.mask_A = ops.fbcheck(ops.nhwc_to_nchw(self.ff_real_A, 2), ops.nhwc_to_nchw(self.bf_real_A, 2))

        self.ff_real_B = self.computeRAFT(self.real_B, self.real_B2)
        self.bf_real_B = self.computeRAFT(self.real_B2, self.real_B)
        self.bf_fake_A = self.computeRAFT(self.fake_A2, self.fake_A)
        self.bf_rec_B = self.computeRAFT(self.rec_B2, self.rec_B)
        self.bf_M_B = self.netM_B.forward_nhwc(self.bf_real_B)
        self.warp_A = warp_nhwc(self.fake_A, ops.nhwc_to_nchw(self.bf_M_B.detach(), 2))
        self.mask_B = ops.fbcheck(ops.nhwc_to_nchw(self.ff_real_B, 2), ops.nhwc_to_nchw(self.bf_real_B, 2))

    def _forward_train_batched(self):
        """forward_train with its passes grouped (per-sample layers, so every sample's result is the
        unbatched one): G_A[real_A, real_A2], G_B[fake_B, fake_B2, real_B, real_B2, (real_A)],
        G_A[fake_A, fake_A2, (real_B)] (the E-step's identity passes ride along), then ONE RAFT call
        over all eight frame pairs and one call per motion net."""
        B = self.real_A.shape[0]
        idt = self.e_step and self.opt.lambda_identity > 0
        ya = self.netG_A.forward_nhwc(torch.cat([self.real_A, self.real_A2]))
        self.fake_B, self.fake_B2 = ya[:B], ya[B:]
        yb = self.netG_B.forward_nhwc(torch.cat([self.fake_B, self.fake_B2, self.real_B, self.real_B2]
                                                + ([self.real_A] if idt else [])))
        self.rec_A, self.rec_A2, self.fake_A, self.fake_A2 = (yb[k * B:(k + 1) * B] for k in range(4))
        yc = self.netG_A.forward_nhwc(torch.cat([self.fake_A, self.fake_A2] + ([self.real_B] if idt else [])))
        self.rec_B, self.rec_B2 = yc[:B], yc[B:2 * B]
        self._idt_pre = (yc[2 * B:], yb[4 * B:]) if idt else None
        firsts = [self.real_A, self.real_A2, self.fake_B2, self.rec_A2, self.real_B, self.real_B2, self.fake_A2,
                  self.rec_B2]
        seconds = [self.real_A2, self.real_A, self.fake_B, self.rec_A, self.real_B2, self.real_B, self.fake_A,
                   self.rec_B]
        inj = self._injected()
        if inj is None:
            fl = self.computeRAFT(torch.cat([t.detach() for t in firsts]), torch.cat([t.detach() for t in seconds]))
            (self.ff_real_A, self.bf_real_A, self.bf_fake_B, self.bf_rec_A,
             self.ff_real_B, self.bf_real_B, self.bf_fake_A, self.bf_rec_B) = (fl[k * B:(k + 1) * B] for k in range(8))
        else:
            for k in self.FLOW_KEYS:
                setattr(self, k, inj[k])
        self.bf_M_A = self.netM_A.forward_nhwc(self.bf_real_A)
        self.warp_B = warp_nhwc(self.fake_B, ops.nhwc_to_nchw(self.bf_M_A.detach(), 2))
        self.mask_A = inj["mask_A"] if inj is not None else ops.fbcheck(ops.nhwc_to_nchw(self.ff_real_A, 2),
                                                                       ops.nhwc_to_nchw(self.bf_real_A, 2))
        self.bf_M_B = self.netM_B.forward_nhwc(self.bf_real_B)
        self.warp_A = warp_nhwc(self.fake_A, ops.nhwc_to_nchw(self.bf_M_B.detach(), 2))
        self.mask_B = inj["mask_B"] if inj is not None else ops.fbcheck(ops.nhwc_to_nchw(self.ff_real_B, 2),
                                                                       ops.nhwc_to_nchw(self.bf_real_B, 2))

    def forward(self):
        """:198-203 (used by test)."""
        self.fake_B = self.netG_A.forward_nhwc(self.real_A)
        self.rec_A = self.netG_B.forward_nhwc(self.fake_B)
        self.fake_A = self.netG_B.forward_nhwc(self.real_B)
        self.rec_B = self.netG_A.forward_nhwc(self.fake_A)

    def forward_eval(self, inp, AtoB=True):
        """:205-212."""
        img = inp.to(self.device).float().contiguous()
        net = self.netG_A if AtoB else self.netG_B
        with torch.no_grad():
            return net(img)

    # ---------------------------------------------------------------------------- backward
    def backward_D_basic(self, netD, real, fake):
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
        self.loss_D_A = self.backward_D_basic(self.netD_A, self.real_B, self.fake_B_pool.query(self.fake_B))

    def backward_D_B(self):
        self.loss_D_B = self.backward_D_basic(self.netD_B, self.real_A, self.fake_A_pool.query(self.fake_A))

    def backward_G(self):
        """:256-303."""
        lambda_idt, lambda_A, lambda_B = self.opt.lambda_identity, self.opt.lambda_A, self.opt.lambda_B
        lambda_MC, lambda_MT = self.opt.lambda_MC, self.opt.lambda_MT
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
        self.loss_G_A = self.criterionGAN(self.netD_A.forward_nhwc(self.fake_B), True, nhwc=True)
        self.loss_G_B = self.criterionGAN(self.netD_B.forward_nhwc(self.fake_A), True, nhwc=True)
        self.loss_cycle_A = networks.l1_loss(self.rec_A, self.real_A, lambda_A)
        self.loss_cycle_B = networks.l1_loss(self.rec_B, self.real_B, lambda_B)
        # MC: both flows are no_grad RAFT outputs -> a constant term (kept for the loss report)
        self.loss_MC_A = masked_l1(self.bf_rec_A, self.bf_real_A, self.mask_A, lambda_MC, 2)
        self.loss_MC_B = masked_l1(self.bf_rec_B, self.bf_real_B, self.mask_B, lambda_MC, 2)
        self.loss_MT_A = masked_l1(self.warp_B, self.fake_B2, self.mask_A, lambda_MT, 3)
        self.loss_MT_B = masked_l1(self.warp_A, self.fake_A2, self.mask_B, lambda_MT, 3)
        self.loss_G = (self.loss_G_A + self.loss_G_B + self.loss_cycle_A + self.loss_cycle_B + self.loss_idt_A
                       + self.loss_idt_B + self.loss_MC_A + self.loss_MC_B + self.loss_MT_A + self.loss_MT_B)
        self.loss_G.backward()

    def backward_M(self):
        """:305-313."""
        lambda_AM = self.opt.lambda_AM
        self.loss_AM_A = masked_l1(self.bf_M_A, self.bf_fake_B, None, lambda_AM, 2)
        self.loss_AM_B = masked_l1(self.bf_M_B, self.bf_fake_A, None, lambda_AM, 2)
        self.loss_M = self.loss_AM_A + self.loss_AM_B
        self.loss_M.backward()

    def optimize_parameters(self, grad_hook_G=None, grad_hook_D=None, grad_hook_M=None):
        """:315-352 (E-step / M-step alternation).  grad_hook_*: the DP gradient exchange."""
        self.forward_train()
        if self.e_step:
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
            self.set_requires_grad([self.netM_A, self.netM_B], True)
            self.set_requires_grad([self.netG_A, self.netG_B], False)
            self.set_requires_grad([self.netD_A, self.netD_B], False)
            self.e_step = False
        else:
            self.optimizer_M.zero_grad()
            self.backward_M()
            if grad_hook_M is not None:
                grad_hook_M([self.netM_A, self.netM_B])
            self.optimizer_M.step()
            self.set_requires_grad([self.netM_A, self.netM_B], False)
            self.set_requires_grad([self.netG_A, self.netG_B], True)
            self.e_step = True

    def _visual(self, t):
        if torch.is_tensor(t) and t.dim() == 4 and t.shape[-1] == 4:
            return ops.nhwc_to_nchw(t.detach().contiguous(), 3)
        return t


MoGANModel = CycleGANModel
