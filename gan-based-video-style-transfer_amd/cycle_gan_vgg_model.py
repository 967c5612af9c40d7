"""CycleGANVGGModel — config C3: the CycleGANCon train step plus a VGG-19 perceptual / Gram style
loss on the temporally-warped frame's translation fake_B2 (CycleGAN + flow-warp
temporal loss + VGG loss on Sintel frame pairs 1024x436, 1 GPU).  Model name 'cycle_gan_vgg'.

The reference has no such step (ConGAN's VGG term is commented out:
methods/GAN-based/ConGAN/models/cycle_gan_model.py:295-296), so the composition is the build's,
made of reference pieces (the oracle oracle/c3_ref.py restates it; tests/golden/c3_small.npz pins it
against the reference CycleGANCon model with the reference network.Vgg19 composed in):
  vgg(x)   = Vgg19(normalize((x + 1) / 2))              network.py:45-78, fast_style_transfer.py:819-822
  loss_G_C = lambda_content * mean((vgg(fake_B2)[relu4_1] - vgg(real_A2)[relu4_1])^2)
  loss_G_S = lambda_style * sum_{relu1_1..relu5_1} mean((gram(vgg(fake_B2)_i) - gram(vgg(real_B)_i))^2)
             gram = F F^T / (h*w) (fast_style_transfer.py:813-817); style target = the B-domain frame
  loss_G  += loss_G_C + loss_G_S                        (CycleGANCon backward_G total, :204-216)
VGG is frozen (network.py:69-70): its backward is the data gradient only; the targets run as
inference.  Everything stays NHWC on the HIP kernels (perceptual.py): the (x + 1) / 2 and the
ImageNet normalisation are one channel-normalise pass ((x / 2) - (mean - 1/2)) / std.
Pretrained VGG weights cannot be fetched offline: the net initialises from `vgg_seed` and loads real
weights with ``netVGG.load_state_dict`` (torchvision `features` keys via load_torchvision_features).
"""
import torch

from . import ops, perceptual
from .cycle_gan_model import CycleGANModel

CONTENT_LEVEL = 3  # relu4_1
# the loss's three VGG forwards as one batch (perceptual._VggMultiFn); False: three calls
VGG_BATCHED = True
SEEDED_LAMBDA = (100.0, 500.0)       # (content, style) for the seeded kaiming fan_out VGG-19
PRETRAINED_LAMBDA = (1.0, 0.01)      # for real (or fan_in-scale) VGG-19 weights


def resolve_loss_weights(opt):
    """Fill unset lambda_content / lambda_style from the VGG weight source (seeded or --vgg_weights)."""
    d = PRETRAINED_LAMBDA if getattr(opt, 'vgg_weights', '') else SEEDED_LAMBDA
    if getattr(opt, 'lambda_content', None) is None:
        opt.lambda_content = d[0]
    if getattr(opt, 'lambda_style', None) is None:
        opt.lambda_style = d[1]
    return opt


class CycleGANVGGModel(CycleGANModel):
    @staticmethod
    def modify_commandline_options(parser, is_train=True):
        parser = CycleGANModel.modify_commandline_options(parser, is_train)
        if is_train:
            # defaults calibrated for the torchvision-initialised VGG-19 (kaiming fan_out, the net's own
            # seeded init; pretrained weights are not available offline) on [-1, 1] frames: its Gram
            # MSE sums to ~2e-3 and the relu4_1 content MSE to ~4e-3, so these weights make both terms
            # O(0.1-1) beside the cycle losses (~4) at any frame size (the Grams are 1/(h*w)
            # normalised).  The reduced-size golden (tests/golden/c3_small.npz) was composed with
            # lambda_content 1, lambda_style 0.01 on a fan_in-initialised VGG whose Grams are ~1e4x larger.
            # Real (pretrained) weights have Grams of that larger order too, so --vgg_weights switches
            # the defaults to 1 / 0.01; explicit values always win.
            parser.add_argument('--lambda_content', type=float, default=None,
                                help='VGG-19 relu4_1 content weight (default 100 seeded VGG, 1 with --vgg_weights)')
            parser.add_argument('--lambda_style', type=float, default=None,
                                help='VGG-19 Gram style weight (default 500 seeded VGG, 0.01 with --vgg_weights)')
            parser.add_argument('--vgg_seed', type=int, default=0, help='seed of the (non-pretrained) VGG-19')
            parser.add_argument('--vgg_weights', type=str, default='',
                                help='torchvision vgg19 state_dict (.pth, loaded weights_only) or its features')
        return parser

    def __init__(self, opt):
        super().__init__(opt)
        self.loss_names = self.loss_names + ['G_C', 'G_S']
        self.netVGG = perceptual.Vgg19(seed=getattr(opt, 'vgg_seed', 0)).to(self.device)
        path = getattr(opt, 'vgg_weights', '')
        if path:
            sd = torch.load(path, map_location='cpu', weights_only=True)
            self.netVGG.load_torchvision_features(sd)
        resolve_loss_weights(opt)
        mean, std = perceptual._mean_std(self.device)
        self._vgg_mean, self._vgg_std = (mean - 0.5).contiguous(), std

    def _vgg_in(self, img_nhwc4):
        """normalize((x + 1) / 2) of an NHWC4 image in [-1, 1] (the VGG input)."""
        return perceptual._NormalizeFn.apply(img_nhwc4, self._vgg_mean, self._vgg_std, 2.0, 3)

    def vgg_features(self, img_nhwc4):
        """Vgg19(normalize((x + 1) / 2)) of an NHWC4 image in [-1, 1] -> 5 NHWC slice outputs."""
        return self.netVGG.forward_nhwc(self._vgg_in(img_nhwc4))

    def extra_G_loss(self):
        if not self.temporal:
            raise NotImplementedError('cycle_gan_vgg composes the temporal (CycleGANCon) step: lambda_T > 0')
        if VGG_BATCHED:  # the three forwards as one batch (perceptual._VggMultiFn): fake_B2 (differentiated), real_B
            # (all levels: style Grams), real_A2 (through the content level only)
            nl = len(self.netVGG.slices_idx)
            with torch.no_grad():
                xb, xa = self._vgg_in(self.real_B), self._vgg_in(self.real_A2)
            f, fb, fa = self.netVGG.forward_multi_nhwc([self._vgg_in(self.fake_B2), xb, xa], [nl, nl, CONTENT_LEVEL + 1])
            fc = fa[CONTENT_LEVEL]
            with torch.no_grad():
                gs = [perceptual.gram_nhwc(t) for t in fb]
        else:
            f = self.vgg_features(self.fake_B2)
            with torch.no_grad():
                fc = self.vgg_features(self.real_A2)[CONTENT_LEVEL]
                gs = [perceptual.gram_nhwc(t) for t in self.vgg_features(self.real_B)]
        self.loss_G_C = perceptual.mse_loss(f[CONTENT_LEVEL], fc, self.opt.lambda_content)
        style = None
        for fi, gi in zip(f, gs):
            term = perceptual.mse_loss(perceptual.gram_nhwc(fi), gi, self.opt.lambda_style)
            style = term if style is None else style + term
        self.loss_G_S = style
        return self.loss_G_C + self.loss_G_S


from . import _lib as _lib_routes  # noqa: E402
_lib_routes.apply_route_overrides(__name__, globals())
