"""C3 oracle — the CycleGANCon train step plus a VGG-19 perceptual / Gram style loss on fake_B2.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  SURVEY.md §8d config C3: CycleGAN + flow-warp
temporal loss + VGG loss, 1 GPU, Sintel frame pairs 1024x436.  The reference has no such step (its
only CycleGAN-family VGG term, ConGAN's, is commented out: methods/GAN-based/ConGAN/models/
cycle_gan_model.py:295-296), so the composition is defined by the build, from reference pieces:
  vgg(x)    = Vgg19(normalize((x + 1) / 2))                 methods/learning-based/network.py:45-78
            (images are in [-1, 1]; normalize = ImageNet mean/std, fast_style_transfer.py:819-822)
  loss_G_C  = lambda_C * mean((vgg(fake_B2)[relu4_1] - vgg(real_A2)[relu4_1])^2)        content
  loss_G_S  = lambda_S * sum_{relu1_1..relu5_1} mean((gram(vgg(fake_B2)_i) - gram(vgg(real_B)_i))^2)
            gram = bmm(F, F^T) / (h*w), fast_style_transfer.py:813-817 (style = the B-domain frame)
  loss_G   += loss_G_C + loss_G_S       added to CycleGANCon's backward_G total (:204-216)
The targets (vgg of real_A2 / real_B) carry no gradient; VGG is frozen (network.py:69-70).
Pinned by tests/golden/c3_small.npz, which oracle/gen_golden_c3.py wrote by running the REFERENCE
CycleGANCon CycleGANModel with the reference network.Vgg19 composed in.
"""
import torch

from oracle import cpu_ref, style_ref

LAMBDA_C, LAMBDA_S = 1.0, 0.01  # seeded (not pretrained) VGG weights: Gram MSE is O(100), scaled to O(1)
CONTENT_LEVEL = 3  # relu4_1


def vgg_in(x):
    return style_ref.normalize((x + 1.0) / 2.0)


def c3_terms(vgg, fake_b2, real_a2, real_b, lambda_c=LAMBDA_C, lambda_s=LAMBDA_S):
    f = vgg(vgg_in(fake_b2))
    with torch.no_grad():
        fc = vgg(vgg_in(real_a2))
        fs = vgg(vgg_in(real_b))
        gs = [style_ref.gram_matrix(t) for t in fs]
    content = ((f[CONTENT_LEVEL] - fc[CONTENT_LEVEL]) ** 2).mean() * lambda_c
    style = 0
    for fi, gi in zip(f, gs):
        style = style + ((style_ref.gram_matrix(fi) - gi) ** 2).mean()
    return content, style * lambda_s


class RefCycleGANConVGG(cpu_ref.RefCycleGANCon):
    loss_names = cpu_ref.RefCycleGANCon.loss_names + ['G_C', 'G_S']

    def __init__(self, ngf=64, ndf=64, lambda_c=LAMBDA_C, lambda_s=LAMBDA_S, **kw):
        super().__init__(ngf=ngf, ndf=ndf, **kw)
        self.vgg = style_ref.RefVGG("vgg19")
        self.lambda_c, self.lambda_s = lambda_c, lambda_s

    def extra_G_loss(self):
        self.loss_G_C, self.loss_G_S = c3_terms(self.vgg, self.fake_B2, self.real_A2, self.real_B,
                                                self.lambda_c, self.lambda_s)
        return self.loss_G_C + self.loss_G_S
