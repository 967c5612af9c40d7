"""gan-based-video-style-transfer_amd — MI355X-native (gfx950) CycleGAN video train step and
generator inference, drop-in for tomstrident/GAN-based-Video-Style-Transfer's hot path.

Import as ``import gbvst`` (root alias module) or via importlib with the directory name.
Submodules: networks (define_G/define_D/GANLoss), cycle_gan_model (CycleGANModel),
models (create_model), base_model, image_pool, flowtools (warp/fbcCheckTorch), options,
optim (FusedAdam), dp (data-parallel gradient exchange), ops (C-ABI wrappers), library (the
C-ABI entries as torch.library ``vst::*`` operators), _lib (loader/build).
"""
from . import _lib  # noqa: F401

__version__ = "0.1.0"


def build(force=False):
    return _lib.build(force=force)
