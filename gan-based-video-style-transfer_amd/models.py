"""Model plugin discovery — mirror of methods/GAN-based/*/models/__init__.py:25-67.

``create_model(opt)`` instantiates the BaseModel subclass registered for ``opt.model``; like the
reference, '<name>' maps to a class named '<Name>Model' (case-insensitive, underscores removed).
The HIP build registers the hot-path plugin 'cycle_gan' (CycleGANCon semantics; ``--lambda_T 0``
gives the plain CycleGAN step), 'cycle_gan_vgg' (config C3: + VGG-19 content / Gram loss,
cycle_gan_vgg_model.py) and 'mogan' (MoGAN's motion-consistent step, mogan_model.py).
"""
from .base_model import BaseModel
from .cycle_gan_model import CycleGANModel
from .cycle_gan_vgg_model import CycleGANVGGModel
from .mogan_model import MoGANModel

_REGISTRY = {"cycle_gan": CycleGANModel, "cycle_gan_vgg": CycleGANVGGModel, "mogan": MoGANModel}


def find_model_using_name(model_name):
    model = _REGISTRY.get(model_name)
    if model is None:
        target = model_name.replace('_', '') + 'model'
        for cls in _REGISTRY.values():
            if cls.__name__.lower() == target.lower() and issubclass(cls, BaseModel):
                model = cls
    if model is None:
        raise NotImplementedError(
            "model [%s] is not on the HIP hot path; available: %s" % (model_name, sorted(_REGISTRY)))
    return model


def get_option_setter(model_name):
    return find_model_using_name(model_name).modify_commandline_options


def create_model(opt):
    model = find_model_using_name(opt.model)
    instance = model(opt)
    print("model [%s] was created" % type(instance).__name__)
    return instance
