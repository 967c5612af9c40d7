"""BaseModel — mirror of methods/GAN-based/CycleGANCon/models/base_model.py:8-230.

Same public methods and checkpoint format ('%s_net_%s.pth' % (epoch, name), CPU state_dict with the
reference's keys), so reference checkpoints load into the HIP networks and back.  Loading uses
``torch.load(..., weights_only=True)`` (tensors only; nothing from the file is executed).
"""
import os
from collections import OrderedDict

import torch

from . import networks


class BaseModel:
    def __init__(self, opt):
        self.opt = opt
        self.gpu_ids = opt.gpu_ids
        self.isTrain = opt.isTrain
        if self.gpu_ids:
            self.device = torch.device('cuda:{}'.format(self.gpu_ids[0]))
        elif torch.cuda.is_available():
            self.device = torch.device('cuda:%d' % torch.cuda.current_device())
        else:
            self.device = torch.device('cpu')
        self.save_dir = os.path.join(opt.checkpoints_dir, opt.name)
        self.loss_names = []
        self.model_names = []
        self.visual_names = []
        self.optimizers = []
        self.image_paths = []
        self.metric = 0

    @staticmethod
    def modify_commandline_options(parser, is_train):
        return parser

    def setup(self, opt):
        """base_model.py:78-89."""
        if self.isTrain:
            self.schedulers = [networks.get_scheduler(optimizer, opt) for optimizer in self.optimizers]
        if not self.isTrain or getattr(opt, 'continue_train', False):
            load_iter = getattr(opt, 'load_iter', 0)
            load_suffix = 'iter_%d' % load_iter if load_iter > 0 else opt.epoch
            self.load_networks(load_suffix)
        self.print_networks(getattr(opt, 'verbose', False))

    def eval(self):
        for name in self.model_names:
            getattr(self, 'net' + name).eval()

    def test(self):
        with torch.no_grad():
            self.forward()
            self.compute_visuals()

    def compute_visuals(self):
        pass

    def get_image_paths(self):
        return self.image_paths

    def update_learning_rate(self):
        """base_model.py:116-126."""
        old_lr = self.optimizers[0].param_groups[0]['lr']
        for scheduler in self.schedulers:
            if self.opt.lr_policy == 'plateau':
                scheduler.step(self.metric)
            else:
                scheduler.step()
        lr = self.optimizers[0].param_groups[0]['lr']
        print('learning rate %.7f -> %.7f' % (old_lr, lr))

    def get_current_visuals(self):
        visual_ret = OrderedDict()
        for name in self.visual_names:
            visual_ret[name] = self._visual(getattr(self, name))
        return visual_ret

    def _visual(self, t):
        return t

    def get_current_losses(self):
        """base_model.py:136-142 (float() = one device->host sync per loss, as in the reference)."""
        errors_ret = OrderedDict()
        for name in self.loss_names:
            errors_ret[name] = float(getattr(self, 'loss_' + name))
        return errors_ret

    def save_networks(self, epoch):
        """base_model.py:144-160: '%s_net_%s.pth' % (epoch, name), CPU state_dict."""
        os.makedirs(self.save_dir, exist_ok=True)
        for name in self.model_names:
            net = getattr(self, 'net' + name)
            sd = {k: v.detach().cpu().clone() for k, v in net.state_dict().items()}
            torch.save(sd, os.path.join(self.save_dir, '%s_net_%s.pth' % (epoch, name)))

    def load_networks(self, epoch):
        """base_model.py:176-199 (legacy InstanceNorm running-stat keys are dropped)."""
        for name in self.model_names:
            net = getattr(self, 'net' + name)
            path = os.path.join(self.save_dir, '%s_net_%s.pth' % (epoch, name))
            print('loading the model from %s' % path)
            sd = torch.load(path, map_location='cpu', weights_only=True)
            sd = {k: v for k, v in sd.items()
                  if not k.endswith(('running_mean', 'running_var', 'num_batches_tracked'))}
            net.load_state_dict(sd)

    def print_networks(self, verbose):
        print('---------- Networks initialized -------------')
        for name in self.model_names:
            net = getattr(self, 'net' + name)
            num_params = sum(p.numel() for p in net.parameters())
            if verbose:
                print(net)
            print('[Network %s] Total number of parameters : %.3f M' % (name, num_params / 1e6))
        print('-----------------------------------------------')

    def set_requires_grad(self, nets, requires_grad=False):
        """base_model.py:219-230 — a frozen HIP net skips its weight-gradient kernels."""
        if not isinstance(nets, list):
            nets = [nets]
        for net in nets:
            if net is not None:
                for param in net.parameters():
                    param.requires_grad = requires_grad
