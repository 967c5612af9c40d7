"""Option system — the flag names/defaults of methods/GAN-based/CycleGANCon/options/
{base_options.py:20-61, train_options.py:10-40} (the CLI contract of train.py), plus the model hook
``modify_commandline_options`` and the HIP-build extras (--world_size is implied by torchrun).

``parse_options(argv, is_train)`` returns an argparse.Namespace with ``gpu_ids`` parsed to ints
(base_options.py:134-142) and ``isTrain`` set; ``default_opt(**overrides)`` builds one in code.
"""
import argparse

from . import models


def _base(parser):
    a = parser.add_argument
    a('--image_dir', default='', help='FC2 .npy frame-pair directory')
    a('--style_dir', default='', help='styled target images directory')
    a('--name', type=str, default='experiment_name')
    a('--gpu_ids', type=str, default='0', help='e.g. 0  0,1,2, 0,2. use -1 for CPU')
    a('--checkpoints_dir', type=str, default='./checkpoints')
    a('--model', type=str, default='cycle_gan')
    a('--input_nc', type=int, default=3)
    a('--output_nc', type=int, default=3)
    a('--ngf', type=int, default=64)
    a('--ndf', type=int, default=64)
    a('--netD', type=str, default='basic')
    a('--netG', type=str, default='resnet_9blocks')
    a('--n_layers_D', type=int, default=3)
    a('--norm', type=str, default='instance')
    a('--init_type', type=str, default='normal')
    a('--init_gain', type=float, default=0.02)
    a('--no_dropout', action='store_true')
    a('--dataset_mode', type=str, default='unaligned')
    a('--direction', type=str, default='AtoB')
    a('--serial_batches', action='store_true')
    a('--num_threads', default=4, type=int)
    a('--batch_size', type=int, default=1)
    a('--load_size', type=int, default=286)
    a('--crop_size', type=int, default=256)
    a('--max_dataset_size', type=int, default=float("inf"))
    a('--preprocess', type=str, default='resize_and_crop')
    a('--no_flip', action='store_true')
    a('--display_winsize', type=int, default=256)
    a('--epoch', type=str, default='latest')
    a('--load_iter', type=int, default=0)
    a('--verbose', action='store_true')
    a('--suffix', default='', type=str)
    return parser


def _train(parser):
    a = parser.add_argument
    a('--display_freq', type=int, default=400)
    a('--display_ncols', type=int, default=4)
    a('--display_id', type=int, default=0)
    a('--display_server', type=str, default="http://localhost")
    a('--display_env', type=str, default='main')
    a('--display_port', type=int, default=8097)
    a('--update_html_freq', type=int, default=1000)
    a('--print_freq', type=int, default=100)
    a('--no_html', action='store_true')
    a('--save_latest_freq', type=int, default=5000)
    a('--save_epoch_freq', type=int, default=5)
    a('--save_by_iter', action='store_true')
    a('--continue_train', action='store_true')
    a('--epoch_count', type=int, default=1)
    a('--phase', type=str, default='train')
    a('--n_epochs', type=int, default=100)
    a('--n_epochs_decay', type=int, default=100)
    a('--beta1', type=float, default=0.5)
    a('--lr', type=float, default=0.0002)
    a('--gan_mode', type=str, default='lsgan')
    a('--pool_size', type=int, default=50)
    a('--lr_policy', type=str, default='linear')
    a('--lr_decay_iters', type=int, default=50)
    return parser


def parse_options(argv=None, is_train=True):
    parser = argparse.ArgumentParser(formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    _base(parser)
    if is_train:
        _train(parser)
    opt, _ = parser.parse_known_args(argv)
    models.get_option_setter(opt.model)(parser, is_train)
    opt = parser.parse_args(argv)
    opt.isTrain = is_train
    opt.gpu_ids = [int(s) for s in str(opt.gpu_ids).split(',') if int(s) >= 0]
    return opt


def default_opt(is_train=True, **overrides):
    opt = parse_options(["--model", overrides["model"]] if "model" in overrides else [], is_train)
    for k, v in overrides.items():
        setattr(opt, k, v)
    return opt
