"""Training entry — the epoch loop of methods/GAN-based/CycleGANCon/train.py:29-130 and the loss log of
util/visualizer.py:52-85,205-221, on the HIP models.

Usage (one process per GPU; ``torchrun --nproc-per-node N -m gbvst.train ...`` for data parallel):

    python -m gbvst.train --image_dir FC2/data/ --style_dir FC2/style/ --name fc2_cyclegan --model cycle_gan
    python -m gbvst.train --synthetic 64 --crop_size 256 --batch_size 4 --n_epochs 1 --n_epochs_decay 0

Same flags, schedule and side effects as the reference loop:
* ``update_learning_rate()`` at the start of every epoch (train.py:62);
* ``print_current_losses`` every ``print_freq`` images, into ``<checkpoints_dir>/<name>/loss_log.txt`` with
  the reference's line format ``(epoch: %d, iters: %d, time: %.3f, data: %.3f) name: %.3f ...``;
* ``save_networks('latest' | 'iter_%d')`` every ``save_latest_freq`` images, and ``'latest'`` + the
  epoch number every ``save_epoch_freq`` epochs (train.py:119-128).
Data parallel (WORLD_SIZE > 1): RCCL process group, rank-0 weights broadcast, the bucketed gradient
all-reduce launched from inside backward (dp.GradExchange); each rank reads its own shard of the
dataset; rank 0 alone logs and checkpoints.  Visdom / HTML display (display_id > 0) is not built.
"""
import os
import sys
import time

import torch
import torch.distributed as dist


class Visualizer:
    """util/visualizer.py — the loss-log part (header at construction, one line per print)."""

    def __init__(self, opt, enabled=True):
        self.enabled = enabled
        self.log_name = os.path.join(opt.checkpoints_dir, opt.name, 'loss_log.txt')
        if enabled:
            os.makedirs(os.path.dirname(self.log_name), exist_ok=True)
            with open(self.log_name, "a") as log_file:
                log_file.write('================ Training Loss (%s) ================\n' % time.strftime("%c"))

    def reset(self):
        pass

    @staticmethod
    def format_losses(epoch, iters, losses, t_comp, t_data):
        """visualizer.py:215-217."""
        message = '(epoch: %d, iters: %d, time: %.3f, data: %.3f) ' % (epoch, iters, t_comp, t_data)
        for k, v in losses.items():
            message += '%s: %.3f ' % (k, v)
        return message

    def print_current_losses(self, epoch, iters, losses, t_comp, t_data):
        message = self.format_losses(epoch, iters, losses, t_comp, t_data)
        if self.enabled:
            print(message)
            with open(self.log_name, "a") as log_file:
                log_file.write('%s\n' % message)
        return message


class SyntheticFC2:
    """Device-resident synthetic FC2 batches (SURVEY §8d shapes: [-1,1] frames, smooth flow, 0/1 mask),
    yielded in the loader format ``(real_A, real_A2, real_B, mask, flow)`` that ``set_input_nhwc`` takes.
    ``num_images`` pairs per epoch, ``batch_size`` per step; seeded per rank."""

    def __init__(self, num_images, batch_size, size, device, seed=0):
        self.num_images, self.batch_size, self.size = num_images, batch_size, size
        self.device, self.seed, self.epoch = torch.device(device), seed, 0

    def __len__(self):
        return self.num_images

    def __iter__(self):
        from . import ops
        import torch.nn.functional as F
        g = torch.Generator().manual_seed(self.seed * 1000003 + self.epoch)
        self.epoch += 1
        S = self.size
        for i in range(0, self.num_images, self.batch_size):
            B = min(self.batch_size, self.num_images - i)
            imgs = [((torch.randint(0, 256, (B, 3, S, S), generator=g).float() / 255.0) - 0.5) / 0.5
                    for _ in range(3)]
            flow = F.interpolate(torch.randn(B, 2, 9, 9, generator=g) * 4.0, size=(S, S), mode="bicubic",
                                 align_corners=True)
            mask = F.interpolate((torch.rand(B, 1, 32, 32, generator=g) < 0.8).float(), size=(S, S),
                                 mode="nearest")
            a, a2, b = [ops.nchw_to_nhwc(t.to(self.device)) for t in imgs]
            yield a, a2, b, mask.to(self.device).contiguous(), flow.to(self.device).contiguous()


def _set_input(model, data):
    """Loader tuples: 5-tuple device NHWC (FC2Loader / SyntheticFC2) or the reference's 6-tuple
    ``(img1, img2, simg, label, mask, flow)`` NCHW (cycle_gan_model.py:124-131)."""
    if len(data) == 5:
        model.set_input_nhwc(*data)
    else:
        model.set_input_fc2(data)


def _optimize(model, grad_hook):
    """optimize_parameters with the DP exchange on EVERY optimizer phase the model has: G and D, plus
    MoGAN's motion-net phase (grad_hook_M, MoGAN/models/cycle_gan_model.py:315-352) — a phase without
    the exchange would let that phase's replicas diverge across ranks."""
    import inspect
    if grad_hook is None:
        return model.optimize_parameters()
    params = inspect.signature(model.optimize_parameters).parameters
    if "grad_hook_M" in params:
        return model.optimize_parameters(grad_hook, grad_hook, grad_hook_M=grad_hook)
    extra = [p for p in params if p.startswith("grad_hook") and p not in ("grad_hook_G", "grad_hook_D")]
    if extra:
        raise NotImplementedError("data-parallel training of %s: optimizer phases %s have no gradient "
                                  "exchange" % (type(model).__name__, extra))
    return model.optimize_parameters(grad_hook, grad_hook)


def shard_indices(n, world, rank):
    """DistributedSampler (drop_last=True, no shuffle) shard: rank r takes items r, r+world, ... of the
    first world*floor(n/world) items, so every rank holds the same count and runs the same number of
    batches (a rank with one more batch would block forever in its gradient all-reduce)."""
    usable = (n // world) * world
    return list(range(rank, usable, world))


def train(opt, dataset, model=None, world=1, rank=0, grad_hook=None, log=print):
    """train.py:48-130.  ``dataset``: an iterable of batches with ``len()`` = images per epoch (per rank).
    Returns (model, total_iters)."""
    from . import models
    dataset_size = len(dataset)
    log('The number of training images = %d' % dataset_size)
    if model is None:
        model = models.create_model(opt)
    model.setup(opt)
    visualizer = Visualizer(opt, enabled=(rank == 0))
    total_iters = 0
    last_epoch = opt.n_epochs + opt.n_epochs_decay
    for epoch in range(opt.epoch_count, last_epoch + 1):
        epoch_start_time = time.time()
        iter_data_time = time.time()
        epoch_iter = 0
        visualizer.reset()
        model.update_learning_rate()
        t_data = 0.0
        for data in dataset:
            iter_start_time = time.time()
            if total_iters % opt.print_freq == 0:
                t_data = iter_start_time - iter_data_time
            total_iters += opt.batch_size
            epoch_iter += opt.batch_size
            _set_input(model, data)
            _optimize(model, grad_hook)
            if total_iters % opt.print_freq == 0:
                losses = model.get_current_losses()  # one host sync, as the reference's float(loss)
                t_comp = (time.time() - iter_start_time) / opt.batch_size
                visualizer.print_current_losses(epoch, epoch_iter, losses, t_comp, t_data)
            if total_iters % opt.save_latest_freq == 0 and rank == 0:
                log('saving the latest model (epoch %d, total_iters %d)' % (epoch, total_iters))
                model.save_networks('iter_%d' % total_iters if opt.save_by_iter else 'latest')
            iter_data_time = time.time()
        if epoch % opt.save_epoch_freq == 0 and rank == 0:
            log('saving the model at the end of epoch %d, iters %d' % (epoch, total_iters))
            model.save_networks('latest')
            model.save_networks(epoch)
        if world > 1:
            dist.barrier()
        log('End of epoch %d / %d \t Time Taken: %d sec' % (epoch, last_epoch, time.time() - epoch_start_time))
    return model, total_iters


def _add_entry_flags(argv):
    """Flags of this entry point only (not the reference's option set): --synthetic N."""
    synthetic = 0
    rest = []
    it = iter(argv)
    for a in it:
        if a == '--synthetic':
            synthetic = int(next(it))
        elif a.startswith('--synthetic='):
            synthetic = int(a.split('=', 1)[1])
        else:
            rest.append(a)
    return synthetic, rest


def main(argv=None):
    from . import _lib, dp, models
    from .fc2 import DatasetFC2, FC2Loader
    from .options import parse_options
    synthetic, argv = _add_entry_flags(sys.argv[1:] if argv is None else argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    opt = parse_options(argv, is_train=True)
    opt.gpu_ids = [local] if world > 1 else (opt.gpu_ids or [0])
    device = torch.device("cuda", opt.gpu_ids[0])
    torch.cuda.set_device(device)
    _lib.load()
    if synthetic:
        dataset = SyntheticFC2(synthetic, opt.batch_size, opt.crop_size, device, seed=rank)
    else:
        full = DatasetFC2(opt.image_dir, opt.style_dir)
        if world > 1:  # rank r reads images r, r+world, ... of an equal-size shard (DistributedSampler)
            full.dataset = [full.dataset[i] for i in shard_indices(len(full.dataset), world, rank)]
            full.num_images = len(full.dataset)
        dataset = FC2Loader(full, batch_size=opt.batch_size, shuffle=not opt.serial_batches,
                            max_dataset_size=opt.max_dataset_size, device=device, seed=rank, drop_last=world > 1)
    model = models.create_model(opt)
    hook = None
    if world > 1:
        nets = [getattr(model, 'net' + n) for n in model.model_names]
        dp.broadcast_params(nets)
        hook = dp.GradExchange(world).attach(nets)
    train(opt, dataset, model=model, world=world, rank=rank, grad_hook=hook,
          log=print if rank == 0 else (lambda *_: None))
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == '__main__':
    sys.exit(main())
