"""Data parallelism: one process per GPU, gradient all-reduce over RCCL (xGMI) / gloo (CPU tests).

The reference's only multi-GPU mechanism is nn.DataParallel in init_net
(methods/GAN-based/CycleGAN/models/networks.py:111-116): single-process, replicate-every-forward.
Here each rank holds full replicas of G_A, G_B, D_A, D_B, takes its own B_local frame pairs, and the
two optimizer phases each exchange their networks' flat gradient buffers with ONE bucketed
all_reduce(SUM) per bucket, then scale by 1/world (the gradients of a mean loss over the global
batch, identical to single-GPU B_global up to fp32 summation order: InstanceNorm is per-sample and
every loss is a batch mean).  The flat buffers make the bucket list static, so the exchange is a
handful of large collectives (default 32 MiB) launched back-to-back on a side stream.
"""
import torch
import torch.distributed as dist

from . import ops

BUCKET_BYTES = 32 << 20


def _buckets(flat, nbytes=BUCKET_BYTES):
    step = max(1, nbytes // flat.element_size())
    return [flat[i:i + step] for i in range(0, flat.numel(), step)]


class GradExchange:
    """Callable grad hook for CycleGANModel.optimize_parameters(grad_hook_G=..., grad_hook_D=...)."""

    def __init__(self, world_size=None, group=None, bucket_bytes=BUCKET_BYTES):
        self.world = world_size or dist.get_world_size(group)
        self.group = group
        self.bucket_bytes = bucket_bytes
        self.stream = None

    def __call__(self, nets):
        if self.world == 1:
            return
        flats = [n.flat_grad for n in nets]
        use_side = flats[0].is_cuda
        if use_side:
            if self.stream is None:
                self.stream = torch.cuda.Stream(device=flats[0].device)
            cur = torch.cuda.current_stream(flats[0].device)
            self.stream.wait_stream(cur)
            ctx = torch.cuda.stream(self.stream)
        else:
            ctx = _Null()
        with ctx:
            works = []
            for f in flats:
                for b in _buckets(f, self.bucket_bytes):
                    works.append(dist.all_reduce(b, op=dist.ReduceOp.SUM, group=self.group, async_op=True))
            for w in works:
                w.wait()
            for f in flats:
                if f.is_cuda:
                    ops.axpby(f, f, 1.0 / self.world, 0.0)
                else:
                    f.mul_(1.0 / self.world)
        if use_side:
            cur.wait_stream(self.stream)
            for f in flats:
                f.record_stream(self.stream)


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def broadcast_params(nets, src=0, group=None):
    """Make every rank start from rank src's weights (one broadcast per flat buffer)."""
    for n in nets:
        dist.broadcast(n.flat_param, src=src, group=group)
        n.bump_version()
