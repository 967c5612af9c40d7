"""Data parallelism: one process per GPU, gradient all-reduce over RCCL (xGMI) / gloo (CPU tests).

The reference's only multi-GPU mechanism is nn.DataParallel in init_net
(methods/GAN-based/CycleGAN/models/networks.py:111-116): single-process, replicate-every-forward,
gradients reduced onto GPU 0 during backward.  Here each rank holds full replicas of G_A, G_B, D_A,
D_B, takes its own B_local frame pairs, and the two optimizer phases each average their networks'
flat gradient buffers across ranks (identical to single-GPU B_global up to fp32 summation order:
InstanceNorm is per sample and every loss is a batch mean).

Overlap with backward: ``GradExchange.attach(nets)`` splits each network's flat gradient buffer into
fixed buckets (default 8 MiB, cut from the END of the buffer, i.e. reverse layer order) and hooks
the networks' backward passes (networks.FlatNet._grad_done).  During the LAST backward pass of a
phase — the pass after which no more gradient accumulates into the buffer — each layer reports that
its gradient slice is final; every bucket lying entirely at or above that layer is then handed to
``dist.all_reduce(async_op=True)`` at once.  With the NCCL (= RCCL) backend the collective is
enqueued on the process group's own stream behind an event on the compute stream, so it runs
beside the remaining backward kernels.  The join (``__call__``, passed as grad_hook_G/_D to
optimize_parameters) launches whatever is left, makes the compute stream wait for every bucket,
and scales by 1/world before the Adam step.  In the CycleGANCon G step this overlaps G_B's whole
exchange and most of G_A's with G_A's last (batched) backward pass; in the D step D_A's exchange
overlaps D_B's backward.  Without ``attach`` the join simply runs the whole exchange.
"""
import torch
import torch.distributed as dist

from . import ops

BUCKET_BYTES = 8 << 20


def _bucket_bounds(n, elem, nbytes=BUCKET_BYTES):
    """[(lo, hi)] covering [0, n), cut from the end: bucket 0 = the LAST elements (ready first)."""
    step = max(1, nbytes // elem)
    out, hi = [], n
    while hi > 0:
        lo = max(0, hi - step)
        out.append((lo, hi))
        hi = lo
    return out


class _NetState:
    def __init__(self, net, bucket_bytes):
        self.net = net
        self.bounds = _bucket_bounds(net.flat_grad.numel(), net.flat_grad.element_size(), bucket_bytes)
        self.next = 0          # index of the next bucket to launch
        self.works = []
        self.launch_log = []   # (bucket index, ready offset) per early launch in the current phase
        self.last_log = []     # launch_log of the last completed phase (tests / diagnostics)


class GradExchange:
    """Callable grad hook for CycleGANModel.optimize_parameters(grad_hook_G=..., grad_hook_D=...)
    (the join); ``attach(nets)`` additionally launches buckets during backward."""

    def __init__(self, world_size=None, group=None, bucket_bytes=BUCKET_BYTES, force=False):
        """force: run the bucketed collectives even at world 1 (they are identities there), so the
        single-GPU test exercises the RCCL async_op / wait stream ordering on hardware."""
        self.world = world_size or dist.get_world_size(group)
        self.group = group
        self.bucket_bytes = bucket_bytes
        self.force = force
        self._states = {}

    def _state(self, net):
        st = self._states.get(id(net))
        if st is None or st.net is not net or st.bounds[0][1] != net.flat_grad.numel():
            st = _NetState(net, self.bucket_bytes)
            self._states[id(net)] = st
        return st

    def attach(self, nets):
        """Hook each network's backward: buckets are all-reduced as soon as the phase's last
        backward pass has written them."""
        if self.world == 1 and not self.force:
            return self
        for net in nets:
            st = self._state(net)
            net._grad_ready_cb = lambda off, st=st: self._on_ready(st, off)
        return self

    def _launch(self, st, i):
        lo, hi = st.bounds[i]
        b = st.net.flat_grad[lo:hi]
        st.works.append(dist.all_reduce(b, op=dist.ReduceOp.SUM, group=self.group, async_op=True))

    def _on_ready(self, st, off):
        # every gradient at flat offset >= off is final: launch each bucket that lies above it
        while st.next < len(st.bounds) and st.bounds[st.next][0] >= off:
            st.launch_log.append((st.next, off))
            self._launch(st, st.next)
            st.next += 1

    def __call__(self, nets):
        """Join: launch the remaining buckets, wait for all, average."""
        if self.world == 1 and not self.force:
            for n in nets:
                _reset(n)
            return
        states = [self._state(n) for n in nets]
        for st in states:
            while st.next < len(st.bounds):
                self._launch(st, st.next)
                st.next += 1
        for st in states:
            for w in st.works:
                w.wait()   # NCCL: the current (compute) stream waits for the comm stream
            st.works = []
            st.next = 0
            st.last_log, st.launch_log = st.launch_log, []
            f = st.net.flat_grad
            if f.is_cuda:
                ops.axpby(f, f, 1.0 / self.world, 0.0)
            else:
                f.mul_(1.0 / self.world)
            _reset(st.net)


def _reset(net):
    r = getattr(net, "_reset_pending", None)
    if r is not None:
        r()


def broadcast_params(nets, src=0, group=None):
    """Make every rank start from rank src's weights (one broadcast per flat buffer)."""
    for n in nets:
        dist.broadcast(n.flat_param, src=src, group=group)
        n.bump_version()
