"""Data parallelism on the real HIP networks (GPU): two ranks share the box's one GPU over the gloo
backend (CUDA tensors), each running CycleGANModel.optimize_parameters on half of a B=4 batch with
GradExchange attached, i.e. the bucketed all-reduce is launched from inside the HIP generator /
discriminator backward passes (networks.FlatNet._grad_done).  Checks: buckets were launched before
the phase's join (during backward), and the averaged gradients equal the single-process B=4
gradients (InstanceNorm per sample, batch-mean losses)."""
import os
import shutil
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from dist_harness import run_ranks

pytestmark = pytest.mark.gpu


def _setup(B_slice=None):
    from gbvst.cycle_gan_model import CycleGANModel
    from gbvst.options import default_opt
    from oracle import cpu_ref, prng
    g = torch.Generator().manual_seed(5)
    m = CycleGANModel(default_opt(True, ngf=8, ndf=8, pool_size=0, gpu_ids=[0]))
    shapes = {"G": cpu_ref.state_shapes(cpu_ref.RefResnetGenerator(3, 3, 8, 9)),
              "D": cpu_ref.state_shapes(cpu_ref.RefNLayerDiscriminator(3, 8))}
    for i, name in enumerate(("G_A", "G_B", "D_A", "D_B")):
        sd = prng.init_state_dict(shapes[name[0]], base_seed=900 + i)
        getattr(m, "net" + name).load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    a, a2, b, mask, flow = cpu_ref.synthetic_batch(4, 64, 64, gen=g)
    data = [a, a2, b, None, mask, flow]
    if B_slice is not None:
        data = [t[B_slice] if t is not None else None for t in data]
    m.set_input_fc2(tuple(data))
    return m


def _grads_hook(store, ex=None):
    def hook(nets):
        if ex is not None:
            ex(nets)
        for n in nets:
            store[id(n)] = n.flat_grad.detach().cpu().clone()
    return hook


def _worker(rank, world):
    import gbvst
    from gbvst import dp
    gbvst._lib.load()
    torch.cuda.set_device(0)
    m = _setup(slice(rank * 2, rank * 2 + 2))
    nets = [m.netG_A, m.netG_B, m.netD_A, m.netD_B]
    ex = dp.GradExchange(world, bucket_bytes=64 << 10).attach(nets)
    grads = {}
    m.optimize_parameters(_grads_hook(grads, ex), _grads_hook(grads, ex))
    torch.cuda.synchronize()
    logs = {name: list(ex._state(getattr(m, "net" + name)).last_log) for name in ("G_A", "G_B", "D_A", "D_B")}
    out = {name: grads[id(getattr(m, "net" + name))].numpy() for name in ("G_A", "G_B", "D_A", "D_B")}
    return out, logs


@pytest.mark.timeout(600)
def test_dp_world2_overlap_equals_single_process():
    world = 2
    res = [(r, out, logs) for r, (out, logs) in enumerate(run_ranks(_worker, world, timeout=400))]
    import gbvst
    gbvst._lib.load()
    m = _setup()
    grads = {}
    m.optimize_parameters(_grads_hook(grads), _grads_hook(grads))
    torch.cuda.synchronize()
    for name in ("G_A", "G_B", "D_A", "D_B"):
        net = getattr(m, "net" + name)
        full = grads[id(net)].numpy().astype(np.float64)
        r0, r1 = res[0][1][name], res[1][1][name]
        assert np.array_equal(r0, r1), name
        # IN-preceded biases carry rounding noise only: compare per parameter without them
        off = 0
        for k, p in net.named_parameters():
            n = p.numel()
            real_bias = k in ("model.26.bias", "model.0.bias", "model.11.bias")
            if not (k.endswith("bias") and not real_bias):
                ref, got = full[off:off + n], r0[off:off + n].astype(np.float64)
                rel = np.linalg.norm(got - ref) / (np.linalg.norm(ref) + 1e-30)
                assert rel < 1e-4, (name, k, rel)
            off += n
        # buckets went out during that network's last backward pass (before the join)
        assert len(res[0][2][name]) > 0, (name, res[0][2][name])


def _nccl_worker(init_file, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", init_method="file://" + init_file, rank=0, world_size=1,
                                device_id=torch.device("cuda", 0))
        import gbvst
        from gbvst import dp, ops
        gbvst._lib.load()
        ops.set_deterministic(True)
        m = _setup()
        nets = [m.netG_A, m.netG_B, m.netD_A, m.netD_B]
        # force: the world-1 short-circuit is bypassed, so every bucket goes through RCCL
        # all_reduce(async_op=True) launched from inside backward and the join's work.wait()
        ex = dp.GradExchange(1, bucket_bytes=64 << 10, force=True).attach(nets)
        grads = {}
        m.optimize_parameters(_grads_hook(grads, ex), _grads_hook(grads, ex))
        torch.cuda.synchronize()
        logs = {name: list(ex._state(getattr(m, "net" + name)).last_log) for name in ("G_A", "G_B", "D_A", "D_B")}
        out = {name: grads[id(getattr(m, "net" + name))].numpy() for name in ("G_A", "G_B", "D_A", "D_B")}
        w = {name: getattr(m, "net" + name).flat_param.detach().cpu().numpy() for name in ("G_A", "D_A")}
        q.put((out, logs, w, dist.get_backend(), None))
        dist.destroy_process_group()
    except Exception:  # report, do not hang the parent
        import traceback
        q.put((None, None, None, None, traceback.format_exc()))


@pytest.mark.timeout(600)
def test_dp_nccl_world1_forced_buckets():
    """The RCCL path on hardware: a one-rank `nccl` (= RCCL) process group with the bucketed exchange
    forced on.  Buckets are all_reduce(async_op=True) calls enqueued from inside the HIP backward
    passes; the join makes the compute stream wait on them before Adam.  A one-rank sum is the
    identity and both runs use the deterministic warp backward, so the step must equal the run without
    any exchange BIT FOR BIT — any stream-ordering fault (Adam reading a bucket before RCCL wrote it
    back, or the join's scaling racing the collective) shows as a differing gradient or weight."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    tmp = tempfile.mkdtemp(prefix="vst_pg_")
    p = ctx.Process(target=_nccl_worker, args=(os.path.join(tmp, "store"), q))
    p.start()
    out, logs, w, backend, err = q.get(timeout=400)
    p.join(timeout=120)
    shutil.rmtree(tmp, ignore_errors=True)
    assert err is None, err
    assert p.exitcode == 0
    assert backend == "nccl"
    import gbvst
    from gbvst import ops
    gbvst._lib.load()
    prev = ops.set_deterministic(True)
    try:
        m = _setup()
        grads = {}
        m.optimize_parameters(_grads_hook(grads), _grads_hook(grads))
        torch.cuda.synchronize()
    finally:
        ops.set_deterministic(prev)
    for name in ("G_A", "G_B", "D_A", "D_B"):
        net = getattr(m, "net" + name)
        ref = grads[id(net)].numpy()
        assert np.array_equal(out[name], ref), (name, np.abs(out[name] - ref).max())
        assert len(logs[name]) > 0, (name, logs[name])   # launched during backward, not at the join
    for name in ("G_A", "D_A"):
        ref = getattr(m, "net" + name).flat_param.detach().cpu().numpy()
        assert np.array_equal(w[name], ref), (name, np.abs(w[name] - ref).max())


# ------------------------------------------------------------------------------ MoGAN (config C5)
# The three exchange phases of MoGAN/models/cycle_gan_model.py:315-352 under DP: the E-step's G and D
# gradients (grad_hook_G / grad_hook_D) and the M-step's motion-net gradients (grad_hook_M), each
# bucket launched from inside that phase's last backward pass.  Every per-sample piece (G / D / M, RAFT,
# warp, fb-check) is batch-independent and every loss a batch mean, so two ranks on half batches with
# averaged gradients equal one process on the whole batch.  Both sides run the deterministic warp
# backward, so the only difference left is the split-K order of the weight gradients (batch size).
_MG_NAMES = ("G_A", "G_B", "D_A", "D_B", "M_A", "M_B")


def _mogan_setup(B_slice=None):
    import argparse
    from gbvst import mogan_model, raft
    from gbvst.options import default_opt
    from oracle import cpu_ref, prng, raft_ref
    r = raft.RAFT(argparse.Namespace(small=False))
    shapes = {k: tuple(v.shape) for k, v in r.state_dict().items()}
    r.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in raft_ref.raft_weights(shapes, 1300, 1e-3).items()})
    opt = default_opt(True, model="mogan", ngf=8, ndf=8, pool_size=0, gpu_ids=[0])
    m = mogan_model.MoGANModel(opt, raft_model=r.to("cuda").eval(), raft_iters=4)
    for i, name in enumerate(_MG_NAMES):
        net = getattr(m, "net" + name)
        sd = prng.init_state_dict(cpu_ref.state_shapes(net), base_seed=950 + i)
        net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    # the E-step's G / D updates frozen (lr 0; the exchange still runs in all three phases): Adam's first
    # step is ~lr * sign(g), so rounding-level differences between the rank-averaged and the whole-batch
    # gradients of near-zero entries would move those weights by up to 2 lr on one side only, and the
    # M-step's RAFT flows of the fake frames amplify that (measured: M_A 2.8e-3 with lr 2e-4)
    for o in (m.optimizer_G, m.optimizer_D):
        o.param_groups[0]["lr"] = 0.0
    imgs = [torch.from_numpy(prng.uniform_f32(960 + i, (4, 3, 128, 128), -1.0, 1.0)) for i in range(4)]
    if B_slice is not None:
        imgs = [t[B_slice] for t in imgs]
    m.set_input_fc2(imgs)
    return m


def _mogan_run(m, ex=None):
    """E-step then M-step; returns {phase: {net: flat grad}} captured at each phase's hook."""
    grads = {"E": {}, "M": {}}

    def hook(phase):
        def h(nets):
            if ex is not None:
                ex(nets)
            for n in nets:
                grads[phase][id(n)] = n.flat_grad.detach().cpu().clone()
        return h
    m.optimize_parameters(hook("E"), hook("E"), hook("E"))
    m.optimize_parameters(hook("M"), hook("M"), hook("M"))
    torch.cuda.synchronize()
    out = {}
    for phase, names in (("E", _MG_NAMES[:4]), ("M", _MG_NAMES[4:])):
        out[phase] = {n: grads[phase][id(getattr(m, "net" + n))].numpy() for n in names}
    return out


def _mogan_worker(rank, world):
    import gbvst
    from gbvst import dp, ops
    gbvst._lib.load()
    torch.cuda.set_device(0)
    ops.set_deterministic(True)
    m = _mogan_setup(slice(rank * 2, rank * 2 + 2))
    nets = [getattr(m, "net" + n) for n in _MG_NAMES]
    ex = dp.GradExchange(world, bucket_bytes=64 << 10).attach(nets)
    out = _mogan_run(m, ex)
    logs = {n: list(ex._state(getattr(m, "net" + n)).last_log) for n in _MG_NAMES}
    return out, logs


@pytest.mark.timeout(600)
def test_mogan_dp_world2_three_phases_equal_single_process():
    world = 2
    res = [(r, out, logs) for r, (out, logs) in enumerate(run_ranks(_mogan_worker, world, timeout=500))]
    import gbvst
    from gbvst import ops
    gbvst._lib.load()
    prev = ops.set_deterministic(True)
    try:
        m = _mogan_setup()
        full = _mogan_run(m)
        # each rank's half batch in one process: what the exchange must average
        halves = [_mogan_run(_mogan_setup(slice(2 * r, 2 * r + 2))) for r in range(world)]
    finally:
        ops.set_deterministic(prev)

    def rel_by_param(net, a, b):
        off = 0
        for k, p in net.named_parameters():
            n = p.numel()
            in_bias = k.endswith("bias") and k not in ("model.26.bias", "model.0.bias", "model.11.bias")
            if not in_bias:
                x, y = a[off:off + n].astype(np.float64), b[off:off + n].astype(np.float64)
                yield k, np.linalg.norm(x - y) / (np.linalg.norm(y) + 1e-30)
            off += n

    # (1) the exchange: every rank holds the mean of the ranks' half-batch gradients (to fp32 rounding
    #     of the bucketed all-reduce).  (2) DP vs the whole batch in one process: the E-step to 1e-4; the
    #     M-step's AM loss is an L1 of M(bf_real) against RAFT's flow of the fake frames, whose batch-size-
    #     dependent plans round differently — sign flips of near-zero residuals move its gradients by
    #     ~3e-3 (measured), so 1e-2 there
    for phase, tol in (("E", 1e-4), ("M", 1e-2)):
        for name, ref in full[phase].items():
            r0, r1 = res[0][1][phase][name], res[1][1][phase][name]
            assert np.array_equal(r0, r1), (phase, name)
            net = getattr(m, "net" + name)
            mean = (halves[0][phase][name].astype(np.float64) + halves[1][phase][name]) / world
            for k, rel in rel_by_param(net, r0, mean):
                assert rel < 1e-6, ("exchange", phase, name, k, rel)
            for k, rel in rel_by_param(net, r0, ref):
                assert rel < tol, (phase, name, k, rel)
            assert len(res[0][2][name]) > 0, (phase, name)   # buckets launched during backward
