#!/usr/bin/env python3
"""Benchmark: CycleGAN video train step (G + D + flow-warp temporal loss), 256x256, B=4 per GPU.

BASELINE.json metric "frames/sec: CycleGAN train step (G+D+flow-warp loss) 256x256 at 1/2/4/8 GPUs".
One step = CycleGANModel.optimize_parameters() (CycleGANCon semantics: 7 generator passes, 6
discriminator passes, temporal warp loss, two Adam updates) over one synthetic batch already
resident in HBM.  Weak scaling: every rank processes B_local=4 frame pairs; value = all frames
processed by all ranks / max-over-ranks wall time of exactly K steps (barrier + device sync on both
sides).  Multi-GPU: one process per GPU (torchrun), gradients exchanged with RCCL all_reduce.

Also reported (same JSON line):
  math          the conv arithmetic of the headline: bf16x6 (fp32-equivalent split products) in
                every forward, data-gradient and weight-gradient conv (--math / VST_CONV_MATH).
  roofline      the dominant conv launch of the step by time, out of roofline_convs: the ResnetBlock
                3x3 conv forward / stride-1 dgrad / wgrad at N=2B=8 (the batched G_A calls), each
                timed with HIP events around each of its launches inside the timed steps:
                algorithmic FLOPs / avg duration vs the ceiling of the arithmetic it runs; traffic =
                PMC-measured HBM bytes per launch from the committed record (PMC_FILE) when that record
                matches the policy / tile / shape, else null.
  mixed_policy  the same step under the round-1 "mixed" policy (x6 forwards, x3 gradients), labelled.
  cpu_baseline  rank 0 only, N=1: the CPU oracle (stock PyTorch, NCHW fp32) with the GPU run's
  parity        initial weights and synthetic batch, on all the CPUs this process may use: one
                warm-up step whose losses are checked against the GPU's step-0 losses (parity),
                then 2 timed B=4 steps (oracle is imported only for this leg).
  inference     generator-only inference fps at 256x256, B=16 (north_star's secondary number),
                under the headline policy.
  extras        generator inference at the Sintel size (1x436x1024); the flow-warp kernel's HBM
                roofline on the SURVEY §8d large synthetic (N=32, C=64, 436x1024); the RAFT
                correlation volume build at fmaps 1x256x55x128; the Johnson (FastStyleNet + VGG16
                perceptual loss) train step at B=4, 256x256.
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3      # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 (spec; 155 measured)
BF16_MFMA_PEAK_TFLOPS = 2500.0     # dense bf16 (v_mfma_f32_32x32x16_bf16); bf16x6 = 6 products / fp32 MAC
HBM_PEAK_GBS = 8000.0              # MI355X_MICROARCH.md: HBM3E 8 TB/s spec (~6.3 achievable)
TRAIN_TFLOP_PER_FRAME = 2.1753     # SURVEY §8d / BASELINE.md: CycleGANCon step conv FLOPs @256^2
TRAIN_TFLOP_PER_FRAME_C3 = 14.831  # the same step's G/D conv FLOPs @1024x436 (VGG not counted)
G_GFLOP_PER_FRAME = 99.10          # ResnetGenerator fwd @256^2


def synthetic_batch(B, H, W, seed, device):
    """SURVEY §8d synthetic C2 inputs: (u8/255-0.5)/0.5 images, smooth flow (bicubic upsample of an
    N(0,4^2) 9x9 grid), Bernoulli(0.8) mask on a 32x32 grid — generated on the device."""
    import torch.nn.functional as F
    g = torch.Generator(device="cpu").manual_seed(seed)
    imgs = [((torch.randint(0, 256, (B, 3, H, W), generator=g).float() / 255.0) - 0.5) / 0.5 for _ in range(3)]
    coarse = torch.randn(B, 2, 9, 9, generator=g) * 4.0
    flow = F.interpolate(coarse, size=(H, W), mode="bicubic", align_corners=True)
    mcoarse = (torch.rand(B, 1, 32, 32, generator=g) < 0.8).float()
    mask = F.interpolate(mcoarse, size=(H, W), mode="nearest")
    return [t.to(device).contiguous() for t in imgs + [mask, flow]]


def _time_on_stream(fn, reps, warm=3):
    """Average ms per call of fn() launched on a dedicated stream, HIP events on that stream."""
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(warm):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            fn()
        e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


# The step's dominant conv launches: the ResnetBlock 3x3 reflect 256->256 @64x64 convs of the batched
# generator calls (N = 2B frames: G_A[real_A, real_A2] and G_A[fake_A, real_B]) — the forward, the
# stride-1 data gradient (a forward conv over the rotated taps onto the 66x66 padded frame: zero pad 2,
# the key that separates it from the forward) and the weight gradient.  Keys: ops.LaunchProbe.
def DOMINANT_KEYS(B):
    N = 2 * B
    return {"resblock_fprop": ("fwd", (N, 64, 64, 256, 256, 3, 1, 1, "reflect")),
            "resblock_dgrad": ("dgrad", (N, 64, 64, 256, 256, 3, 1, 1, "reflect")),
            "resblock_wgrad": ("wgrad", (N, 64, 64, 256, 256, 3, 1, 1, "reflect"))}


PMC_FILE = os.path.join(HERE, "profiles", "r06z_conv_pmc.json")
PROBE_EVERY = 13  # conv_roofline's sampling stride (ops.LaunchProbe.every)


def _pmc_record(name, key):
    """This kernel's entry of the committed rocprofv3 PMC record, only if it was taken on the same
    policy, tile and shape and on the same kernel sources / knobs (source stamp); else None."""
    try:
        rec = json.load(open(PMC_FILE)).get(name)
    except (OSError, ValueError):
        return None
    if not rec or any(rec.get("key", {}).get(k) != v for k, v in key.items()):
        return None
    from gbvst import _lib
    if rec.get("source_stamp") != _lib.source_stamp():   # taken on other kernel code or knobs
        return None
    return rec


def _pmc_traffic(name, key):
    """HBM bytes per launch from the PMC record (FETCH_SIZE x2 per the gfx950 wide-read correction +
    WRITE_SIZE, separate passes), or None."""
    rec = _pmc_record(name, key)
    return rec.get("hbm_bytes_per_launch") if rec else None


NOMINAL_CLOCK_GHZ = 2.4   # the clock the dense MFMA peaks are quoted at (MI355X_MICROARCH.md)


def _held_clock(entry, name, key):
    """peak_at_held_clock: the ceiling scaled to the clock the chip held under this kernel (the PMC
    record's SQ_WAVE_CYCLES-derived effective clock), and the fraction against it — the DVFS share of
    the gap to the nominal-clock ceiling as a number."""
    rec = _pmc_record(name, key)
    clk = rec.get("effective_clock_GHz") if rec else None
    if not clk:
        entry.update(held_clock_GHz=None, peak_at_held_clock=None, frac_at_held_clock=None)
        return entry
    pk = entry["peak"] * clk / NOMINAL_CLOCK_GHZ
    entry.update(held_clock_GHz=clk, peak_at_held_clock=round(pk, 1), frac_at_held_clock=round(entry["achieved"] / pk, 4),
                 mfma_busy_at_held_clock=rec.get("mfma_busy_frac_actual_clock"))
    return entry


def _mfma(m):
    """The MFMA instruction the split-bf16 GEMMs of arithmetic m issue in this build (vst_build_info)."""
    from gbvst import ops
    if m == "fp32":
        return "v_mfma_f32_32x32x2_f32"
    info = ops.lib().vst_build_info().decode()
    tag = "x6_mfma=" if m == "bf16x6" else "x3_mfma="
    shape = info.split(tag)[1].split()[0] if tag in info else "32x32x16"
    return "v_mfma_f32_%s_bf16" % shape


def _rb_nhwc(N, H, W, C):
    from gbvst import networks
    return networks._rb_wgrad_nhwc(N, H, W, C)


def conv_roofline(name, probe, math):
    """Roofline entry of one probed conv: algorithmic FLOPs (2*M*N*K of the conv it computes) per
    launch / the average duration of its launches inside the timed steps (HIP events on the launch
    stream) vs the ceiling of the arithmetic it executes (dense bf16 MFMA peak / 6 products per
    fp32-equivalent MAC for bf16x6, / 3 for bf16x3; the fp32 MFMA peak for fp32)."""
    from gbvst import ops
    if not probe.events:
        return None
    ms = probe.mean_ms()
    op, (N, H, W, Cx, Cop, R, st, pad, mode) = probe.key
    flop = 2.0 * (N * 64 * 64) * 256 * (256 * 9)
    role = "bwd" if name != "resblock_fprop" else "fwd"
    m = ops._POLICIES[math][role]
    peak = {"bf16x6": BF16_MFMA_PEAK_TFLOPS / 6.0, "bf16x3": BF16_MFMA_PEAK_TFLOPS / 3.0,
            "fp32": FP32_MFMA_PEAK_TFLOPS}[m]
    achieved = flop / (ms * 1e-3) / 1e12
    if op == "fwd":
        kind, ms_ = ops.conv_plan_fwd(N, H, W, Cx, Cop, R, R, st, pad, pad, m)
        ks = ops.conv_plan_fwd_tail(N, H, W, Cx, Cop, R, R, st, pad, m) if (ms_ and ops.FWD_SPLITK) else 0
        tail = (" + split-K tail (%d splits) + reduction" % ks) if ks else (" + small-tile tail launch" if ms_ else "")
        kernel = "conv_fprop_bf_k<%s, %s, %s>%s" % (ops.TILE_NAMES.get(kind, kind), m, _mfma(m), tail)
        key = {"math": m, "tile": kind, "m_split": ms_, "N": N, "mfma": _mfma(m), "ksplit": ks}
        note = ("stride-1 data gradient as a forward conv over the rotated taps (66x66 padded frame)"
                if name == "resblock_dgrad" else "ResnetBlock conv forward")
    elif op == "dgrad":
        from gbvst import networks
        key = {"math": m, "N": N, "mfma": _mfma(m), "op": "dgrad_refl"}
        if networks.DGRAD_EPI:
            kernel = ("vst_conv2d_dgrad_refl_in_epi: conv_fprop_bf_inb_k interior (zero pad 1, %s; the IN-backward "
                      "partials of the layer below in its epilogue) + the K-restricted border GEMM (split-K "
                      "conv_fprop_bf_k<REFL=5>, 128x128) + dgrad_border5_add_inb_k [%s]" % (m, _mfma(m)))
            note = ("stride-1 reflect data gradient as the step runs it: interior conv + border GEMM + the border add "
                    "with the IN-backward partials (traffic: the PMC record of the same GEMMs without the partials)")
        else:
            kernel = ("vst_conv2d_dgrad_refl: conv_fprop_bf_k interior (zero pad 1, %s) + the K-restricted border "
                      "GEMM (split-K conv_fprop_bf_k<REFL=5>, 128x128) + dgrad_border5_add_k [%s]" % (m, _mfma(m)))
            note = ("stride-1 reflect data gradient: interior conv + border GEMM (no padded frame, no fold); "
                    "dgrad_border5_add_k adds the border slabs")
    elif m == "bf16x6" and _rb_nhwc(N, H, W, Cx):
        # round 6: x = the conv's own NHWC fp32 input, dy = the NHWC bf16 planes the planes-only IN backward
        # writes; the kernel stages both through k-major LDS images (ds_read_b64_tr_b16)
        kernel = ("vst_conv2d_wgrad_nhwc: conv_wgrad_nhwc_k (x NHWC fp32 split in the kernel + dy NHWC planes, "
                  "split-K slabs) + slab_group_sum_k / wgrad_reduce_store_k [%s]" % _mfma(m))
        key = {"math": m, "N": N, "mfma": _mfma(m)}
        note = "whole weight-gradient op as the train step runs it (its launches timed together)"
        name = "resblock_wgrad_nhwc"  # the PMC record of this route (tools/kbench.py wgrad_nhwc)
    else:
        # the step's route (networks.py IN_XT / IN_PLANES): the IN apply writes x's padded channel-major
        # image and the IN backward dy's bf16 planes, so the op is the GEMM + the split-K reduction
        kernel = ("vst_conv2d_wgrad on producer-written operands (x image from the IN apply, dy planes from the "
                  "IN backward): conv_wgrad_bf_k (split-K slabs) + wgrad_reduce_store_k, %s" % m if m != "fp32" else
                  "vst_conv2d_wgrad: channel-major copies + conv_wgrad_rk_k + wgrad_reduce_store_k, fp32")
        key = {"math": m, "N": N, "mfma": _mfma(m)}
        kernel += " [%s]" % _mfma(m)
        note = "whole weight-gradient op as the train step runs it (its launches timed together)"
        name = "resblock_wgrad_pre"   # the PMC record of this route (tools/kbench.py wgrad_pre)
    entry = {"kernel": kernel, "what": note + " — ResnetBlock 3x3 reflect 256->256 @64x64, N=%d" % N,
             "bound": "mfma", "achieved": round(achieved, 2), "peak": round(peak, 1), "unit": "TFLOP/s",
             "frac": round(achieved / peak, 4),
             "peak_basis": "dense bf16 MFMA %.0f TFLOP/s / products per fp32-equivalent MAC (%s)" % (BF16_MFMA_PEAK_TFLOPS, m),
             "traffic": _pmc_traffic(name, key), "avg_launch_ms": round(ms, 4), "flop_per_launch": flop,
             "launches_timed": len(probe.events), "launches_per_step": round(probe.seen / max(1, probe.steps), 2),
             "timing": "HIP event pair around 1 launch in %d of this op inside the timed steps" % probe.every,
             "ms_per_step": round(ms * probe.seen / max(1, probe.steps), 3),
             "fp32_mfma_peak": FP32_MFMA_PEAK_TFLOPS}
    return _held_clock(entry, name, key)


def warp_roofline(device, N=32, C=64, H=436, W=1024, reps=10):
    """vst_warp_fwd (utils/flowtools.py warp) on the SURVEY §8d large synthetic: HBM-bound; algorithmic
    bytes = N*H*W*(4C gather-once + 8 flow + 4C write).  The flow is §8d's generator at the Sintel size
    (bicubic upsample of an N(0, 4^2) 9x9 grid, x4 as for C3: smooth, up to ~+-40 px); the same kernel on
    an i.i.d. N(0, 3^2) px per-pixel flow (no neighbour locality: every corner a separate cache line
    set) is reported as the worst case."""
    import torch.nn.functional as F
    from gbvst import ops
    x = torch.randn(N, H, W, C, device=device)
    g = torch.Generator(device="cpu").manual_seed(4321)
    coarse = torch.randn(N, 2, 9, 9, generator=g) * 4.0
    flow = (F.interpolate(coarse, size=(H, W), mode="bicubic", align_corners=True) * 4.0).to(device).contiguous()
    out = torch.empty_like(x)
    nbytes = N * H * W * (8.0 * C + 8.0)

    def timed(fl):
        fn = lambda: ops.lib().vst_warp_fwd(x.data_ptr(), fl.data_ptr(), out.data_ptr(), N, H, W, C, 0,  # noqa: E731
                                            torch.cuda.current_stream().cuda_stream)
        ms = _time_on_stream(fn, reps)
        return ms, nbytes / (ms * 1e-3) / 1e9

    ms, gbs = timed(flow)
    del flow
    iid = torch.randn(N, 2, H, W, device=device) * 3.0
    ms_iid, gbs_iid = timed(iid)
    del x, out, iid
    return {"kernel": "warp_fwd_k (N=%d, C=%d, %dx%d)" % (N, C, H, W), "bound": "hbm",
            "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
            "avg_launch_ms": round(ms, 4), "bytes_per_launch": nbytes,
            "traffic": _pmc_traffic("warp", {"N": N, "C": C, "H": H, "W": W}),
            "flow": "SURVEY 8d smooth synthetic (bicubic 9x9 N(0,4^2) grid, x4)",
            "iid_flow_worst_case": {"flow": "i.i.d. N(0, 3^2) px per pixel", "achieved": round(gbs_iid, 1),
                                    "frac": round(gbs_iid / HBM_PEAK_GBS, 4), "avg_launch_ms": round(ms_iid, 4)}}


def corr_volume(device, B=1, D=256, H=55, W=128, reps=5):
    """RAFT CorrBlock build (utils/raft/raft/corr.py) at Sintel 440x1024 / 8: all-pairs GEMM on MFMA +
    3-level average-pool pyramid, then one 4-level radius-4 lookup."""
    from gbvst import raft_corr
    f1 = torch.randn(B, D, H, W, device=device)
    f2 = torch.randn(B, D, H, W, device=device)
    ys, xs = torch.meshgrid(torch.arange(H, device=device), torch.arange(W, device=device), indexing="ij")
    coords = torch.stack([xs, ys])[None].float().repeat(B, 1, 1, 1)
    holder = {}

    def build():
        holder["cb"] = raft_corr.CorrBlock(f1, f2, 4, 4)
    ms = _time_on_stream(build, reps)
    cb = holder["cb"]
    ms_lookup = _time_on_stream(lambda: cb.lookup_nhwc(coords), reps)
    flop = raft_corr.corr_flops(B, D, H, W)
    return {"config": "fmaps %dx%dx%dx%d, 4 levels, radius 4" % (B, D, H, W), "build_ms": round(ms, 4),
            "gemm_tflops_lower_bound": round(flop / (ms * 1e-3) / 1e12, 2), "lookup_ms": round(ms_lookup, 4),
            "note": "build = GEMM + pyramid + layout; TFLOP/s counts the GEMM's 2*(HW)^2*D over the whole build"}


def sintel_inference_fps(device, reps=5):
    """Generator-only inference at the Sintel frame size (1x3x436x1024)."""
    from gbvst import networks
    G = networks.define_G(3, 3, 64, "resnet_9blocks", "instance", False, "normal", 0.02, [device.index or 0])
    x = torch.randn(1, 3, 436, 1024, device=device)
    with torch.no_grad():
        ms = _time_on_stream(lambda: G(x), reps, warm=2)
    return {"metric": "generator-only inference fps 1024x436", "batch": 1, "value": round(1000.0 / ms, 2),
            "unit": "frames/s", "tflops": round(675.14 / ms, 2),
            "roofline": _mfma_roofline(675.14 / ms, "whole generator forward at 1x3x436x1024: 675.14 GFLOP/frame")}


def johnson_train_fps(device, B=4, S=256, steps=5):
    """Learning-based (Johnson) train step: FastStyleNet + VGG16 content/Gram-style/TV losses + Adam
    (fs_johnson.py), B frames of SxS, random-init weights (pretrained VGG is unavailable offline)."""
    from gbvst import faststyle, ops
    g = torch.Generator(device="cpu").manual_seed(7)
    J = faststyle.Johnson([torch.rand(1, 3, S, S, generator=g)], lr=1e-3, batch_sz=B, device=device)
    x = torch.rand(B, 3, S, S, generator=g).to(device)
    J.train_step(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        J.train_step(x)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    tf = _count_tflop(lambda: J.train_step(x))
    return {"metric": "Johnson fast-style train step frames/s %dx%d" % (S, S), "batch": B,
            "value": round(B / dt, 2), "unit": "frames/s", "ms_per_step": round(dt * 1e3, 3),
            "tflop_per_step": round(tf, 4),
            "roofline": _mfma_roofline(tf / dt, "FastStyleNet + VGG-16 conv / Gram FLOPs of one step "
                                               "(tools/convflops) over the step time")}


def _count_tflop(fn):
    """Algorithmic conv TFLOPs of one call of fn (tools/convflops.Counter: every gbvst.ops conv entry,
    real channel counts), run once untimed after the timed region."""
    from tools import convflops
    with convflops.Counter() as c:
        fn()
    torch.cuda.synchronize()
    return c.flops / 1e12


def stargan_train_fps(device, B=4, S=256, c_dim=4, cycles=2):
    """StarGAN C4: solver.py's training iteration at SxS, c_dim 4, n_critic 5, B_local
    images per rank; one timed cycle = 5 D iterations (each with the WGAN-GP double backward) + 1 G
    step.  Reported as per-D-iteration images/s (BASELINE.md's C4 line).  Random-init weights."""
    from gbvst import stargan
    g = torch.Generator(device="cpu").manual_seed(11)
    sol = stargan.StarGANSolver(image_size=S, c_dim=c_dim, n_critic=5, device=device)
    x = (torch.rand(B, 3, S, S, generator=g) * 2 - 1).to(device)
    lo = torch.randint(0, c_dim, (B,), generator=g)
    lt = torch.randint(0, c_dim, (B,), generator=g)
    for _ in range(10):
        sol.train_step(x, lo, lt)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5 * cycles):
        sol.train_step(x, lo, lt)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / (5 * cycles)

    def cycle():
        for _ in range(5):
            sol.train_step(x, lo, lt)
    tf = _count_tflop(cycle) / 5.0  # per D iteration (a cycle's G step shared over its 5)
    return {"metric": "StarGAN train images/s per D iteration %dx%d (n_critic 5)" % (S, S), "batch": B,
            "value": round(B / dt, 2), "unit": "images/s", "ms_per_d_iteration": round(dt * 1e3, 3),
            "tflop_per_d_iteration": round(tf, 4),
            "roofline": _mfma_roofline(tf / dt, "G/D conv FLOPs of one n_critic cycle (5 D iterations with the "
                                               "WGAN-GP double backward + 1 G step, counted per conv op by "
                                               "tools/convflops) / 5, over the D-iteration time")}


def raft_inference(device, B=1, H=436, W=1024, iters=20, reps=3):
    """RAFT (full model) flow for one frame pair as the Sintel TCL harness / MoGAN call it
    (InputPadder + test_mode, 20 iterations); random-init weights (raft-chairs.pth is unavailable)."""
    import argparse
    from gbvst import raft
    m = raft.RAFT(argparse.Namespace(small=False)).to(device).eval()
    g = torch.Generator(device="cpu").manual_seed(5)
    i1 = (torch.rand(B, 3, H, W, generator=g) * 255).to(device)
    i2 = (torch.rand(B, 3, H, W, generator=g) * 255).to(device)
    raft.compute_raft(m, i1, i2, it=iters)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        raft.compute_raft(m, i1, i2, it=iters)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    pads = raft.InputPadder((B, 3, H, W)).pads
    fl = raft.raft_flops(B, H + pads[2] + pads[3], W + pads[0] + pads[1], iters)
    return {"metric": "RAFT flow %dx%d, %d iterations" % (H, W, iters), "batch": B, "ms_per_call": round(dt * 1e3, 3),
            "pairs_per_s": round(B / dt, 2), "tflops": round(fl / dt / 1e12, 2),
            "roofline": _mfma_roofline(fl / dt / 1e12, "RAFT conv + correlation FLOPs (raft.raft_flops) over the "
                                                       "call time")}


def mogan_train_fps(device, B=4, S=256, pairs=2, H=None, W=None):
    """MoGAN C5-style step: CycleGAN ngf=ndf=64 generators / discriminators, motion nets,
    8 RAFT flows (20 iterations; one batched call) per optimize_parameters, E-step / M-step alternating; B frame pairs
    of SxS, random-init weights.  Reported per optimize_parameters call (E and M averaged)."""
    from gbvst import mogan_model
    from gbvst.options import default_opt
    opt = default_opt(True, model="mogan", pool_size=50, gpu_ids=[device.index or 0])
    m = mogan_model.MoGANModel(opt)
    g = torch.Generator(device="cpu").manual_seed(3)
    H, W = H or S, W or S
    imgs = [(torch.rand(B, 3, H, W, generator=g) * 2 - 1) for _ in range(4)]
    m.set_input_fc2(imgs)
    for _ in range(2):
        m.optimize_parameters()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(2 * pairs):
        m.optimize_parameters()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / (2 * pairs)

    def pair():
        m.optimize_parameters()
        m.optimize_parameters()
    tf = _count_tflop(pair) / 2.0  # per optimize_parameters (E and M averaged)
    return {"metric": "MoGAN optimize_parameters frames/s %dx%d (8 RAFT flows x 20 iterations per step)" % (W, H),
            "batch": B, "value": round(B / dt, 2), "unit": "frames/s", "ms_per_step": round(dt * 1e3, 3),
            "tflop_per_step": round(tf, 4),
            "roofline": _mfma_roofline(tf / dt, "conv FLOPs of one E + one M step (G/D/motion nets and the 8 RAFT "
                                               "flows' convs, tools/convflops) / 2, over the step time")}


VGG19_TO_RELU5_1 = [(3, 64), (64, 64), "pool", (64, 128), (128, 128), "pool", (128, 256), (256, 256), (256, 256),
                    (256, 256), "pool", (256, 512), (512, 512), (512, 512), (512, 512), "pool", (512, 512)]
VGG19_SLICE_ENDS = (0, 2, 4, 8, 12)   # conv index after which relu1_1 .. relu5_1 are taken


def vgg19_c3_flops(H, W):
    """Algorithmic FLOPs of the VGG-19 work in one C3 step (cycle_gan_vgg_model.extra_G_loss, network.py:45-78):
    3 forwards to relu5_1 (fake_B2 with grad, the real_A2 content target and the real_B style target),
    1 data-gradient pass (the frozen VGG's backward to fake_B2: every conv's dgrad, conv1_1's included),
    5 Grams each for fake_B2 and real_B (c^2 hw MACs, fast_style_transfer.py:813-817) and the Gram
    backward (c^2 hw).  3x3 convs: 9 Cin Cout MACs per output pixel."""
    h, w, conv, levels = H, W, 0.0, []
    for i, L in enumerate(VGG19_TO_RELU5_1):
        if L == "pool":
            h, w = h // 2, w // 2
            continue
        ci, co = L
        conv += 9.0 * ci * co * h * w
        n_conv = sum(1 for x in VGG19_TO_RELU5_1[:i + 1] if x != "pool") - 1
        if n_conv in VGG19_SLICE_ENDS:
            levels.append(co * co * h * w)
    gram = sum(levels)
    return {"conv_fwd_gflop": 2 * conv / 1e9, "total_tflop": (2 * conv * 4 + 2 * gram * 3) / 1e12}


def c3_train_fps(device, B=1, H=436, W=1024, steps=4):
    """Config C3: CycleGANCon step + VGG-19 content / Gram loss on fake_B2
    (gbvst.cycle_gan_vgg_model) on synthetic Sintel-size frame pairs 1x3x436x1024 (flow x4), random-init
    generator / discriminator weights, seeded VGG-19 (no pretrained weights offline); frames/s of
    optimize_parameters under the headline policy."""
    from gbvst import ops
    from gbvst.cycle_gan_vgg_model import CycleGANVGGModel
    from gbvst.options import default_opt
    m = CycleGANVGGModel(default_opt(True, model="cycle_gan_vgg", pool_size=50, gpu_ids=[device.index or 0]))
    a, a2, b, mask, flow = synthetic_batch(B, H, W, seed=4360, device=device)
    m.set_input_nhwc(ops.nchw_to_nhwc(a), ops.nchw_to_nhwc(a2), ops.nchw_to_nhwc(b), mask.contiguous(),
                     (flow * 4.0).contiguous())
    for _ in range(2):
        m.optimize_parameters()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        m.optimize_parameters()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    vgg = vgg19_c3_flops(H, W)
    return {"metric": "C3 train step frames/s %dx%d (CycleGANCon + flow-warp + VGG-19 content/Gram loss)" % (W, H),
            "batch": B, "value": round(B / dt, 3), "unit": "frames/s", "ms_per_step": round(dt * 1e3, 2),
            "tflops_conv_G_D": round(TRAIN_TFLOP_PER_FRAME_C3 / dt, 2),
            "roofline": _mfma_roofline((TRAIN_TFLOP_PER_FRAME_C3 + vgg["total_tflop"]) / dt,
                                       "G/D conv FLOPs (14.831 TFLOP/frame, SURVEY §8d) + the VGG-19 conv / Gram FLOPs "
                                       "(%.3f TFLOP/frame: 3 forwards to relu5_1, 1 data-gradient pass, 10 Grams + "
                                       "their backward) over the whole step time" % vgg["total_tflop"]),
            "loss_weights": {"lambda_content": m.opt.lambda_content, "lambda_style": m.opt.lambda_style},
            "losses": {k: round(v, 4) for k, v in m.get_current_losses().items()}}


def _g_inference_model(device):
    from gbvst import networks
    return networks.define_G(3, 3, 64, "resnet_9blocks", "instance", False, "normal", 0.02, [device.index or 0])


def _mfma_roofline(tflops, what):
    """Whole-workload MFMA roofline of an fp32-equivalent (bf16x6) conv path: algorithmic conv
    TFLOP/s vs the x6 ceiling (dense bf16 peak / 6 products per fp32 MAC)."""
    peak = BF16_MFMA_PEAK_TFLOPS / 6.0
    return {"bound": "mfma", "achieved": round(tflops, 2), "peak": round(peak, 1), "unit": "TFLOP/s",
            "frac": round(tflops / peak, 4), "what": what, "traffic": None}


def inference_fps(device, B=16, reps=10, G=None):
    """Generator-only inference (forward_eval, CycleGAN/models/cycle_gan_model.py:164-171) at 256x256:
    batch B throughput, plus B=1 per-frame with a device sync after every frame (the reference's DT
    metric, CycleGAN/sintel_eval.py:210-214, which itself has no sync)."""
    G = G or _g_inference_model(device)
    x = torch.randn(B, 3, 256, 256, device=device)
    x1 = x[:1].contiguous()
    with torch.no_grad():
        for _ in range(2):
            G(x)
            G(x1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            G(x)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        t1 = []
        for _ in range(3 * reps):
            a = time.perf_counter()
            G(x1)
            torch.cuda.synchronize()
            t1.append(time.perf_counter() - a)
    fps = B / dt
    dt1 = sorted(t1)[len(t1) // 2]
    tf = fps * G_GFLOP_PER_FRAME / 1e3
    return {"metric": "generator-only inference fps 256x256", "batch": B, "value": round(fps, 2),
            "unit": "frames/s", "tflops": round(tf, 2),
            "roofline": _mfma_roofline(tf, "whole generator forward, B=%d: 99.10 GFLOP/frame" % B),
            "batch1": {"value": round(1.0 / dt1, 2), "unit": "frames/s", "ms_per_frame": round(dt1 * 1e3, 3),
                       "timing": "median of %d single-frame calls, device sync after each" % (3 * reps),
                       "roofline": _mfma_roofline(G_GFLOP_PER_FRAME / dt1 / 1e3, "B=1 forward")}}


def inference_cpu_baseline(device, G=None):
    """§8(d) CPU leg of generator inference: oracle/cpu_ref.RefResnetGenerator (stock PyTorch NCHW
    fp32, the reference arithmetic) holding the GPU generator's weights, timed on the host cores at
    256x256 B=1 and B=16 and 436x1024 B=1; parity = max |GPU - CPU| of the same frames."""
    from oracle import cpu_ref
    threads = host_cpus()
    torch.set_num_threads(threads)
    G = G or _g_inference_model(device)
    R = cpu_ref.RefResnetGenerator(3, 3, 64, 9)
    R.load_state_dict({k: v.detach().cpu() for k, v in G.state_dict().items()})
    g = torch.Generator().manual_seed(77)
    out, err = {}, 0.0
    for name, (B, H, W, reps) in {"256x256_b1": (1, 256, 256, 3), "256x256_b16": (16, 256, 256, 1),
                                  "436x1024_b1": (1, 436, 1024, 1)}.items():
        x = torch.rand(B, 3, H, W, generator=g) * 2 - 1
        with torch.no_grad():
            y = R(x)                      # warm-up (and the parity frame)
            t0 = time.perf_counter()
            for _ in range(reps):
                R(x)
            dt = (time.perf_counter() - t0) / reps
            yg = G(x.to(device)).cpu()
        err = max(err, (yg - y).abs().max().item())
        out[name] = {"value": round(B / dt, 3), "unit": "frames/s", "s_per_call": round(dt, 3)}
    return {"kind": "port", "cores": threads, "sample": "oracle/cpu_ref.RefResnetGenerator forward, torch threads=%d "
            "(%s); 1 warm-up + timed calls per size" % (threads, cpu_model()), "sizes": out,
            "parity": {"what": "max |G_gpu(x) - G_cpu(x)| over the timed frames (outputs in [-1, 1])",
                       "max_abs": err, "bound": 1e-3, "pass": err <= 1e-3}}


def c1_faststyle(device, reps=10):
    """Config C1: the Johnson FastStyleNet (methods/learning-based/network.py:263-298) single 256x256
    frame forward — on the GPU (HIP) and, as the configuration itself is stated, on PyTorch-CPU (the
    oracle style_ref.RefFastStyleNet on the host cores), same counter-PRNG weights; parity of the
    stylised image."""
    from gbvst import faststyle
    from oracle import prng, style_ref
    threads = host_cpus()
    torch.set_num_threads(threads)
    ref = style_ref.RefFastStyleNet(3)
    sd = style_ref.fsn_weights(ref, 5100)
    style_ref.load_np(ref, sd)
    net = faststyle.FastStyleNet(3, 1)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    net = net.to(device)
    x = torch.from_numpy(prng.uniform_f32(5101, (1, 3, 256, 256)))
    xd = x.to(device)
    with torch.no_grad():
        for _ in range(3):
            net(xd)
        torch.cuda.synchronize()
        t = []
        for _ in range(reps):
            a = time.perf_counter()
            y = net(xd)[1]
            torch.cuda.synchronize()
            t.append(time.perf_counter() - a)
        yr = ref(x)[1]
        t0 = time.perf_counter()
        for _ in range(3):
            ref(x)
        dtc = (time.perf_counter() - t0) / 3
    dtg = sorted(t)[len(t) // 2]
    err = (y.cpu() - yr).abs().max().item() / (yr.abs().max().item())
    return {"metric": "C1: FastStyleNet 256x256 single-frame forward", "value": round(1.0 / dtg, 2), "unit": "frames/s",
            "ms_per_frame": round(dtg * 1e3, 3), "cpu_baseline": {"value": round(1.0 / dtc, 3), "unit": "frames/s",
                                                                  "cores": threads, "kind": "port",
                                                                  "sample": "oracle/style_ref.RefFastStyleNet, 3 timed "
                                                                            "forwards after 1 warm-up"},
            "parity": {"max_rel": err, "bound": 1e-3, "pass": err <= 1e-3}}


def host_cpus():
    """CPUs this process may run on: the affinity set, capped by a cgroup-v2 CPU quota if one is
    set (on a shared GPU box os.cpu_count() reports the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = max(1, min(n, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return n


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return ""


def cpu_baseline_and_parity(init_sd, batch_cpu, hip_losses0, steps=2):
    """cpu_baseline + parity leg (rank 0, N=1): the CPU oracle (oracle/cpu_ref.RefCycleGANCon —
    stock PyTorch, NCHW fp32, the reference's arithmetic) loaded with the SAME initial weights and
    fed the SAME synthetic batch as the GPU run.  Its first optimize_parameters() is the warm-up and
    the parity check: step-0 losses vs the GPU model's step-0 losses (max relative difference over
    the 9 loss terms; north_star bound 1e-3).  Then `steps` more B=4 steps are timed on all the host
    CPUs this process may use."""
    from oracle import cpu_ref
    threads = host_cpus()
    torch.set_num_threads(threads)
    m = cpu_ref.RefCycleGANCon(device="cpu")
    for name, net in m.nets().items():
        net.load_state_dict(init_sd[name])
    m.set_input_fc2(*batch_cpu)
    m.optimize_parameters()
    ref = m.get_current_losses()
    rel = {k: abs(hip_losses0[k] - v) / abs(v) for k, v in ref.items()}
    parity = {"what": "step-0 losses, GPU (HIP) vs CPU oracle, same weights and inputs", "max_rel": max(rel.values()),
              "worst": max(rel, key=rel.get), "bound": 1e-3, "pass": max(rel.values()) <= 1e-3}
    t0 = time.perf_counter()
    for _ in range(steps):
        m.optimize_parameters()
    dt = (time.perf_counter() - t0) / steps
    B, _, H, W = batch_cpu[0].shape
    base = {"value": round(B / dt, 4), "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"oracle/cpu_ref.RefCycleGANCon: {steps} timed train steps B={B} {H}x{W} fp32 after 1 "
                      f"warm-up/parity step ({dt:.1f} s/step; torch threads={threads} = the CPUs this process may "
                      f"use of os.cpu_count()={os.cpu_count()}; {cpu_model()})"}
    return base, parity


def time_steps(model, steps, hook_g, hook_d, world, device):
    return time_fn(lambda: model.optimize_parameters(hook_g, hook_d), steps, world, device)


def time_fn(step, steps, world, device):
    """Wall time of exactly `steps` calls of step(), barrier + device sync on both sides, max over
    ranks."""
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    return elapsed


# What each conv arithmetic policy computes in (gbvst.ops._POLICIES); the headline runs "bf16x6".
MATH_LABEL = {"bf16x6": "fp32 (bf16x6 split products: fp32-equivalent, fp32 accumulate) in every conv: fwd, dgrad, wgrad",
              "mixed": "mixed: bf16x6 (fp32-equivalent) training forwards / bf16x3 (~2^-16 rel. products) dgrad, wgrad, inference",
              "fp32": "fp32 (v_mfma_f32_32x32x2_f32) in every conv",
              "bf16x3": "bf16x3 split products (~2^-16 relative) in every conv"}


def _isolated(fn, *a, **kw):
    """Run one extra from a clean allocator state (its own warm-up is inside fn), so its value does
    not depend on which extras ran before it."""
    import gc
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    t0 = time.perf_counter()
    r = fn(*a, **kw)
    torch.cuda.synchronize()
    r["wall_s"] = round(time.perf_counter() - t0, 2)
    return r


def _line(metric, value, unit, world, args, ms, config, math):
    return {"metric": metric, "value": round(value, 3), "unit": unit, "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fp32" if math in ("bf16x6", "fp32") else math,
            "math": {"policy": math, "conv": MATH_LABEL[math]}, "data": "synthetic (random-init weights)",
            "config": config}


def workload_c4(args, world, rank, local, device):
    """Config C4: StarGAN (methods/GAN-based/StarGAN/solver.py:241-411) at 256x256, c_dim 4, n_critic 5,
    B_local images per rank, data parallel: every D iteration (with the WGAN-GP double backward) and
    every 5th G step exchange their gradients with RCCL all_reduce (dp.GradExchange on the solver's
    grad_hook).  value = images of all ranks per D iteration / s."""
    from gbvst import dp, stargan
    B = args.batch
    sol = stargan.StarGANSolver(image_size=args.size, c_dim=4, n_critic=5, device=device)
    if world > 1:
        dp.broadcast_params([sol.G, sol.D])
        sol.grad_hook = dp.GradExchange(world).attach([sol.G, sol.D])
    g = torch.Generator(device="cpu").manual_seed(11 + rank)
    x = (torch.rand(B, 3, args.size, args.size, generator=g) * 2 - 1).to(device)
    lo, lt = torch.randint(0, 4, (B,), generator=g), torch.randint(0, 4, (B,), generator=g)
    for _ in range(max(5, args.warmup)):
        sol.train_step(x, lo, lt)
    el = time_fn(lambda: sol.train_step(x, lo, lt), args.steps, world, device)
    cfg = {"workload": "C4: StarGAN solver iteration (D step + WGAN-GP every iteration, G step every 5th), "
                       "%dx%d, c_dim 4, conv_dim 64, 6+6 repeats, B_local=%d" % (args.size, args.size, B),
           "global_batch": B * world, "height": args.size, "width": args.size, "parallelism": "dp%d" % world,
           "dp_exchange": "RCCL all_reduce of the D (every iteration) and G (every 5th) flat gradients" if world > 1
           else None}
    return _line("images/sec: StarGAN train per D iteration (n_critic 5) 256x256", B * world * args.steps / el,
                 "images/s", world, args, el / args.steps * 1e3, cfg, args.math)


def workload_c5(args, world, rank, local, device):
    """Config C5: Mocycle-GAN (methods/GAN-based/MoGAN/models/cycle_gan_model.py:297-331) at 1024x436,
    B_local frame pairs per rank, 8 RAFT flows x 20 iterations per optimize_parameters, E-step / M-step
    alternating, data parallel with the G, D (E-step) and M (M-step) gradients exchanged with RCCL
    from inside backward (grad_hook_G / _D / _M).  value = frames of all ranks / s."""
    from gbvst import dp, mogan_model
    from gbvst.options import default_opt
    B, H, W = args.batch, 436, 1024
    m = mogan_model.MoGANModel(default_opt(True, model="mogan", pool_size=args.pool, gpu_ids=[local]))
    nets = [getattr(m, "net" + n) for n in ("G_A", "G_B", "D_A", "D_B", "M_A", "M_B")]
    ex = None
    if world > 1:
        dp.broadcast_params(nets)
        ex = dp.GradExchange(world).attach(nets)
    g = torch.Generator(device="cpu").manual_seed(3 + rank)
    m.set_input_fc2([(torch.rand(B, 3, H, W, generator=g) * 2 - 1) for _ in range(4)])
    for _ in range(max(2, args.warmup + args.warmup % 2)):   # even: the timed steps start at an E-step
        m.optimize_parameters(ex, ex, ex)
    el = time_fn(lambda: m.optimize_parameters(ex, ex, ex), args.steps, world, device)
    cfg = {"workload": "C5: MoGAN optimize_parameters (E/M alternating, 8 RAFT flows x 20 iterations), "
                       "ngf=ndf=64, %dx%d, B_local=%d, pool_size=%d" % (W, H, B, args.pool),
           "global_batch": B * world, "height": H, "width": W, "parallelism": "dp%d" % world,
           "dp_exchange": "RCCL all_reduce of G/D (E-step) and M (M-step) buckets launched during backward"
           if world > 1 else None}
    return _line("frames/sec: MoGAN train step (RAFT flow) 1024x436", B * world * args.steps / el, "frames/s", world,
                 args, el / args.steps * 1e3, cfg, args.math)


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n):
    """`bench.py --gpus N` run directly: N ranks as child processes of a torchrun on this node (the
    reference scales with nn.DataParallel over gpu_ids, CycleGAN/models/networks.py:111-116; here it is
    one process per GPU), each re-running this script with the same arguments.  The parent makes no
    GPU call; it returns the launcher's exit status."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % n,
           "--master-addr=127.0.0.1", "--master-port=%d" % free_port(), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # RCCL on this host: dmabuf IPC only
    return subprocess.call(cmd, env=env)


def workload_dpcheck(args, world, rank, local):
    """The launcher check: every rank joins the process group (gloo: no GPU is touched), all-reduces
    its rank + 1, and rank 0 prints the group's size and the sum."""
    if world > 1:
        dist.init_process_group("gloo")
        world = dist.get_world_size()
        assert world == args.gpus, (world, args.gpus)
    t = torch.tensor([rank + 1.0])
    if world > 1:
        dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"metric": "dpcheck", "n_gpus": world, "rank_sum": t.item(),
                          "expected": world * (world + 1) / 2}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=["c2", "c4", "c5", "dpcheck"], default="c2",
                    help="c2 (default, the BASELINE metric): CycleGANCon step; c4: StarGAN DP; c5: MoGAN DP; "
                         "dpcheck: the launcher's rank check alone (no GPU work)")
    ap.add_argument("--batch", type=int, default=None,
                    help="per-GPU batch (c2: 4 frame pairs, c4: 4 images, c5: 1 frame pair)")
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--pool", type=int, default=50)
    ap.add_argument("--math", default=os.environ.get("VST_CONV_MATH", "bf16x6"),
                    help="conv arithmetic policy of the headline (fp32-equivalent bf16x6 by default)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true")
    args = ap.parse_args()
    if args.batch is None:
        args.batch = {"c2": 4, "c4": 4, "c5": 1, "dpcheck": 1}[args.workload]

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # --gpus N without an outer launcher: start the N ranks here, one process per GPU, before
        # this process touches the GPU (it never does: it only waits for its children)
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but the launcher started WORLD_SIZE=%d ranks" % (args.gpus, world))
    if args.workload == "dpcheck":
        return workload_dpcheck(args, world, rank, local)
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        world = dist.get_world_size()           # n_gpus is the process group's size
        assert world == args.gpus, (world, args.gpus)
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    import gbvst
    gbvst._lib.load()
    from gbvst import dp, ops
    from gbvst.cycle_gan_model import CycleGANModel
    from gbvst.options import default_opt

    ops.set_conv_math(args.math)
    torch.manual_seed(0)
    if args.workload != "c2":
        out = {"c4": workload_c4, "c5": workload_c5}[args.workload](args, world, rank, local, device)
        if rank == 0:
            print(json.dumps(out), flush=True)
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    opt = default_opt(True, gpu_ids=[local], pool_size=args.pool)
    model = CycleGANModel(opt)
    nets = {"G_A": model.netG_A, "G_B": model.netG_B, "D_A": model.netD_A, "D_B": model.netD_B}
    hookG = hookD = None
    if world > 1:
        dp.broadcast_params(list(nets.values()))
        ex = dp.GradExchange(world).attach(list(nets.values()))
        hookG = hookD = ex
    init_sd = {k: {n: t.detach().cpu().clone() for n, t in v.state_dict().items()} for k, v in nets.items()}
    B, S = args.batch, args.size
    batch_cpu = synthetic_batch(B, S, S, seed=1234 + rank, device="cpu")
    a, a2, b, mask, flow = [t.to(device) for t in batch_cpu]
    model.set_input_nhwc(ops.nchw_to_nhwc(a), ops.nchw_to_nhwc(a2), ops.nchw_to_nhwc(b), mask.contiguous(),
                         flow.contiguous())

    losses0 = None
    for i in range(max(1, args.warmup)):
        model.optimize_parameters(hookG, hookD)
        if i == 0:
            losses0 = model.get_current_losses()  # step 0: what the parity leg checks
    # one launch in 13 of each probed op timed (36 per step each): HIP event pairs idle the stream between kernels
    probes = {k: ops.LaunchProbe(v, every=PROBE_EVERY) for k, v in DOMINANT_KEYS(B).items()}
    ops.set_launch_probes(list(probes.values()))
    elapsed = time_steps(model, args.steps, hookG, hookD, world, device)
    ops.set_launch_probes([])
    for p in probes.values():
        p.steps = args.steps
    losses = model.get_current_losses()

    frames = B * world * args.steps
    value = frames / elapsed
    out = {
        "metric": "frames/sec: CycleGAN train step (G+D+flow-warp loss) 256x256",
        "value": round(value, 3), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "fp32" if args.math in ("bf16x6", "fp32") else args.math,
        "math": {"policy": args.math, "conv": MATH_LABEL[args.math],
                 "elementwise_and_reductions": "fp32 / fp64 (IN statistics, losses, bias sums)"},
        "data": "synthetic (SURVEY §8d generator; random-init weights, init_type=normal 0.02)",
        "config": {"workload": "C2: CycleGANCon optimize_parameters, resnet_9blocks G + basic PatchGAN D, "
                               "ngf=ndf=64, %dx%d, B_local=%d, pool_size=%d, flow-warp temporal loss" % (S, S, B, args.pool),
                   "global_batch": B * world, "height": S, "width": S, "parallelism": "dp%d" % world,
                   "dp_exchange": "RCCL all_reduce of 8 MiB flat-gradient buckets launched during backward" if world > 1 else None},
        "algorithmic_tflops": round(value * TRAIN_TFLOP_PER_FRAME, 2),
        "step_roofline": _mfma_roofline(value / world * TRAIN_TFLOP_PER_FRAME,
                                        "whole train step per GPU: 2.1753 TFLOP/frame of conv work (SURVEY §8d)"),
        "final_losses": {k: round(v, 5) for k, v in losses.items()},
    }
    if rank == 0 and not args.no_extras:
        rl = {k: conv_roofline(k, p, args.math) for k, p in probes.items()}
        # the dominant kernel of the step is conv_fprop_bf_k<256x128> (its forward AND stride-1
        # data-gradient launches); its roofline line is the forward launch (one kernel, whole CU
        # rounds, no tail); the dgrad / wgrad ops (with their tail / copy / reduce launches) are in
        # roofline_convs
        out["roofline"] = rl["resblock_fprop"] or next(v for v in rl.values() if v)
        out["roofline_convs"] = rl
    if rank == 0 and world == 1 and not args.no_extras:
        G_inf = _g_inference_model(device)
        out["inference"] = _isolated(inference_fps, device, G=G_inf)
        # the same step under the round-1 "mixed" policy, separately labelled (not the headline)
        prev = ops.set_conv_math("mixed")
        model.optimize_parameters()
        el = time_steps(model, args.steps, None, None, 1, device)
        out["mixed_policy"] = {"value": round(B * args.steps / el, 3), "unit": "frames/s",
                               "ms_per_step": round(el / args.steps * 1e3, 3), "dtype": "mixed",
                               "math": MATH_LABEL["mixed"], "inference": _isolated(inference_fps, device, G=G_inf)}
        ops.set_conv_math(prev)
        out["extras"] = {"c3_train": _isolated(c3_train_fps, device),
                         "sintel_inference": _isolated(sintel_inference_fps, device),
                         "warp_roofline": _isolated(warp_roofline, device),
                         "raft_corr": _isolated(corr_volume, device),
                         "c1_faststyle": _isolated(c1_faststyle, device),
                         "johnson_train": _isolated(johnson_train_fps, device),
                         "stargan_train": _isolated(stargan_train_fps, device),
                         "raft_sintel": _isolated(raft_inference, device),
                         "raft_mogan": _isolated(raft_inference, device, B=4, H=256, W=256),
                         "mogan_train_c5": _isolated(mogan_train_fps, device, B=1, H=436, W=1024),
                         "mogan_train": _isolated(mogan_train_fps, device)}
        if not args.no_cpu_baseline:
            out["inference"]["cpu_baseline"] = inference_cpu_baseline(device, G=G_inf)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"], out["parity"] = cpu_baseline_and_parity(init_sd, batch_cpu, losses0)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
