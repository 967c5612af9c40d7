"""Per-layer roofline table of the C2 train step's conv ops: every conv-family
entry of gbvst.ops called during one optimize_parameters() (after warm-up) is wrapped with HIP events
on the current stream (outermost call only), keyed by (op, shapes); algorithmic FLOPs use the
reference's real channel counts (3-channel images, 1-channel PatchGAN head), so a frac counts padding
as waste.  usage: layertable.py [steps] -> JSON lines {op, layer, n, us, tflops, frac} + aggregates."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
import gbvst  # noqa: E402
from gbvst import ops  # noqa: E402
from gbvst.cycle_gan_model import CycleGANModel  # noqa: E402
from gbvst.options import default_opt  # noqa: E402

PEAK = bench.BF16_MFMA_PEAK_TFLOPS / 6.0


def real(c):
    return 3 if c == 4 else c


def fl_fwd(a, k):
    x, cop, R, S, st, pad = a[0], a[3], a[4], a[5], a[6], a[7]
    N, H, W, C = x.shape
    Ho, Wo = (H + 2 * pad - R) // st + 1, (W + 2 * pad - S) // st + 1
    co = k.get("co_real") or real(cop)
    return 2.0 * N * Ho * Wo * real(C) * co * R * S, "conv%dx%d s%d %d->%d @%dx%d N=%d" % (R, S, st, real(C), co, H, W, N)


def fl_wgrad(a, k):
    x, dy, R, S, st, co, ci = a[0], a[1], a[4], a[5], a[6], a[9], a[10]
    N, Ho, Wo, _ = dy.shape
    return 2.0 * N * Ho * Wo * co * ci * R * S, "wgrad %dx%d s%d %d->%d out %dx%d N=%d" % (R, S, st, ci, co, Ho, Wo, N)


def fl_dgrad_s1(a, k):
    dy, H, W, cx, R = a[0], a[2], a[3], a[4], a[5]
    N, _, _, C = dy.shape
    return 2.0 * N * H * W * real(C) * real(cx) * R * R, "dgrad%dx%d s1 %d->%d @%dx%d N=%d" % (R, R, real(C), real(cx), H, W, N)


def fl_convT(a, k):
    x, cop = a[0], a[3]
    N, H, W, C = x.shape
    return 2.0 * N * H * W * C * real(cop) * 9, "convT/s2-dgrad 3x3 %d->%d in %dx%d N=%d" % (C, real(cop), H, W, N)


def fl_c4s2(a, k):
    dy, cop = a[0], a[2]
    N, H, W, C = dy.shape
    return 2.0 * N * H * W * C * real(cop) * 16, "dgrad 4x4 s2 %d->%d in %dx%d N=%d" % (C, real(cop), H, W, N)


def fl_tap(a, k):
    x, R = a[0], a[3] if len(a) > 3 else a[2]
    N, H, W, C = x.shape
    return 2.0 * N * H * W * 64 * 3 * 49, "7x7 64<->3 tap route @%dx%d N=%d" % (H, W, N)


def fl_tfwd(a, k):
    dy, Ho, Wo, cx, R, S, st = a[0], a[3], a[4], a[5], a[6], a[7], a[8]
    N, Hi, Wi, Cy = dy.shape
    cy = 1 if Cy == 4 and cx == 512 else real(Cy)  # the PatchGAN head's data gradient: 1 real channel
    return 2.0 * N * Hi * Wi * cy * real(cx) * R * S, "tdgrad %dx%d s%d %d->%d out %dx%d N=%d" % (R, S, st, cy, real(cx), Ho, Wo, N)


OPS = {"conv2d_fwd": fl_fwd, "conv2d_tfwd": fl_tfwd, "conv2d_fwd_in": fl_fwd, "conv2d_wgrad": fl_wgrad, "conv2d_dgrad_s1": fl_dgrad_s1,
       "convT3s2_fwd": fl_convT, "conv4s2_dgrad": fl_c4s2, "tap_conv_fwd_h": fl_tap, "tap_conv_dgrad_h": fl_tap,
       "tap_conv_wgrad_h": fl_tap, "tap_conv_wgrad_swap": fl_tap, "c4_dgrad_reflect": fl_tap}
rec, depth = {}, [0]


def wrap(name, fn, flops):
    def w(*a, **k):
        if depth[0] or not rec.get("_on"):
            depth[0] += 1
            try:
                return fn(*a, **k)
            finally:
                depth[0] -= 1
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        depth[0] += 1
        try:
            out = fn(*a, **k)
        finally:
            depth[0] -= 1
        e1.record()
        f, lab = flops(a, k)
        rec.setdefault((name, lab), []).append((e0, e1, f))
        return out
    return w


for name, f in OPS.items():
    setattr(ops, name, wrap(name, getattr(ops, name), f))

gbvst._lib.load()
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
dev = torch.device("cuda", 0)
m = CycleGANModel(default_opt(True, gpu_ids=[0], pool_size=50))
a, a2, b, mask, flow = bench.synthetic_batch(4, 256, 256, 1234, dev)
m.set_input_nhwc(ops.nchw_to_nhwc(a), ops.nchw_to_nhwc(a2), ops.nchw_to_nhwc(b), mask.contiguous(), flow.contiguous())
for _ in range(4):
    m.optimize_parameters()
torch.cuda.synchronize()
rec["_on"] = True
for _ in range(steps):
    m.optimize_parameters()
torch.cuda.synchronize()
rec.pop("_on")
rows, tot_ms, tot_f, res_ms, res_f = [], 0.0, 0.0, 0.0, 0.0
for (name, lab), evs in rec.items():
    ms = sum(e0.elapsed_time(e1) for e0, e1, _ in evs)
    f = sum(x for _, _, x in evs)
    resblock = "256->256" in lab and "@64x64" in lab or ("256->256" in lab and "out 64x64" in lab)
    rows.append({"op": name, "layer": lab, "calls_per_step": len(evs) / steps, "ms_per_step": round(ms / steps, 3),
                 "us_per_call": round(ms / len(evs) * 1e3, 1), "tflops": round(f / (ms * 1e-3) / 1e12, 1),
                 "frac": round(f / (ms * 1e-3) / 1e12 / PEAK, 3), "resblock": bool(resblock)})
    if resblock:
        res_ms, res_f = res_ms + ms, res_f + f
    else:
        tot_ms, tot_f = tot_ms + ms, tot_f + f
rows.sort(key=lambda r: -r["ms_per_step"])
for r in rows:
    print(json.dumps(r))
print(json.dumps({"aggregate_non_resblock": {"ms_per_step": round(tot_ms / steps, 2), "tflop_per_step": round(tot_f / steps / 1e12, 3),
                                             "frac": round(tot_f / (tot_ms * 1e-3) / 1e12 / PEAK, 3)},
                  "aggregate_resblock": {"ms_per_step": round(res_ms / steps, 2), "tflop_per_step": round(res_f / steps / 1e12, 3),
                                         "frac": round(res_f / (res_ms * 1e-3) / 1e12 / PEAK, 3)}}))
