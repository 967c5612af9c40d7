"""Developer A/B timing of the ResnetBlock conv kernels (N = KB_B frames, 64x64x256, 3x3 reflect)
under the current VST_CONV_MATH policy: fprop, dgrad (stride-1 data gradient as a forward conv over
the padded frame + fold), wgrad; HIP events on the launch stream, median of 5 x 20 launches.
Run with VST_LIB_VARIANT=<variant .so> to compare builds (tools/build_variant.py)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import gbvst  # noqa: E402
from gbvst import ops  # noqa: E402

gbvst._lib.load()
if os.environ.get("KB_TILE"):  # force the forward / dgrad tile kind (vst_debug_set_tiles)
    ops.debug_set_tiles(int(os.environ["KB_TILE"]), -1, -1)
dev = torch.device("cuda")
out = {"lib": os.environ.get("VST_LIB_VARIANT", "default"), "math": ops.get_conv_math(),
       "tile": os.environ.get("KB_TILE", "auto")}
for B in [int(b) for b in os.environ.get("KB_B", "8,12").split(",")]:
    H, C = 64, 256
    x = torch.randn(B, H, H, C, device=dev)
    if os.environ.get("KB_RELU") == "1":  # half-zero activations, as the step's (the clock depends on the data)
        x = torch.relu(x)
    w = torch.randn(C, C, 3, 3, device=dev) * 0.02
    kc, ikf = ops.weight_pack(w, ops.PACK_FWD), ops.weight_pack(w, ops.PACK_IKF)
    gy = torch.randn(B, H, H, C, device=dev)
    dw = torch.zeros(C, C, 3, 3, device=dev)
    flop = 2.0 * B * H * H * C * C * 9
    fns = {"fprop": lambda: ops.conv2d_fwd(x, kc, None, C, 3, 3, 1, 1, "reflect"),
           "dgrad": lambda: ops.conv2d_fwd(gy, ikf, None, C, 3, 3, 1, 2, "zero", role="bwd"),
           "wgrad": lambda: ops.conv2d_wgrad(x, gy, dw, None, 3, 3, 1, 1, "reflect", C, C, C * 9, 9)}
    for name, fn in fns.items():
        for _ in range(5):
            fn()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) / 20 * 1e3)
        us = sorted(ts)[2]
        out["%s_N%d_us" % (name, B)] = round(us, 1)
        out["%s_N%d_TF" % (name, B)] = round(flop / us / 1e6, 1)
if os.environ.get("KB_EXTRA", "1") != "0":
    # the image-side 7x7 forward (generator c0: 3(+1) -> 64 channels, reflect 3) at N=8, 256x256, and
    # the warp kernel at bench.py's roofline shape
    def _t(fn, reps=10):
        for _ in range(3):
            fn()
        ts = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) / reps * 1e3)
        return round(sorted(ts)[1], 1)
    x4 = torch.randn(8, 256, 256, 4, device=dev)
    x4[..., 3] = 0
    w0 = torch.randn(64, 3, 7, 7, device=dev) * 0.05
    k0 = ops.weight_pack(w0, ops.PACK_FWD)
    b0 = torch.zeros(64, device=dev)
    out["c0fwd_N8_us"] = _t(lambda: ops.conv2d_fwd_in(x4, k0, b0, 64, 7, 7, 1, 3, "reflect"))
    xw = torch.randn(32, 436, 1024, 64, device=dev)
    fl = torch.randn(32, 2, 436, 1024, device=dev) * 3.0
    ow = torch.empty_like(xw)
    us = _t(lambda: ops.lib().vst_warp_fwd(xw.data_ptr(), fl.data_ptr(), ow.data_ptr(), 32, 436, 1024, 64, 0,
                                            torch.cuda.current_stream().cuda_stream), reps=5)
    out["warp_us"] = us
    out["warp_TBs"] = round(32 * 436 * 1024 * (8.0 * 64 + 8.0) / us / 1e6, 3)
    del xw, fl, ow
print(json.dumps(out), flush=True)
