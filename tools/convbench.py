"""Developer microbenchmark: time the conv kernel families on the CycleGAN layer shapes (B=4, 256^2)
for each GEMM tile choice (vst_debug_set_tiles), with HIP events on the launch stream."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import gbvst  # noqa: E402
from gbvst import ops  # noqa: E402

gbvst._lib.load()
dev = torch.device("cuda")
B = int(os.environ.get("B", "4"))
# name -> (fprop/tconv rk kind, wgrad TileKind)
TILES = {"auto": (-1, -1), "k0": (0, 0), "k1": (1, 1), "k2": (2, 2), "k3": (3, 3),
         "k4": (4, 4), "legacy": (-1, 8), "k5": (5, 5), "k6": (6, 6)}
if os.environ.get("TILES"):
    TILES = {k: v for k, v in TILES.items() if k in os.environ["TILES"].split(",")}
ONLY = os.environ.get("LAYERS")


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


# (name, Cin, H, Cout, k, stride, pad, mode)
LAYERS = [
    ("res", 256, 64, 256, 3, 1, 1, "reflect"),
    ("d128", 64, 256, 128, 3, 2, 1, "zero"),
    ("d256", 128, 128, 256, 3, 2, 1, "zero"),
    ("c7s1_64", 4, 256, 64, 7, 1, 3, "reflect"),
    ("D2", 64, 128, 128, 4, 2, 1, "zero"),
    ("D4", 256, 32, 512, 4, 1, 1, "zero"),
]
res = []
_w = torch.randn(4096, 4096, device=dev)
for _ in range(50):
    _w @ _w  # clock ramp
for name, Ci, H, Co, k, st, pad, mode in LAYERS:
    if ONLY and name not in ONLY.split(","):
        continue
    x = torch.randn(B, H, H, Ci, device=dev)
    w = torch.randn(Co, Ci, k, k, device=dev) * 0.02
    kc, ck = ops.weight_pack(w, ops.PACK_FWD), ops.weight_pack(w, ops.PACK_DGRAD)
    ikf = ops.weight_pack(w, ops.PACK_IKF)
    Ho = (H + 2 * pad - k) // st + 1
    gy = torch.randn(B, Ho, Ho, Co, device=dev)
    dw = torch.zeros(Co, Ci, k, k, device=dev)
    flop = 2.0 * B * Ho * Ho * Co * Ci * k * k
    for tname, tv in TILES.items():
        ops.debug_set_tiles(tv[0], tv[0], tv[1])
        try:
            tf = timeit(lambda: ops.conv2d_fwd(x, kc, None, Co, k, k, st, pad, mode))
            tt = timeit(lambda: ops.conv2d_tfwd(gy, ck, None, H, H, Ci, k, k, st, pad, pad_mode=mode))
            tw = timeit(lambda: ops.conv2d_wgrad(x, gy, dw, None, k, k, st, pad, mode, Co, Ci, Ci * k * k, k * k))
            td = timeit(lambda: ops.conv2d_dgrad_s1(gy, ikf, H, H, Ci, k, pad, mode)) if st == 1 and Co % 8 == 0 else float("nan")
        except Exception as e:  # noqa
            print(name, tname, "ERR", e)
            continue
        r = {"layer": name, "tile": tname, "fprop_us": round(tf, 1), "tconv_us": round(tt, 1),
             "wgrad_us": round(tw, 1), "fprop_TF": round(flop / tf / 1e6, 1),
             "tconv_TF": round(flop / tt / 1e6, 1), "wgrad_TF": round(flop / tw / 1e6, 1),
             "dgrad_fprop_us": round(td, 1)}
        res.append(r)
        print(json.dumps(r), flush=True)
ops.debug_set_tiles(-1, -1, -1)
