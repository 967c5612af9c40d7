"""Developer: launch one conv family on the ResnetBlock shape (B=4, 64x64x256, 3x3 reflect) a few
times (batch KB_B, default 8) — the target of rocprofv3 --pmc passes.  usage: kbench.py fprop|dgrad|tconv|wgrad|warp [reps]
warp: vst_warp_fwd on bench.py's warp_roofline shape (N=32, C=64, 436x1024, random flow)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import gbvst  # noqa: E402
from gbvst import ops  # noqa: E402

gbvst._lib.load()
which = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
dev = torch.device("cuda")
if which == "warp":
    N, C, H, W = 32, 64, 436, 1024
    xw = torch.randn(N, H, W, C, device=dev)
    flow = torch.randn(N, 2, H, W, device=dev) * 3.0
    out = torch.empty_like(xw)
    for _ in range(reps):
        ops.lib().vst_warp_fwd(xw.data_ptr(), flow.data_ptr(), out.data_ptr(), N, H, W, C, 0,
                               torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    sys.exit(0)
B, H, C = int(os.environ.get("KB_B", "8")), 64, 256  # 8 = the batched G_A calls of the train step
x = torch.randn(B, H, H, C, device=dev)
w = torch.randn(C, C, 3, 3, device=dev) * 0.02
kc, ck = ops.weight_pack(w, ops.PACK_FWD), ops.weight_pack(w, ops.PACK_DGRAD)
ikf = ops.weight_pack(w, ops.PACK_IKF)
gy = torch.randn(B, H, H, C, device=dev)
dw = torch.zeros(C, C, 3, 3, device=dev)
for _ in range(reps):
    if which == "fprop":
        ops.conv2d_fwd(x, kc, None, C, 3, 3, 1, 1, "reflect")
    elif which == "dgrad":  # stride-1 data gradient as a forward conv over rotated taps (train path)
        ops.conv2d_dgrad_s1(gy, ikf, H, H, C, 3, 1, "reflect")
    elif which == "tconv":
        ops.conv2d_tfwd(gy, ck, None, H, H, C, 3, 3, 1, 1, pad_mode="reflect")
    else:
        ops.conv2d_wgrad(x, gy, dw, None, 3, 3, 1, 1, "reflect", C, C, C * 9, 9)
torch.cuda.synchronize()
