"""Developer: the generator's last-layer weight gradient (64 -> 3, 7x7 reflect 3, N = KB_B frames of
256x256) two ways, checked against torch fp64 and HIP-event timed (us/call printed):
  h:    ops.tap_conv_wgrad_h (the 7x1 conv's gradient: dy column-shifted into 28 channels, M = 448)
  swap: ops.tap_conv_wgrad_swap — the 7x7 wgrad of the zero-padded 4-channel dy (M = 196 (tap, co))
        against the reflect-padded x as 64 "output" channels over the 262 x 264 frame.
Run under rocprofv3 --kernel-trace --stats for the per-kernel split."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import gbvst  # noqa: E402
from gbvst import ops  # noqa: E402

gbvst._lib.load()
ops.set_conv_math("bf16x6")
dev = torch.device("cuda")
B, reps = int(os.environ.get("KB_B", "8")), int(os.environ.get("KB_REPS", "20"))
g = torch.Generator().manual_seed(5)
x = torch.randn(B, 64, 256, 256, generator=g)
gy = torch.randn(B, 3, 256, 256, generator=g)
ref = torch.nn.grad.conv2d_weight(F.pad(x.double(), (3,) * 4, mode="reflect"), (3, 64, 7, 7), gy.double())
xn = x.permute(0, 2, 3, 1).contiguous().to(dev)
dy4 = torch.zeros(B, 256, 256, 4, device=dev)
dy4[..., :3] = gy.permute(0, 2, 3, 1).to(dev)


def run_h(dw):
    ops.tap_conv_wgrad_h(xn, dy4, dw, 7, 3, "reflect", accumulate=False)


st = torch.zeros((B, 64, 2), device=dev)
st[..., 1] = 1.0
_, xpl = ops.instnorm_act_fwd(xn, st, "none", xpl=(3, "reflect", ops.tap_swap_geom(256, 7)[0]))


def run_swap(dw):  # the x planes made by the IN apply beforehand, as in the train step
    ops.tap_conv_wgrad_swap(xn, dy4, dw, 7, 3, "reflect", accumulate=False, x_pl=xpl)


for name, fn in (("h", run_h), ("swap", run_swap)):
    dw = torch.zeros(3, 64, 7, 7, device=dev)
    fn(dw)
    torch.cuda.synchronize()
    err = ((dw.cpu().double() - ref).norm() / ref.norm()).item()
    for _ in range(2):
        fn(dw)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn(dw)
    e1.record()
    torch.cuda.synchronize()
    print("%s rel_err %.3e  %.1f us/call (incl. glue)" % (name, err, 1000 * e0.elapsed_time(e1) / reps), flush=True)
print("plan swap", ops.conv_plan_wgrad(B, 256, 258, 4, 262, 264, 64, 7, 7, 1, "bf16x6"), flush=True)
time.sleep(0.1)
