"""Developer: launch the direct 64 -> 4 7x7 tap kernel (vst_tapconv_h_fwd, conv_tap64.hip) at the train
step's shape (N=KB_B, 256x256): reflect pad 3 + tanh (the last layer's forward) or zero pad 6 (the first
layer's data-gradient form, KB_MODE=dgrad) — the target of rocprofv3 --pmc / --kernel-trace passes.
usage: kbench_tap64.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import gbvst  # noqa: E402
from gbvst import ops  # noqa: E402

gbvst._lib.load()
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
B, dev = int(os.environ.get("KB_B", "8")), torch.device("cuda")
x = torch.randn(B, 256, 256, 64, device=dev)
w = torch.randn(3, 64, 7, 7, device=dev) * 0.02
sok = ops.weight_pack(w, ops.PACK_SOK, Op=4)
bp = torch.zeros(4, device=dev)
dgrad = os.environ.get("KB_MODE", "fwd") == "dgrad"
for _ in range(3):
    ops.tap_conv_fwd_h(x, sok, None if dgrad else bp, 7, 6 if dgrad else 3, "zero" if dgrad else "reflect",
                       act="none" if dgrad else "tanh")
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    ops.tap_conv_fwd_h(x, sok, None if dgrad else bp, 7, 6 if dgrad else 3, "zero" if dgrad else "reflect",
                       act="none" if dgrad else "tanh")
e1.record()
torch.cuda.synchronize()
print("tap64 %s N=%d: %.1f us/call" % ("dgrad" if dgrad else "fwd", B, e0.elapsed_time(e1) / reps * 1e3))
