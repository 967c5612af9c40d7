"""Developer: generator-only inference (forward_eval: no_grad G_A, CycleGAN/models/cycle_gan_model.py:164-171)
at one size, `reps` calls after 3 warm-ups — the target of rocprofv3 --kernel-trace for the inference
trace.  usage: infbench.py B H W [reps] [eager|graph]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import gbvst  # noqa: E402
from gbvst import networks  # noqa: E402

gbvst._lib.load()
B, H, W = (int(a) for a in sys.argv[1:4])
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 10
dev = torch.device("cuda")
G = networks.define_G(3, 3, 64, "resnet_9blocks", "instance", False, "normal", 0.02, [0])
x = torch.rand(B, 3, H, W, device=dev) * 2 - 1
with torch.no_grad():
    for _ in range(3):
        G(x)
    torch.cuda.synchronize()
    t = []
    for _ in range(reps):
        a = time.perf_counter()
        G(x)
        torch.cuda.synchronize()
        t.append(time.perf_counter() - a)
t.sort()
print("B=%d %dx%d: median %.3f ms/call, %.1f frames/s" % (B, H, W, t[len(t) // 2] * 1e3, B / t[len(t) // 2]))
