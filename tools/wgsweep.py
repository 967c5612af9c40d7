"""Developer: time the channel-major weight-gradient kernel per wgrad tile kind (vst_debug_set_tiles)
on the train step's ResnetBlock shape (3x3 reflect 256->256 @64x64, bf16x3), N in {8, 12}."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import gbvst  # noqa: E402
from gbvst import ops  # noqa: E402

gbvst._lib.load()
dev = torch.device("cuda")
H, C = 64, 256
for N in (8, 12):
    x = torch.randn(N, H, H, C, device=dev)
    gy = torch.randn(N, H, H, C, device=dev)
    dw = torch.zeros(C, C, 3, 3, device=dev)
    for kind in (-1, 0, 1, 2, 4, 5, 6, -1):
        ops.debug_set_tiles(-1, -1, kind)
        def run():
            ops.conv2d_wgrad(x, gy, dw, None, 3, 3, 1, 1, "reflect", C, C, C * 9, 9, role="bwd")
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            run()
        e1.record()
        torch.cuda.synchronize()
        print("wgrad N=%d kind=%d %.1f us (incl. copies, slab sum, store)" % (N, kind, e0.elapsed_time(e1) * 50.0),
              flush=True)
ops.debug_set_tiles(-1, -1, -1)
