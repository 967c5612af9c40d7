"""Developer: time the split-bf16 forward kernel per tile kind on the train step's ResnetBlock
shapes (fprop x6 and the stride-1 reflect dgrad-as-fprop x3 over the padded frame), N in {8, 12}.
usage: tilesweep.py  -> one line per (op, N, kind): avg us over 10 launches (HIP events)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import gbvst  # noqa: E402
from gbvst import ops  # noqa: E402

gbvst._lib.load()
dev = torch.device("cuda")
H, C = 64, 256
w = torch.randn(C, C, 3, 3, device=dev) * 0.02
kc, ikf = ops.weight_pack(w, ops.PACK_FWD), ops.weight_pack(w, ops.PACK_IKF)
for N in (8, 12):
    x = torch.randn(N, H, H, C, device=dev)
    for op in ("fprop", "dgrad"):
        for kind in [-1] + list(range(8)) * (os.environ.get("ALL", "0") == "1"):
            ops.debug_set_tiles(kind, -1, -1)
            def run():
                if op == "fprop":
                    ops.conv2d_fwd(x, kc, None, C, 3, 3, 1, 1, "reflect", role="fwd")
                else:
                    ops.conv2d_fwd(x, ikf, None, C, 3, 3, 1, 2, "zero", role="bwd")
            run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                run()
            e1.record()
            torch.cuda.synchronize()
            print("%s N=%d kind=%d %.1f us" % (op, N, kind, e0.elapsed_time(e1) * 100.0), flush=True)
ops.debug_set_tiles(-1, -1, -1)
