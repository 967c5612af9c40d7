"""Developer: the ResnetBlock stride-1 reflect data gradient at N = KB_B (default 8), 64x64x256,
both routes — padded frame + fold (VST_DGRAD_BORDER=0 path) and interior + border GEMM — with and
without the residual addend; HIP events per route (median of 5 x 20).  Run under rocprofv3
--kernel-trace --stats for the per-kernel split."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import gbvst  # noqa: E402
from gbvst import ops  # noqa: E402

gbvst._lib.load()
dev = torch.device("cuda")
B, H, C = int(os.environ.get("KB_B", "8")), 64, 256
w = torch.randn(C, C, 3, 3, device=dev) * 0.02
ikf = ops.weight_pack(w, ops.PACK_IKF)
gy = torch.randn(B, H, H, C, device=dev)
add = torch.randn(B, H, H, C, device=dev)
out = {"N": B}
for border in (False, True):
    ops.DGRAD_BORDER = border
    for a in (None, add):
        fn = lambda: ops.conv2d_dgrad_s1(gy, ikf, H, H, C, 3, 1, "reflect", addend=a)  # noqa: E731
        for _ in range(3):
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
        out["%s%s_us" % ("border" if border else "fold", "_add" if a is not None else "")] = round(sorted(ts)[2], 1)
print(json.dumps(out), flush=True)
