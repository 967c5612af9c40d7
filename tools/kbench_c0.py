"""Developer: the generator's first conv (4-channel image -> 64, 7x7 reflect 3) at N = KB_B frames of
256x256, with the InstanceNorm partials (ops.conv2d_fwd_in), KB_REPS launches — for rocprofv3 counter
passes over the 4-channel kernels (VST_C4_DIRECT=0: the implicit-GEMM route)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import gbvst  # noqa: E402
from gbvst import ops  # noqa: E402

gbvst._lib.load()
dev = torch.device("cuda")
B, reps = int(os.environ.get("KB_B", "8")), int(os.environ.get("KB_REPS", "20"))
x4 = torch.rand(B, 256, 256, 4, device=dev) * 2 - 1
x4[..., 3] = 0
w0 = torch.randn(64, 3, 7, 7, device=dev) * 0.05
k0 = ops.weight_pack(w0, ops.PACK_FWD)
b0 = torch.zeros(64, device=dev)
for _ in range(reps):
    ops.conv2d_fwd_in(x4, k0, b0, 64, 7, 7, 1, 3, "reflect")
torch.cuda.synchronize()
print("done", reps)
