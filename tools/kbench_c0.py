"""Developer: the generator's first conv (4-channel image -> 64, 7x7 reflect 3) at N = KB_B frames of
256x256, KB_REPS launches, HIP-event timed (us/call printed) — KB_MODE=in (default: with the
InstanceNorm partials, ops.conv2d_fwd_in, as the train step runs it) or plain (ops.conv2d_fwd).  Also
the rocprofv3 counter-pass target (tools/pmc_c0.sh); VST_C4_DIRECT=0: the implicit-GEMM route."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import gbvst  # noqa: E402
from gbvst import ops  # noqa: E402

gbvst._lib.load()
dev = torch.device("cuda")
B, reps = int(os.environ.get("KB_B", "8")), int(os.environ.get("KB_REPS", "20"))
mode = os.environ.get("KB_MODE", "in")
x4 = torch.rand(B, 256, 256, 4, device=dev) * 2 - 1
x4[..., 3] = 0
w0 = torch.randn(64, 3, 7, 7, device=dev) * 0.05
k0 = ops.weight_pack(w0, ops.PACK_FWD)
b0 = torch.zeros(64, device=dev)


def run():
    if mode == "in":
        ops.conv2d_fwd_in(x4, k0, b0, 64, 7, 7, 1, 3, "reflect")
    else:
        ops.conv2d_fwd(x4, k0, b0, 64, 7, 7, 1, 3, "reflect")


for _ in range(3):
    run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    run()
e1.record()
torch.cuda.synchronize()
print("c0 %s N=%d: %.1f us/call (incl. IN finalize for mode in)" % (mode, B, e0.elapsed_time(e1) * 1e3 / reps))
