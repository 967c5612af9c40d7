"""Developer timing probe (not a bench line): the C2 train step replayed from ONE captured HIP graph vs
the eager step, pool_size 0 and the Adam bias correction frozen at the capture step (timing only —
the numbers of the replayed steps are not checked here).  usage: stepgraph_probe.py [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
import gbvst  # noqa: E402
from gbvst import ops  # noqa: E402
from gbvst.cycle_gan_model import CycleGANModel  # noqa: E402
from gbvst.options import default_opt  # noqa: E402

gbvst._lib.load()
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda", 0)
m = CycleGANModel(default_opt(True, gpu_ids=[0], pool_size=0))
a, a2, b, mask, flow = bench.synthetic_batch(4, 256, 256, 1234, dev)
m.set_input_nhwc(ops.nchw_to_nhwc(a), ops.nchw_to_nhwc(a2), ops.nchw_to_nhwc(b), mask.contiguous(), flow.contiguous())
for _ in range(5):
    m.optimize_parameters()
torch.cuda.synchronize()


def timed(fn, n):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


eager = timed(m.optimize_parameters, steps)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    m.optimize_parameters()
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
t0 = time.perf_counter()
with torch.cuda.graph(g):
    m.optimize_parameters()
cap = time.perf_counter() - t0
graphed = timed(g.replay, steps)
eager2 = timed(m.optimize_parameters, steps)
print("eager %.3f ms/step, graphed %.3f ms/step, eager again %.3f ms/step (capture %.2f s)" % (eager, graphed, eager2, cap))
