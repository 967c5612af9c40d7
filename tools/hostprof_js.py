"""Host-side profile of the Johnson fast-style train step (bench.johnson_train_fps's workload, B=4 256x256): host
enqueue time vs enqueue + drain per step, and a cProfile of the enqueue sorted by own time.  usage: hostprof_js.py"""
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

if __name__ == "__main__":
    from gbvst import _lib, faststyle, ops
    _lib.load()
    ops.set_conv_math("bf16x6")
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(7)
    J = faststyle.Johnson([torch.rand(1, 3, 256, 256, generator=g)], lr=1e-3, batch_sz=4, device=dev)
    x = torch.rand(4, 3, 256, 256, generator=g).to(dev)
    for _ in range(5):
        J.train_step(x)
    torch.cuda.synchronize()
    enq, tot = [], []
    for _ in range(10):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        J.train_step(x)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        enq.append((t1 - t0) * 1e3)
        tot.append((time.perf_counter() - t0) * 1e3)
    print("host enqueue ms/step: %s" % " ".join("%.2f" % v for v in enq))
    print("enqueue+drain ms/step: %s" % " ".join("%.2f" % v for v in tot))
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(10):
        J.train_step(x)
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
    print(s.getvalue())
