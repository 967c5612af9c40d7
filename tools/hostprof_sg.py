"""Host-side profile of the StarGAN C4 D iteration (bench.stargan_train_fps's workload): the host time to enqueue one
solver train_step from a drained stream against its GPU time, and a cProfile of the enqueue sorted by own time —
where the host is the bound (the D iteration's many small launches), its Python overhead is the step time.
usage: hostprof_sg.py [iterations]"""
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

if __name__ == "__main__":
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda:0")
    from gbvst import _lib, ops, stargan
    _lib.load()
    ops.set_conv_math("bf16x6")
    g = torch.Generator(device="cpu").manual_seed(11)
    B, S, c_dim = 4, 256, 4
    sol = stargan.StarGANSolver(image_size=S, c_dim=c_dim, n_critic=5, device=dev)
    x = (torch.rand(B, 3, S, S, generator=g) * 2 - 1).to(dev)
    lo = torch.randint(0, c_dim, (B,), generator=g)
    lt = torch.randint(0, c_dim, (B,), generator=g)
    for _ in range(10):
        sol.train_step(x, lo, lt)
    torch.cuda.synchronize()
    enq, tot = [], []
    for _ in range(iters):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sol.train_step(x, lo, lt)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        enq.append((t1 - t0) * 1e3)
        tot.append((t2 - t0) * 1e3)
    print("host enqueue ms/iter: %s" % " ".join("%.2f" % v for v in enq))
    print("enqueue+drain ms/iter: %s" % " ".join("%.2f" % v for v in tot))
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(iters):
        sol.train_step(x, lo, lt)
    torch.cuda.synchronize()
    pr.disable()
    for key in ("tottime", "cumulative"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(40)
        print(s.getvalue())
