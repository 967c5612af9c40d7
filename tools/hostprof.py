"""Host-side profile of the C2 train step (bench.py's model and batch): how long the host takes to enqueue one
optimize_parameters() (the stream drained first, no sync inside), against the step's GPU time, plus a cProfile of
the enqueue (sorted by own time).  Where the host enqueue of a phase takes longer than its kernels run, the stream
idles between launches (the >20 us gaps of the kernel trace).  usage: hostprof.py [steps]"""
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda:0")
    import gbvst
    gbvst._lib.load()
    from gbvst import ops
    from gbvst.cycle_gan_model import CycleGANModel
    from gbvst.options import default_opt
    ops.set_conv_math("bf16x6")
    torch.manual_seed(0)
    model = CycleGANModel(default_opt(True, gpu_ids=[0], pool_size=50))
    a, a2, b, mask, flow = [t.to(dev) for t in bench.synthetic_batch(4, 256, 256, seed=1234, device="cpu")]
    model.set_input_nhwc(ops.nchw_to_nhwc(a), ops.nchw_to_nhwc(a2), ops.nchw_to_nhwc(b), mask.contiguous(),
                         flow.contiguous())
    for _ in range(4):
        model.optimize_parameters()
    torch.cuda.synchronize()
    enq, tot = [], []
    for _ in range(steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        model.optimize_parameters()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        enq.append((t1 - t0) * 1e3)
        tot.append((t2 - t0) * 1e3)
    print("host enqueue ms/step: %s" % " ".join("%.2f" % v for v in enq))
    print("enqueue+drain ms/step: %s" % " ".join("%.2f" % v for v in tot))
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(steps):
        model.optimize_parameters()
    pr.disable()
    torch.cuda.synchronize()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(35)
    print(s.getvalue())
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(45)
    print(s.getvalue())
