"""Does batching generator passes help?  Time G forward+backward at B=4 (x2) vs B=8 (x1)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from gbvst import _lib, networks, ops  # noqa: E402

_lib.load()
dev = torch.device("cuda:0")
G = networks.define_G(3, 3, 64, "resnet_9blocks", "instance", False, "normal", 0.02, [0])
D = networks.define_D(3, 64, "basic", 3, "instance", "normal", 0.02, [0])


def run(net, B, reps=10, cin=3):
    x = ops.nchw_to_nhwc(torch.rand(B, cin, 256, 256, device=dev) * 2 - 1)
    for _ in range(3):
        y = net.forward_nhwc(x)
        y.sum().backward()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        y = net.forward_nhwc(x)
        y.sum().backward()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


for name, net in (("G", G), ("D", D)):
    t4, t8, t16 = run(net, 4), run(net, 8), run(net, 16)
    print(name, "B4 %.2f ms  B8 %.2f ms (%.3f of 2xB4)  B16 %.2f ms (%.3f of 4xB4)" % (t4, t8, t8 / (2 * t4), t16,
                                                                                    t16 / (4 * t4)))
