"""Developer probe: is torch's float64 conv2d / conv_transpose2d / grid_sample usable on this GPU (for
running the fp64 oracle of the parity tests on the device)?  Times a ResnetBlock-shape conv fwd+bwd."""
import time

import torch
import torch.nn.functional as F

dev = torch.device("cuda")
for dt in (torch.float32, torch.float64):
    x = torch.randn(8, 256, 64, 64, device=dev, dtype=dt, requires_grad=True)
    w = (torch.randn(256, 256, 3, 3, device=dev, dtype=dt) * 0.02).requires_grad_(True)
    for _ in range(2):
        y = F.conv2d(F.pad(x, (1,) * 4, mode="reflect"), w)
        y.sum().backward()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        y = F.conv2d(F.pad(x, (1,) * 4, mode="reflect"), w)
        y.sum().backward()
    torch.cuda.synchronize()
    print(dt, "resblock conv fwd+bwd N=8: %.2f ms" % ((time.perf_counter() - t0) / 3 * 1e3), flush=True)
    xt = torch.randn(4, 256, 64, 64, device=dev, dtype=dt)
    wt = torch.randn(256, 128, 3, 3, device=dev, dtype=dt)
    yt = F.conv_transpose2d(xt, wt, stride=2, padding=1, output_padding=1)
    g = F.grid_sample(torch.randn(1, 3, 64, 64, device=dev, dtype=dt), torch.rand(1, 64, 64, 2, device=dev, dtype=dt) * 2 - 1,
                      align_corners=False)
    torch.cuda.synchronize()
    print(dt, "convT", tuple(yt.shape), "grid_sample", tuple(g.shape), flush=True)
