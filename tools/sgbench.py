"""StarGAN C4 iteration timing (bench.stargan_train_fps) standalone, optional per-phase breakdown."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402


def phases(device, B=4, S=256, reps=3):
    from gbvst import stargan
    sol = stargan.StarGANSolver(image_size=S, c_dim=4, n_critic=5, device=device)
    x = (torch.rand(B, 3, S, S) * 2 - 1).to(device)
    c = stargan.label2onehot(torch.tensor([0, 1, 2, 3][:B] * (B // 4 or 1)), 4, device)
    out = {}

    def tm(name, fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        out[name] = round((time.perf_counter() - t0) / reps * 1e3, 3)

    tm("G_fwd_grad", lambda: sol.G(x, c))
    with torch.no_grad():
        tm("G_fwd_nograd", lambda: sol.G(x, c))
    tm("D_fwd", lambda: sol.D(x))

    def d_fb():
        s, cl = sol.D(x)
        (s.mean() + cl.mean()).backward()
    tm("D_fwd_bwd", d_fb)

    def gp():
        xh = x.clone().requires_grad_(True)
        s, _ = sol.D(xh)
        stargan.gradient_penalty(s, xh).backward()
    tm("D_gp_double_bwd", gp)

    def g_fb():
        y = sol.G(x, c)
        y.mean().backward()
    tm("G_fwd_bwd", g_fb)
    return out


if __name__ == "__main__":
    dev = torch.device("cuda:0")
    from gbvst import _lib
    _lib.load()
    print(json.dumps(phases(dev)))
    print(json.dumps(bench.stargan_train_fps(dev)))
