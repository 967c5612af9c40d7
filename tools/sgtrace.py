"""StarGAN C4 iterations for a kernel trace (rocprofv3 --kernel-trace --stats -- python3 tools/sgtrace.py):
3 n_critic cycles of warm-up, then `cycles` traced cycles (5 D iterations + 1 G step each) bracketed by
roctx-free synchronisation; the summary divides by the number of train_step calls (profsum.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main(cycles=2, B=4, S=256):
    from gbvst import _lib, stargan
    _lib.load()
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(11)
    sol = stargan.StarGANSolver(image_size=S, c_dim=4, n_critic=5, device=dev)
    x = (torch.rand(B, 3, S, S, generator=g) * 2 - 1).to(dev)
    lo = torch.randint(0, 4, (B,), generator=g)
    lt = torch.randint(0, 4, (B,), generator=g)
    for _ in range(5 * (3 + cycles)):
        sol.train_step(x, lo, lt)
    torch.cuda.synchronize()
    print("steps", 5 * (3 + cycles))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 2)
