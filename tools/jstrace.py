"""Johnson fast-style train steps for a kernel trace (rocprofv3 --kernel-trace --stats -- python3 tools/jstrace.py):
3 warm-up steps, then `steps` traced steps (bench.johnson_train_fps's workload: B=4, 256x256)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main(steps=10, B=4, S=256):
    from gbvst import _lib, faststyle
    _lib.load()
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(7)
    J = faststyle.Johnson([torch.rand(1, 3, S, S, generator=g)], lr=1e-3, batch_sz=B, device=dev)
    x = torch.rand(B, 3, S, S, generator=g).to(dev)
    for _ in range(3 + steps):
        J.train_step(x)
    torch.cuda.synchronize()
    print("steps", 3 + steps)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 10)
