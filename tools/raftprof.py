"""RAFT inference loop for rocprofv3 (kernel stats): B x 3 x H x W, 20 iterations, eager (no graph)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=4)
    ap.add_argument("--H", type=int, default=256)
    ap.add_argument("--W", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from gbvst import _lib, raft
    _lib.load()
    dev = torch.device("cuda:0")
    m = raft.RAFT(argparse.Namespace(small=False)).to(dev).eval()
    m.use_graphs = False
    i1 = torch.rand(a.B, 3, a.H, a.W, device=dev) * 255
    i2 = torch.rand(a.B, 3, a.H, a.W, device=dev) * 255
    for _ in range(a.reps):
        raft.compute_raft(m, i1, i2, it=20)
    torch.cuda.synchronize()
    print("done")
