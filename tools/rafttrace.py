"""RAFT (full model, 436x1024, 20 iterations, B=1) calls for a kernel trace (rocprofv3 --kernel-trace --stats --
python3 tools/rafttrace.py): 2 warm-up calls, then `calls` traced calls (bench.raft_inference's workload)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main(calls=5, B=1, H=436, W=1024):
    from gbvst import _lib, raft
    _lib.load()
    dev = torch.device("cuda:0")
    m = raft.RAFT(argparse.Namespace(small=False)).to(dev).eval()
    g = torch.Generator(device="cpu").manual_seed(5)
    i1 = (torch.rand(B, 3, H, W, generator=g) * 255).to(dev)
    i2 = (torch.rand(B, 3, H, W, generator=g) * 255).to(dev)
    for _ in range(2 + calls):
        raft.compute_raft(m, i1, i2, it=20)
    torch.cuda.synchronize()
    print("calls", 2 + calls)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 5)
