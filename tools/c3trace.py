"""C3 train steps (bench.c3_train_fps's workload: CycleGANCon + flow warp + VGG-19 content / Gram losses at
1x436x1024) for a kernel trace: rocprofv3 --kernel-trace --stats -- python3 tools/c3trace.py [steps]."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    from gbvst import _lib, ops
    _lib.load()
    ops.set_conv_math("bf16x6")
    print(bench.c3_train_fps(torch.device("cuda:0"), steps=steps))
