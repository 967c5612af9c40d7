"""MoGAN step timing standalone (bench.mogan_train_fps)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    from gbvst import _lib
    _lib.load()
    print(json.dumps(bench.mogan_train_fps(torch.device("cuda:0"))))
