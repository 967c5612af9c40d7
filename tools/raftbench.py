"""RAFT inference timing standalone (bench.raft_inference) at the Sintel and MoGAN sizes."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    from gbvst import _lib, ops
    _lib.load()
    dev = torch.device("cuda:0")
    for pol in sys.argv[1:] or ["mixed"]:
        ops.set_conv_math(pol)
        print(pol, json.dumps(bench.raft_inference(dev)))
        print(pol, json.dumps(bench.raft_inference(dev, B=4, H=256, W=256)))
