"""Johnson (B=4 256^2) and C3 (1x436x1024) train-step timings (bench.johnson_train_fps / c3_train_fps) standalone:
the A/B tool for the VGG backward route (VST_VGG_DGRAD_FPROP)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda:0")
    from gbvst import _lib
    _lib.load()
    j = bench.johnson_train_fps(dev, steps=10)
    c = bench.c3_train_fps(dev)
    print(json.dumps({"arm": os.environ.get("VST_VGG_DGRAD_FPROP", "default") + "/" + os.environ.get("VST_FS_DGRAD_FPROP", "default"), "johnson_ms": j["ms_per_step"],
                      "johnson_frac": j["roofline"]["frac"], "c3_ms": c["ms_per_step"], "c3_frac": c["roofline"]["frac"]}))
