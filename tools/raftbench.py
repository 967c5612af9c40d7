"""RAFT timings (bench.raft_inference at 436x1024 B=1 and 256x256 B=4, 20 iterations) standalone: the A/B tool for
the SepConvGRU convs' split-K plans (VST_FWD_HW_SPLITK)."""
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
    a = bench.raft_inference(dev, reps=5)
    b = bench.raft_inference(dev, B=4, H=256, W=256, reps=5)
    print(json.dumps({"arm": os.environ.get("VST_FWD_HW_SPLITK", "d") + "/" + os.environ.get("VST_RAFT_CS8", "d"), "sintel_ms": a["ms_per_call"],
                      "sintel_frac": a["roofline"]["frac"], "b4_256_ms": b["ms_per_call"], "b4_256_frac": b["roofline"]["frac"]}))
