"""Johnson (B=4 256^2) and C3 (1x436x1024) train-step timings (bench.johnson_train_fps / c3_train_fps) standalone,
with the peak device memory of each, under the batched VGG forwards (perceptual._VggMultiFn, the default) and the
per-image calls (`python tools/vggbench.py unbatched`): the A/B of the batched route's time and memory (ADVICE r5:
the batch keeps the target images' activations until backward)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda:0")
    from gbvst import _lib, cycle_gan_vgg_model, faststyle
    _lib.load()
    arm = sys.argv[1] if len(sys.argv) > 1 else "batched"
    faststyle.VGG_BATCHED = cycle_gan_vgg_model.VGG_BATCHED = arm == "batched"
    torch.zeros(1, device=dev)  # the allocator's device state exists only once the context does
    torch.cuda.reset_peak_memory_stats(dev)
    j = bench.johnson_train_fps(dev, steps=10)
    j_mem = torch.cuda.max_memory_allocated(dev)
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats(dev)
    c = bench.c3_train_fps(dev)
    c_mem = torch.cuda.max_memory_allocated(dev)
    print(json.dumps({"arm": arm, "johnson_ms": j["ms_per_step"], "johnson_frac": j["roofline"]["frac"],
                      "johnson_peak_mib": round(j_mem / 2 ** 20, 1), "c3_ms": c["ms_per_step"],
                      "c3_frac": c["roofline"]["frac"], "c3_peak_mib": round(c_mem / 2 ** 20, 1)}))
