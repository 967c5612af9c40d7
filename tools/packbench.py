"""Developer: time one batched weight-pack refresh (ops.PackBatch.run, vst_weight_pack_batch) of the C2 networks
(ResnetGenerator, PatchGAN D) and the StarGAN C4 discriminator / generator; VST_PACK_KERNEL selects the kernel form.
Prints one JSON line of per-network microseconds (HIP events, median of 20)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import gbvst  # noqa: E402
from gbvst import networks, stargan  # noqa: E402

gbvst._lib.load()
dev = torch.device("cuda")
nets = {"cyclegan_G": networks.define_G(3, 3, 64, "resnet_9blocks", "instance", False, "normal", 0.02, [0]),
        "cyclegan_D": networks.define_D(3, 64, "basic", 3, "instance", "normal", 0.02, [0]),
        "stargan_D": stargan.Discriminator(256, 64, 4, 6).to(dev), "stargan_G": stargan.Generator(64, 4, 6).to(dev)}
out = {"kernel": os.environ.get("VST_PACK_KERNEL", "default")}
for name, net in nets.items():
    net.packs()
    pb = net._packs[2]
    ts = []
    for _ in range(25):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        pb.run()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    out[name + "_us"] = round(sorted(ts[5:])[10], 1)
print(json.dumps(out))
