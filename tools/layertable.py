"""Per-layer roofline table of the C2 train step's conv ops: every conv-family
entry of gbvst.ops called during one optimize_parameters() (after warm-up) is wrapped with HIP events
on the current stream (outermost call only), keyed by (op, shapes); algorithmic FLOPs use the
reference's real channel counts (3-channel images, 1-channel PatchGAN head), so a frac counts padding
as waste.  usage: layertable.py [steps] -> JSON lines {op, layer, n, us, tflops, frac} + aggregates."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
import gbvst  # noqa: E402
from gbvst import ops  # noqa: E402
from tools import convflops  # noqa: E402
from gbvst.cycle_gan_model import CycleGANModel  # noqa: E402
from gbvst.options import default_opt  # noqa: E402

PEAK = bench.BF16_MFMA_PEAK_TFLOPS / 6.0


rec = {}


def timed(name, lab, f, fn, a, k):
    """convflops.Counter hook: HIP events on the current stream around the outermost op call."""
    if not rec.get("_on"):
        return fn(*a, **k)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    out = fn(*a, **k)
    e1.record()
    rec.setdefault((name, lab), []).append((e0, e1, f))
    return out


gbvst._lib.load()
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
dev = torch.device("cuda", 0)
m = CycleGANModel(default_opt(True, gpu_ids=[0], pool_size=50))
a, a2, b, mask, flow = bench.synthetic_batch(4, 256, 256, 1234, dev)
m.set_input_nhwc(ops.nchw_to_nhwc(a), ops.nchw_to_nhwc(a2), ops.nchw_to_nhwc(b), mask.contiguous(), flow.contiguous())
with convflops.Counter(on_call=timed):
    for _ in range(4):
        m.optimize_parameters()
    torch.cuda.synchronize()
    rec["_on"] = True
    for _ in range(steps):
        m.optimize_parameters()
    torch.cuda.synchronize()
    rec.pop("_on")
rows, tot_ms, tot_f, res_ms, res_f = [], 0.0, 0.0, 0.0, 0.0
for (name, lab), evs in rec.items():
    ms = sum(e0.elapsed_time(e1) for e0, e1, _ in evs)
    f = sum(x for _, _, x in evs)
    resblock = "256->256" in lab and "@64x64" in lab or ("256->256" in lab and "out 64x64" in lab)
    rows.append({"op": name, "layer": lab, "calls_per_step": len(evs) / steps, "ms_per_step": round(ms / steps, 3),
                 "us_per_call": round(ms / len(evs) * 1e3, 1), "tflops": round(f / (ms * 1e-3) / 1e12, 1),
                 "frac": round(f / (ms * 1e-3) / 1e12 / PEAK, 3), "resblock": bool(resblock)})
    if resblock:
        res_ms, res_f = res_ms + ms, res_f + f
    else:
        tot_ms, tot_f = tot_ms + ms, tot_f + f
rows.sort(key=lambda r: -r["ms_per_step"])
for r in rows:
    print(json.dumps(r))
print(json.dumps({"aggregate_non_resblock": {"ms_per_step": round(tot_ms / steps, 2), "tflop_per_step": round(tot_f / steps / 1e12, 3),
                                             "frac": round(tot_f / (tot_ms * 1e-3) / 1e12 / PEAK, 3)},
                  "aggregate_resblock": {"ms_per_step": round(res_ms / steps, 2), "tflop_per_step": round(res_f / steps / 1e12, 3),
                                         "frac": round(res_f / (res_ms * 1e-3) / 1e12 / PEAK, 3)}}))
