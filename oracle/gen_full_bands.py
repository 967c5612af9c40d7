"""Generate tests/golden/full_bands.npz — TEST INFRASTRUCTURE: the rounding bands of the reference
arithmetic at the full sizes of tests/test_gpu_fullsize.py (StarGAN C4 iteration, RAFT at the Sintel
frame size, MoGAN E + M step, C3 step).

Each oracle run of that module (sg_oracle, raft_oracle, mg_oracle, c3_oracle: the CPU restatements,
pinned to the reference by tests/test_oracle_*.py) is repeated with every weight scaled by
(1 + 1e-6 N(0,1)) — a forward change of the size any other fp32 summation order makes — and the
largest deviation over the perturbed runs is stored per quantity (loss: relative; gradient:
norm-wise relative; tensor: max-abs relative to max|ref|), plus the fraction of fb-check mask pixels
that flip.  The GPU tests recompute the unperturbed oracle live and allow max(floor, 3 x band).

    python oracle/gen_full_bands.py [sg raft mogan c3]     (default: all; merges into the file)
"""
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
OUT = os.path.join(REPO, "tests", "golden", "full_bands.npz")
SEEDS = {"sg": 2, "raft": 2, "mogan": 2, "c3": 2}


def main(which):
    import test_gpu_fullsize as t
    fns = {"sg": t.sg_oracle, "raft": t.raft_oracle, "mogan": t.mg_oracle, "c3": t.c3_oracle}
    out = dict(np.load(OUT)) if os.path.exists(OUT) else {}
    for name in which:
        t0 = time.time()
        ref = fns[name]()
        prefix = name + "|"
        for k in [k for k in out if k.startswith(prefix)]:
            del out[k]
        for s in range(SEEDS[name]):
            run = fns[name](t.PERTURB, seed=100 + 10 * s)
            for key, r in ref.items():
                dev = t.deviation(key, run[key], r)
                out[prefix + key] = np.array(max(float(out.get(prefix + key, 0.0)), dev))
            if name == "mogan":
                flip = float((run["e_tensor|mask_A"] != ref["e_tensor|mask_A"]).double().mean())
                out["mogan|e_maskflip"] = np.array(max(float(out.get("mogan|e_maskflip", 0.0)), flip))
        np.savez_compressed(OUT, **out)
        big = sorted(((float(v), k) for k, v in out.items() if k.startswith(prefix)), reverse=True)
        print(name, "%.0f s" % (time.time() - t0), [(k, "%.2e" % v) for v, k in big if "bias" not in k][:8],
              flush=True)


if __name__ == "__main__":
    torch.set_num_threads(os.cpu_count() or 1)
    main(sys.argv[1:] or ["sg", "raft", "mogan", "c3"])
