"""Generate tests/golden/full_step_band.npz: the rounding band of the reference's own arithmetic for
one full-size C2 train step (ngf=ndf=64, 256x256, B=4, pool_size 0) — TEST INFRASTRUCTURE.

The CPU oracle (oracle/cpu_ref.RefCycleGANCon, pinned to the reference by tests/test_oracle_golden)
runs the step once in fp32 and once in fp64 on the counter-PRNG weights / synthetic inputs of
tests/test_gpu_models.py::test_full_size_train_step_vs_oracle.  Stored per parameter: the norm-wise
relative fp64-vs-fp32 gradient deviation; plus the step-0 losses of both runs and the max |fp64 -
fp32| of G_A(probe) after the Adam update (Adam's first step is ~lr*sign(g), so rounding-level
gradient noise moves near-zero parameters by 2*lr).  The GPU test recomputes the fp32 oracle live
and uses these bands as its tolerance scale (the fp64 step takes minutes on a CPU).
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]


def main():
    import test_gpu_models as t
    torch.manual_seed(0)
    l32, g32, p32 = t._oracle_full_step(torch.float32)
    l64, g64, p64 = t._oracle_full_step(torch.float64)
    out = {"loss_names": np.array(sorted(l32)),
           "losses32": np.array([l32[k] for k in sorted(l32)]),
           "losses64": np.array([l64[k] for k in sorted(l64)]),
           "probe_dev64": np.array((p64 - p32).abs().max().item())}
    for n in g32:
        for k in g32[n]:
            out[f"band_{n}_{k}"] = np.array(t._norm_rel(g32[n][k], g64[n][k]))
    np.savez_compressed(os.path.join(REPO, "tests", "golden", "full_step_band.npz"), **out)
    print({k: float(v) for k, v in out.items() if k.startswith("band") and float(v) > 1e-4})


if __name__ == "__main__":
    main()
