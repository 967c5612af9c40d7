"""TEST INFRASTRUCTURE ONLY: writes tests/golden/fullsize_<case>.npz, the references of the full-size
parity tests (tests/test_gpu_fullsize.py), by running each case's oracle (oracle/fullsize_cases.py) in
fp64 (the exact result the HIP path is held to) and in fp32 on the CPU (the reference's own arithmetic,
whose distance to fp64 sets the tolerance), then summarising both (fullsize_cases.summarize).

usage: python oracle/gen_fullsize_refs.py [--out DIR] [case ...]   (cases: sg mg256 mgc5 c3)
The fp64 run goes to fullsize_cases.R64_DEVICE[case]: the CPU here, except the C5 MoGAN step, whose fp64
autograd graph outgrows this container's 64 GB — it runs in fp64 on a GPU box (torch's fp64 convs /
grid_sample, an exact-to-1e-15 reference like the CPU's), its fp32 run on that box's CPU:
    gpurun -- python oracle/gen_fullsize_refs.py --out gpurun_out/fixtures mgc5
A heartbeat line every 30 s keeps a long CPU run visibly alive.
"""
import argparse
import os
import sys
import threading
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from oracle import fullsize_cases  # noqa: E402


def _heartbeat(stop):
    t0 = time.time()
    while not stop.wait(30):
        print("  ... %.0f s" % (time.time() - t0), flush=True)


def main(argv):
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(REPO, "tests", "golden"))
    ap.add_argument("cases", nargs="*")
    a = ap.parse_args(argv)
    os.makedirs(a.out, exist_ok=True)
    stop = threading.Event()
    threading.Thread(target=_heartbeat, args=(stop,), daemon=True).start()
    try:
        for case in a.cases or list(fullsize_cases.ORACLES):
            run, dev = fullsize_cases.ORACLES[case], fullsize_cases.R64_DEVICE[case]
            t0 = time.time()
            r64 = run(torch.float64, dev)
            t1 = time.time()
            print("%s: fp64 on %s %.0f s" % (case, dev, t1 - t0), flush=True)
            r32 = run(torch.float32, "cpu")
            t2 = time.time()
            summ = fullsize_cases.summarize(r32, r64)
            path = os.path.join(a.out, "fullsize_%s.npz" % case)
            np.savez(path, **summ)
            print("%s: fp32 on cpu %.0f s, %d quantities, %.0f KB" % (
                case, t2 - t1, sum(k[0] in "LN" for k in summ), os.path.getsize(path) / 1024), flush=True)
    finally:
        stop.set()


if __name__ == "__main__":
    main(sys.argv[1:])
