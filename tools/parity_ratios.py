"""Per-parameter view of the full-size parity logs (VST_PARITY_LOG=<dir> pytest tests/test_gpu_fullsize.py):
for every gradient the ratio of the HIP deviation from the fp64 reference to the reference's OWN fp32
deviation (dev_hip_vs_ref64 / dev_ref32_vs_ref64), the largest per case, and the keys above a threshold.
usage: parity_ratios.py <log dir> [threshold]"""
import glob
import json
import os
import sys

d = sys.argv[1]
thr = float(sys.argv[2]) if len(sys.argv) > 2 else 10.0
worst = []
for f in sorted(glob.glob(os.path.join(d, "fullsize_*.json"))):
    rows = json.load(open(f))
    rat = []
    for k, v in rows.items():
        if "grad" not in k.split("|", 1)[0]:
            continue
        h, r = v["dev_hip_vs_ref64"], v["dev_ref32_vs_ref64"]
        rat.append((h / max(r, 1e-12), k, h, r, v["tol"]))
    rat.sort(reverse=True)
    print("%s: %d gradients, max HIP/own-fp32 ratio %.2f (%s: dev %.2e own %.2e tol %.2e)" % (
        os.path.basename(f), len(rat), rat[0][0], rat[0][1], rat[0][2], rat[0][3], rat[0][4]) if rat else f)
    for r_ in rat:
        if r_[0] > thr and r_[2] > 2e-3:
            print("   above %.0f with dev > 2e-3: %s ratio %.2f dev %.2e own %.2e" % (thr, r_[1], r_[0], r_[2], r_[3]))
    worst += rat[:1]
