"""Generate tests/golden/formats.npz with the READ-ONLY reference utils/flowlib.py.

TEST INFRASTRUCTURE ONLY — build container only.

    cd /tmp && PYTHONDONTWRITEBYTECODE=1 python /root/repo/oracle/gen_golden_formats.py

The reference writeFlow writes a .flo for a seeded flow (non-square, negative and fractional values);
the fixture keeps the file's bytes and readFlow's result, so tests/test_formats.py checks our reader
and writer byte for byte.
"""
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from oracle import prng  # noqa: E402


def main():
    sys.path.insert(0, "/root/reference/utils")
    import flowlib  # noqa
    flow = prng.normal(901, (7, 11, 2), std=5.0)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "a.flo")
        flowlib.writeFlow(p, flow)
        raw = np.frombuffer(open(p, "rb").read(), np.uint8).copy()
        back = flowlib.readFlow(p)
    out = os.path.join(REPO, "tests", "golden", "formats.npz")
    np.savez_compressed(out, flo_flow=flow, flo_bytes=raw, flo_read=back)
    print(out, os.path.getsize(out))


if __name__ == "__main__":
    main()
