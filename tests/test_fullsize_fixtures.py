"""CPU checks of the full-size parity machinery (tests/test_gpu_fullsize.py): the CountSketch norm
estimator (oracle/sketch.py) and the committed fullsize_*.npz references."""
import os

import numpy as np
import pytest
import torch

from oracle import fullsize_cases as fc
from oracle import sketch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("rel", [1e-3, 2e-2])
def test_sketch_estimates_deviation_norm(rel):
    g = torch.Generator().manual_seed(7)
    ref = torch.randn(400_000, generator=g, dtype=torch.float64)
    ratios = []
    for t in range(4):
        noise = torch.randn(ref.numel(), generator=g, dtype=torch.float64)
        got = ref + rel * float(ref.norm()) / ref.numel() ** 0.5 * noise
        est = sketch.sketch_dev(sketch.count_sketch(got), sketch.count_sketch(ref), float(ref.norm()))
        ratios.append(est / (float((got - ref).norm()) / float(ref.norm())))
    assert max(abs(r - 1) for r in ratios) < 0.1, ratios


def test_sketch_is_linear_and_layout_free():
    a = torch.randn(3, 5000, dtype=torch.float64)
    b = torch.randn(3, 5000, dtype=torch.float64)
    assert torch.allclose(sketch.count_sketch(a + 2 * b), sketch.count_sketch(a) + 2 * sketch.count_sketch(b))
    assert torch.equal(sketch.count_sketch(a), sketch.count_sketch(a.reshape(-1)))


def test_deviations_against_a_summary():
    g = torch.Generator().manual_seed(3)
    r64 = fc.flatten({"x": 2.0}, {"G": {"w": torch.randn(64, 64, 3, 3, generator=g, dtype=torch.float64),
                                        "b": torch.randn(64, generator=g, dtype=torch.float64)}}, {})
    r32 = {k: (v if isinstance(v, float) else v.float().double()) for k, v in r64.items()}
    summ = fc.summarize(r32, r64)
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "vst_fullsize_selftest.npz")
    np.savez(path, **summ)
    fx = np.load(path, allow_pickle=False)
    got = {k: (v * 1.001 if isinstance(v, float) else v * 1.001) for k, v in r64.items()}
    rows = fc.deviations(got, fx)
    assert set(rows) == set(r64)
    for k, (dev, dref) in rows.items():
        assert abs(dev - 1e-3) < 1e-4, (k, dev)
        assert dref < 1e-6


@pytest.mark.parametrize("case", list(fc.ORACLES))
def test_fullsize_fixture_committed(case):
    fx = np.load(os.path.join(GOLDEN, "fullsize_%s.npz" % case), allow_pickle=False)
    keys = {n.split(":", 1)[1] for n in fx.files}
    losses = [k for k in keys if fc.kind(k) == "loss"]
    grads = [k for k in keys if fc.kind(k) == "grad"]
    assert losses and len(grads) > 20
    for k in grads:
        n64, d32, numel = fx["N:" + k]
        assert n64 >= 0 and numel >= 1
        # the reference's own fp32 error is small except where the exact gradient is ~0 (IN-preceded
        # biases: rounding noise on every side; magnitude-checked in the GPU test)
        assert n64 < 1e-10 or 0 <= d32 < 0.2, (k, n64, d32)
        assert ("V:" + k in fx.files) != ("S:" + k in fx.files)
