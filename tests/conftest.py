import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    return load


# Conv arithmetic policies (gbvst.ops.set_conv_math): uniform ones for single-op tests, the
# training-capable ones (forward at fp32 accuracy) for network-gradient / train-step tests.
OP_MATHS = ["fp32", "bf16x3", "bf16x6"]
TRAIN_MATHS = ["fp32", "bf16x6", "mixed"]
# written tolerances for conv-family results, relative to max|ref|: exact fp32 MFMA differs from
# the CPU only in summation order; bf16x6 is fp32-equivalent (dropped terms <= 2^-24 relative);
# bf16x3 products carry <= ~2^-16 relative error each.
CONV_TOL = {"fp32": 2e-5, "bf16x3": 1e-4, "bf16x6": 2e-5, "mixed": 1e-4}


def _math_fixture(request):
    import gbvst
    from gbvst import ops
    gbvst._lib.load()
    prev = ops.set_conv_math(request.param)
    yield request.param
    ops.set_conv_math(prev)


@pytest.fixture(params=OP_MATHS)
def conv_math(request):
    """Run the test under each uniform conv arithmetic (VST_MATH_F32 / _BF16X3 / _BF16X6)."""
    yield from _math_fixture(request)


@pytest.fixture(params=TRAIN_MATHS)
def train_math(request):
    """Run the test under each training policy (fp32, bf16x6, mixed = x6 forward + x3 gradients)."""
    yield from _math_fixture(request)


@pytest.fixture(params=OP_MATHS + ["mixed"])
def infer_math(request):
    yield from _math_fixture(request)


@pytest.fixture(params=["bf16x6", "mixed"])
def prod_math(request):
    """The policies bench.py measures (bf16x6 headline, mixed labelled): the full-size parity tests."""
    yield from _math_fixture(request)
