"""Host-side argument validation of the C ABI (include/vst_hip.h): every entry point given null pointers
or bad shapes returns an error status BEFORE any launch, so these calls run without a GPU.  Run under
the host-ASan build by tools/asan_host.sh (VST_LIB_VARIANT=<asan lib>): any out-of-bounds host access
in the validation / planning code aborts the process."""
import ctypes

import pytest


@pytest.fixture(scope="module")
def lib():
    import gbvst
    return gbvst._lib.load()


def test_bad_arguments_rejected_on_host(lib):
    import os
    from gbvst import _lib
    if os.environ.get("VST_LIB_VARIANT"):  # the ASan run: the instrumented build is the one loaded
        assert _lib.LIB_PATH == os.environ["VST_LIB_VARIANT"] and "asan" in _lib.LIB_PATH
    null = None
    assert lib.vst_warp_fwd(null, null, null, 1, 8, 8, 4, 0, null) != 0
    assert lib.vst_warp_bwd_input(null, null, null, 1, 8, 8, 4, 0, null) != 0
    assert lib.vst_warp_bwd_input_det(null, null, null, null, 0, 1, 8, 8, 4, 3, 0, 0, 0, null) != 0
    assert lib.vst_fbcheck(null, null, null, 1, 8, 8, null) != 0
    assert lib.vst_loss_temporal(null, null, null, null, null, null, 1, 8, 8, 4, 3, 10.0, null) != 0
    msg = lib.vst_last_error()
    assert msg and b"bad args" in msg


def test_workspace_queries_are_host_only(lib):
    assert lib.vst_warp_bwd_det_ws_bytes(2, 64, 80) >= 2 * 4 * 2 * 64 * 80 * 8
    for N in (1, 8):
        assert lib.vst_conv2d_wgrad_ws_bytes(N, 64, 64, 256, 64, 64, 256, 3, 3, 1) > 0
    kind, ms, tk = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    for N in (1, 4, 8, 12, 16):
        assert lib.vst_conv_plan_fwd(N, 64, 64, 256, 256, 3, 3, 1, 1, 1, 2, ctypes.byref(kind), ctypes.byref(ms),
                                     ctypes.byref(tk)) == 0
