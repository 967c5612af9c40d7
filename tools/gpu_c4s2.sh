#!/bin/bash
# Last-layer forward as the 7x1 conv + column tap sum (vst_tapconv_h_fwd): parity tests, model tests,
# kernel stats of one step, step A/B vs the 1x1 conv + full tap-sum route.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/c4s2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "conv4s2 or convT or conv_transpose" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_models.py > $O/pytest_models.log 2>&1; rc=$?; tail -3 $O/pytest_models.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/pytest_models.log | head -20; exit $rc; }
ARMS="default VST_C4S2_GROUPED=0" TAG=c4s2 STEPS=20 bash tools/ab_step.sh
