#!/bin/bash
# wgrad_reduce_store_k 16-row blocks (VST_WG_RED16=1): wgrad tests under it, then the step A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/wgred
mkdir -p $O
VST_WG_RED16=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "wgrad or production or conv_fwd_dgrad_wgrad" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/pytest.log | head -20; exit $rc; }
ARMS="default VST_WG_RED16=1" TAG=wgred STEPS=20 bash tools/ab_step.sh
