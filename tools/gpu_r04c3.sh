#!/bin/bash
# Round-4 GPU check of the 3-row image-input weight gradient (VST_WG_C3): the conv / wgrad parity tests,
# the generator / step tests, then the same-box step A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04c3
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ops.py tests/test_gpu_models.py tests/test_gpu_train.py > $O/t.log 2>&1 || { echo tests failed; tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
ARMS="default VST_WG_C3=0" TAG=r04c3/ab bash tools/ab_step.sh
