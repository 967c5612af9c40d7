#!/bin/bash
# The batched-VGG equivalence test.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r05ee
timeout -k 10 300 python3 -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_style.py -m gpu -k "vgg" -p no:cacheprovider > gpurun_out/r05ee/t.log 2>&1; rc=$?; tail -25 gpurun_out/r05ee/t.log; exit $rc
