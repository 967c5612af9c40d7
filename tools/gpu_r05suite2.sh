#!/bin/bash
# The convT phase tests, then the whole GPU suite on the current tree (round-5 final record).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r05suite
timeout -k 10 200 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -m gpu -k convT_phases -p no:cacheprovider > gpurun_out/r05suite/t1.log 2>&1 || { tail -20 gpurun_out/r05suite/t1.log; exit 1; }
tail -1 gpurun_out/r05suite/t1.log
timeout -k 10 700 python3 -u -m pytest -q --timeout 280 --timeout-method thread tests -m gpu -p no:cacheprovider > gpurun_out/r05suite/t.log 2>&1; rc=$?; tail -3 gpurun_out/r05suite/t.log; exit $rc
