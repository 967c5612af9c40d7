#!/bin/bash
# The whole GPU suite on the current tree (round-5 final record).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r05suite
timeout -k 10 700 python3 -u -m pytest -q --timeout 280 --timeout-method thread tests -m gpu -p no:cacheprovider > gpurun_out/r05suite/t.log 2>&1; rc=$?; tail -3 gpurun_out/r05suite/t.log; exit $rc
