#!/bin/bash
# Round-5: patch.hip kernels — parity tests, then the step kernel trace (their in-step durations).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05d}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_patch.py ${EXTRA_TESTS} > $O/t.log 2>&1 || { echo tests failed; tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
TAG=${TAG:-r05d}/trace bash tools/gpu_trace.sh > /dev/null || exit 1
grep -E "${PAT:-patch|skinny|chsum}" $O/trace/step_summary.txt | cut -c1-170
head -1 $O/trace/step_summary.txt
