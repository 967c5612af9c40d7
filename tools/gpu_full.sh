#!/bin/bash
# The whole GPU suite, then smoke() — one process each, bounded.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-full}
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests > $OUT/pytest.log 2>&1; rc=$?
tail -4 $OUT/pytest.log
[ $rc -ne 0 ] && { grep -E "^FAILED|^ERROR|Error" $OUT/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; tail -2 $OUT/smoke.log; exit $rc
