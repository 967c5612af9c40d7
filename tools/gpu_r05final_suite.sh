#!/bin/bash
# The whole GPU suite + smoke() on the final tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r05final
timeout -k 10 700 python3 -u -m pytest -q --timeout 280 --timeout-method thread tests -m gpu -p no:cacheprovider > gpurun_out/r05final/t.log 2>&1 || { tail -30 gpurun_out/r05final/t.log; exit 1; }
tail -1 gpurun_out/r05final/t.log
timeout -k 10 300 python3 -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > gpurun_out/r05final/smoke.log 2>&1 || { tail -20 gpurun_out/r05final/smoke.log; exit 1; }
tail -1 gpurun_out/r05final/smoke.log
