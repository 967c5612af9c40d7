#!/bin/bash
# Round-5: the whole GPU suite on the current sources, then a same-box step A/B ($ARMS).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05f}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/t.log 2>&1 || { echo tests failed; tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
[ -n "$ARMS" ] && TAG=${TAG:-r05f}/ab bash tools/ab_step.sh
exit 0
