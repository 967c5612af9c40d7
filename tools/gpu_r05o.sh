#!/bin/bash
# Round-5: the whole GPU suite on the current defaults (APRE_BWD on) + the StarGAN trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05o}
mkdir -p $O
timeout -k 10 700 python -u -m pytest -q --timeout 250 --timeout-method thread -m gpu tests > $O/t.log 2>&1
rc=$?
tail -2 $O/t.log
grep -E "^FAILED" $O/t.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc $rc: stop"; exit 1; fi
TAG=${TAG:-r05o}/sg bash tools/gpu_sgtrace.sh || exit 1
exit 0
