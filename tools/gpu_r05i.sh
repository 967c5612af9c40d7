#!/bin/bash
# Round-5 batch: the whole GPU suite (DGRAD_EPI on by default), the step trace, the weight-gradient cold-operand
# experiment, the StarGAN trace, the B=1 all-split tile A/B.  A test failure (rc 1) does not stop the batch;
# any other non-zero status (fault, abort, time limit) does.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05i}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests > $O/t.log 2>&1
rc=$?
tail -3 $O/t.log
grep -E "^FAILED" $O/t.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc $rc: stop"; exit 1; fi
TAG=${TAG:-r05i}/trace bash tools/gpu_trace.sh > /dev/null || exit 1
head -12 $O/trace/step_summary.txt | cut -c1-170
TAG=${TAG:-r05i}/wgcold bash tools/gpu_wgcold.sh || exit 1
TAG=${TAG:-r05i}/sg bash tools/gpu_sgtrace.sh || exit 1
ARMS="default VST_FULLSPLIT_TILE=128" TAG=${TAG:-r05i}/infab bash tools/gpu_infab.sh || exit 1
exit 0
