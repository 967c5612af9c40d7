#!/bin/bash
# RAFT Sintel-size kernel trace (tools/rafttrace.py under rocprofv3 --kernel-trace --stats) + the Johnson trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-rafttrace}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o p -- python3 tools/rafttrace.py 5 > $OUT/r.log 2> $OUT/r.err || { echo "raft trace failed"; tail -20 $OUT/r.err; exit 1; }
CSV=$(find $OUT/kt -name '*kernel_trace.csv' | head -1)
python3 tools/profsum.py "$CSV" 7 90 > $OUT/raft_summary.txt && head -40 $OUT/raft_summary.txt | cut -c1-200
TAG=$TAG/js bash tools/gpu_jstrace.sh > /dev/null || exit 1
head -30 $OUT/js/js_summary.txt | cut -c1-200
