#!/bin/bash
# Johnson train-step kernel trace (tools/jstrace.py under rocprofv3 --kernel-trace --stats), summarised per kernel
# and grid per train step into gpurun_out/$TAG/js_summary.txt.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-jstrace}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o p -- python3 tools/jstrace.py 10 > $OUT/js.log 2> $OUT/js.err || { echo "js trace failed"; tail -20 $OUT/js.err; exit 1; }
CSV=$(find $OUT/kt -name '*kernel_trace.csv' | head -1)
python3 tools/profsum.py "$CSV" 13 90 > $OUT/js_summary.txt && head -40 $OUT/js_summary.txt | cut -c1-200
