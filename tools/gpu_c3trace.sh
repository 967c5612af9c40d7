#!/bin/bash
# C3 train-step kernel trace (tools/c3trace.py under rocprofv3 --kernel-trace --stats), summarised per kernel and
# grid per step into gpurun_out/$TAG/c3_summary.txt.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-c3trace}
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o p -- python3 tools/c3trace.py 4 > $OUT/c3.log 2> $OUT/c3.err || { echo "c3 trace failed"; tail -20 $OUT/c3.err; exit 1; }
CSV=$(find $OUT/kt -name '*kernel_trace.csv' | head -1)
python3 tools/profsum.py "$CSV" 6 90 > $OUT/c3_summary.txt && head -40 $OUT/c3_summary.txt | cut -c1-200
