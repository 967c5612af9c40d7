#!/bin/bash
# StarGAN C4 kernel trace (tools/sgtrace.py under rocprofv3 --kernel-trace --stats), summarised per kernel and
# grid per train_step call into gpurun_out/$TAG/sg_summary.txt.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-sgtrace}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o p -- python3 tools/sgtrace.py 2 > $OUT/sg.log 2> $OUT/sg.err || { echo "sg trace failed"; tail -20 $OUT/sg.err; exit 1; }
CSV=$(find $OUT/kt -name '*kernel_trace.csv' | head -1)
python3 tools/profsum.py "$CSV" 25 90 > $OUT/sg_summary.txt && head -30 $OUT/sg_summary.txt | cut -c1-200
