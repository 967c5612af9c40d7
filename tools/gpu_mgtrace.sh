#!/bin/bash
# MoGAN C5 kernel trace (tools/mgtrace.py under rocprofv3 --kernel-trace --stats), per optimize_parameters call.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-mgtrace}
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o p -- python3 tools/mgtrace.py 4 > $OUT/m.log 2> $OUT/m.err || { echo "mogan trace failed"; tail -20 $OUT/m.err; exit 1; }
CSV=$(find $OUT/kt -name '*kernel_trace.csv' | head -1)
python3 tools/profsum.py "$CSV" 6 90 > $OUT/mg_summary.txt && head -45 $OUT/mg_summary.txt | cut -c1-200
