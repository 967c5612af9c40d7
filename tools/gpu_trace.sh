#!/bin/bash
# Step kernel trace of the C2 bench line (rocprofv3 --kernel-trace --stats), summarised per kernel
# and grid into gpurun_out/$TAG/step_summary.txt (tools/profsum.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-trace}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o p -- python3 bench.py --steps 7 --warmup 3 --no-cpu-baseline --no-extras > $OUT/bench_kt.json 2> $OUT/bench_kt.err || { echo "trace failed"; tail -20 $OUT/bench_kt.err; exit 1; }
CSV=$(find $OUT/kt -name '*kernel_trace.csv' | head -1)
python3 tools/profsum.py "$CSV" 10 80 > $OUT/step_summary.txt && head -45 $OUT/step_summary.txt | cut -c1-200
