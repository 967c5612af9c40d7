#!/bin/bash
# Inference kernel traces (rocprofv3 --kernel-trace --stats) of tools/infbench.py at B=1 / B=16 256x256
# and 1x436x1024, summarised per kernel into gpurun_out/$TAG/inf_<cfg>.txt (tools/profsum.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-inftrace}
mkdir -p $OUT
for cfg in "1 256 256 30" "16 256 256 10" "1 436 1024 10"; do
  set -- $cfg
  name=b$1_$2x$3
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$name -o p -- python3 tools/infbench.py $cfg > $OUT/$name.log 2>&1 || { echo "trace failed $name"; tail -20 $OUT/$name.log; exit 1; }
  CSV=$(find $OUT/kt_$name -name '*kernel_trace.csv' | head -1)
  # the 3 warm-up calls are in the trace too: per-call figures divide by reps + 3
  python3 tools/profsum.py "$CSV" $(( $4 + 3 )) 60 > $OUT/inf_$name.txt && head -30 $OUT/inf_$name.txt | cut -c1-200
  cat $OUT/$name.log | tail -1
done
