#!/bin/bash
# Same-box kernel A/B of the ResnetBlock weight gradient (N=8): the channel-major route (tools/kbench.py wgrad_pre:
# the IN passes' premade x image / dy planes) against the NHWC-operand kernel (wgrad_nhwc), two interleaved rounds
# of rocprofv3 kernel traces; per-kernel averages into gpurun_out/$TAG/wgrad_ab.txt.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-wgrad_ab}
mkdir -p $OUT
for round in 1 2; do
  for op in wgrad_pre wgrad_nhwc; do
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_${op}_$round -o p -- python3 tools/kbench.py $op 20 > $OUT/${op}_$round.log 2>&1 || { echo "kbench $op failed"; tail -5 $OUT/${op}_$round.log; exit 1; }
    CSV=$(find $OUT/kt_${op}_$round -name '*kernel_stats.csv' | head -1)
    echo "== round $round $op" >> $OUT/wgrad_ab.txt
    grep -E "wgrad|reduce_store" "$CSV" | cut -d, -f1-8 >> $OUT/wgrad_ab.txt
  done
done
cat $OUT/wgrad_ab.txt
