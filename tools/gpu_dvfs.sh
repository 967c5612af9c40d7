#!/bin/bash
# Operand-data dependence of the x6 GEMM times (DVFS): kernel traces of tools/kbench.py fprop / wgrad_pre / dgrad at
# N=8 with randn operands vs KB_RELU=1 (half-zero activations, as in the step).  Summary in gpurun_out/$TAG/dvfs.txt.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-dvfs}
mkdir -p $OUT
: > $OUT/dvfs.txt
for op in fprop wgrad_pre dgrad; do
  for rl in 0 1; do
    d=$OUT/${op}_r$rl
    KB_RELU=$rl VST_CONV_MATH=bf16x6 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o p -- python3 tools/kbench.py $op 20 > $d.log 2>&1 || { echo "kt fail $op $rl"; tail -5 $d.log; exit 1; }
    CSV=$(find $d -name '*kernel_trace.csv' | head -1)
    echo "== $op KB_RELU=$rl" >> $OUT/dvfs.txt
    python3 tools/profsum.py "$CSV" 20 3 >> $OUT/dvfs.txt
  done
done
cut -c1-170 $OUT/dvfs.txt
