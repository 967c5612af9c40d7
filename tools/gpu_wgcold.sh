#!/bin/bash
# The in-step vs isolated weight-gradient gap: kernel traces of tools/kbench.py wgrad_pre / fprop at N=8 with
# warm operands (repeat calls: x image and dy planes MALL-resident), KB_FLUSH=1 (all cold) and KB_FLUSH=2 (dy
# planes re-made just before, x cold: the step's state).  Per-kernel averages into gpurun_out/$TAG/wgcold.txt.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-wgcold}
mkdir -p $OUT
: > $OUT/wgcold.txt
for op in wgrad_pre fprop; do
  for fl in 0 1 2; do
    [ $op = fprop ] && [ $fl = 2 ] && continue
    if [ $fl = 0 ]; then envs=""; else envs="KB_FLUSH=$fl"; fi
    d=$OUT/${op}_f$fl
    env $envs VST_CONV_MATH=bf16x6 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o p -- python3 tools/kbench.py $op 20 > $d.log 2>&1 || { echo "kt fail $op $fl"; tail -5 $d.log; exit 1; }
    CSV=$(find $d -name '*kernel_trace.csv' | head -1)
    echo "== $op KB_FLUSH=$fl" >> $OUT/wgcold.txt
    python3 tools/profsum.py "$CSV" 20 6 >> $OUT/wgcold.txt
  done
done
cut -c1-170 $OUT/wgcold.txt
