#!/bin/bash
# Same-box A/B of the StarGAN direct D-gradient accumulation / frozen D in the G step (VST_SG_DIRECT), 3 rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05t; mkdir -p $O
for r in 1 2 3; do
  for arm in default VST_SG_DIRECT=0; do
    if [ "$arm" = default ]; then envs=""; else envs="$arm"; fi
    env $envs timeout -k 10 200 python3 tools/sgbench.py > $O/sg_${arm}_$r.log 2>&1 || { echo "sgbench $arm failed"; tail -5 $O/sg_${arm}_$r.log; exit 1; }
    echo "$arm $(tail -1 $O/sg_${arm}_$r.log | grep -o '"ms_per_d_iteration": [0-9.]*')"
  done
done
exit 0
