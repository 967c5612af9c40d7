#!/bin/bash
# Same-box step A/B: bench.py (no extras, no CPU leg) under each environment setting in $ARMS
# (space-separated NAME=VALUE or "default"), two interleaved rounds.  usage: ARMS="default VST_C4_DIRECT=0" tools/ab_step.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab_step}
mkdir -p $OUT
for round in 1 2; do
  for arm in $ARMS; do
    if [ "$arm" = default ]; then envs=""; else envs="${arm//,/ }"; fi
    env $envs timeout -k 10 300 python -u bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --no-extras > $OUT/b.json 2> $OUT/b.err || { echo "arm $arm failed"; tail -5 $OUT/b.err; exit 1; }
    ms=$(grep -o '"ms_per_step": [0-9.]*' $OUT/b.json | head -1)
    echo "{\"round\": $round, \"arm\": \"$arm\", $ms}" | tee -a $OUT/ab.jsonl
  done
done
