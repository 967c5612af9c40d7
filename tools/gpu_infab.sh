#!/bin/bash
# Same-box inference A/B: tools/infbench.py (B=1 256x256, per-call synchronised median) under each setting in
# $ARMS (space-separated NAME=VALUE[,NAME=VALUE] or "default"), three interleaved rounds; B=16 once per arm.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-infab}
mkdir -p $OUT
for round in 1 2 3; do
  for arm in $ARMS; do
    if [ "$arm" = default ]; then envs=""; else envs="${arm//,/ }"; fi
    r=$(env $envs timeout -k 10 120 python3 tools/infbench.py 1 256 256 200 2> $OUT/err.log) || { echo "arm $arm failed"; tail -5 $OUT/err.log; exit 1; }
    echo "{\"round\": $round, \"arm\": \"$arm\", \"b1\": \"$r\"}" | tee -a $OUT/infab.jsonl
    if [ $round = 1 ]; then
      r=$(env $envs timeout -k 10 120 python3 tools/infbench.py 16 256 256 20 2> $OUT/err.log) || { echo "arm $arm failed"; exit 1; }
      echo "{\"round\": $round, \"arm\": \"$arm\", \"b16\": \"$r\"}" | tee -a $OUT/infab.jsonl
    fi
  done
done
