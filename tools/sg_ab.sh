#!/bin/bash
# Same-box A/B of the StarGAN C4 line (bench.stargan_train_fps, 6 n_critic cycles) over route settings:
# ARMS="default VST_ROUTES=ops.X=0" (each arm an environment assignment or "default"), two rounds,
# -> gpurun_out/$TAG/sg_ab.jsonl
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-sgab}
mkdir -p $OUT
for r in 1 2; do
  for arm in $ARMS; do
    if [ "$arm" = default ]; then envs=""; else envs="$arm"; fi
    env $envs timeout -k 10 300 python3 -c "
import json, sys, torch
sys.path.insert(0, '.')
import bench, gbvst
gbvst._lib.load()
from gbvst import ops
ops.set_conv_math('bf16x6')
d = bench.stargan_train_fps(torch.device('cuda:0'), cycles=6)
print(json.dumps({'round': $r, 'arm': '$arm', 'ms_per_d_iteration': d['ms_per_d_iteration'], 'frac': d['roofline']['frac']}))
" >> $OUT/sg_ab.jsonl 2>> $OUT/sg_ab.err || { echo "arm $arm failed"; tail -5 $OUT/sg_ab.err; exit 1; }
  done
done
cat $OUT/sg_ab.jsonl
