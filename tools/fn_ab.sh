#!/bin/bash
# Same-box A/B of one bench.py line function (FN, e.g. c3_train_fps, sintel_inference_fps, stargan_train_fps) over
# environment arms: ARMS="default VST_LIB_VARIANT=..." two interleaved rounds -> gpurun_out/$TAG/fn_ab.jsonl
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-fnab}
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
d = bench.$FN(torch.device('cuda:0'))
keep = {k: d[k] for k in ('value', 'ms_per_step', 'ms_per_frame', 'ms_per_d_iteration') if k in d}
keep['frac'] = d.get('roofline', {}).get('frac')
print(json.dumps(dict(round=$r, arm='$arm', fn='$FN', **keep)))
" >> $OUT/fn_ab.jsonl 2>> $OUT/fn_ab.err || { echo "arm $arm failed"; tail -5 $OUT/fn_ab.err; exit 1; }
  done
done
cat $OUT/fn_ab.jsonl
