#!/bin/bash
# Round-5 batch: StarGAN routes (phase data gradients, GP input-only pass, split skinny heads) — their tests and
# the full-size iteration vs the oracle, StarGAN per-arm timing + trace; the ConvTranspose tile rule and the
# prefetching epi epilogue — op tests, per-layer table, step A/B ($ARMS).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05j}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests/test_gpu_ops.py tests/test_gpu_stargan.py tests/test_gpu_fullsize.py -k "skinny_split or convT or conv4s2 or dgrad_refl_in or stargan or one_real_channel" > $O/t.log 2>&1 || { echo tests failed; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for arm in default VST_SG_PHASES=0 VST_SKINNY_SPLIT=0; do
  if [ "$arm" = default ]; then envs=""; else envs="$arm"; fi
  env $envs timeout -k 10 200 python3 tools/sgbench.py > $O/sg_$arm.log 2>&1 || { echo "sgbench $arm failed"; tail -5 $O/sg_$arm.log; exit 1; }
  echo "$arm $(tail -1 $O/sg_$arm.log | grep -o '"ms_per_d_iteration": [0-9.]*')"
done
TAG=${TAG:-r05j}/sg bash tools/gpu_sgtrace.sh > /dev/null || exit 1
head -16 $O/sg/sg_summary.txt | cut -c1-170
timeout -k 10 240 python -u tools/layertable.py 3 2> $O/layertable.err | grep '^{' > $O/layertable.jsonl || { echo layertable failed; tail -20 $O/layertable.err; exit 1; }
tail -1 $O/layertable.jsonl
[ -n "$ARMS" ] && TAG=${TAG:-r05j}/ab bash tools/ab_step.sh
exit 0
