#!/bin/bash
# Round-5 developer variants: the A operand by LDS-DMA (lib_adma: VST_BF_FAKE_ADMA, timing only) on the ResnetBlock
# GEMMs (tools/kbench_time.py, relu'd activations), and the weight gradient's dy planes by LDS-DMA (lib_glw:
# VST_BF_GLDS_W=1) on the per-layer table (the image-layer weight gradients).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05k}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests/test_gpu_ops.py tests/test_gpu_stargan.py tests/test_gpu_fullsize.py -k "skinny_split or conv4s2 or stargan" > $O/t.log 2>&1 || { echo tests failed; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for arm in default VST_SG_PHASES=0; do
  if [ "$arm" = default ]; then envs=""; else envs="$arm"; fi
  env $envs timeout -k 10 200 python3 tools/sgbench.py > $O/sg_$arm.log 2>&1 || { echo "sgbench $arm failed"; tail -5 $O/sg_$arm.log; exit 1; }
  echo "$arm $(tail -1 $O/sg_$arm.log | grep -o '"ms_per_d_iteration": [0-9.]*')"
done
TAG=${TAG:-r05k}/sg bash tools/gpu_sgtrace.sh > /dev/null || exit 1
head -16 $O/sg/sg_summary.txt | cut -c1-170
KB_RELU=1 VARIANTS="adma" TAG=${TAG:-r05k}/adma bash tools/ab_variants.sh || exit 1
for v in default glw; do
  if [ $v = default ]; then unset VST_LIB_VARIANT; else export VST_LIB_VARIANT=gan-based-video-style-transfer_amd/_build/variants/lib_$v.so; fi
  timeout -k 10 240 python -u tools/layertable.py 3 2> $O/lt_$v.err | grep '^{' > $O/lt_$v.jsonl || { echo "layertable $v failed"; tail -20 $O/lt_$v.err; exit 1; }
  grep -E "7x7|wgrad" $O/lt_$v.jsonl | cut -c1-150
done
unset VST_LIB_VARIANT
TAG=${TAG:-r05k}/dvfs bash tools/gpu_dvfs.sh > /dev/null || exit 1
exit 0
