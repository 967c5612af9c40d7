#!/bin/bash
# Batched VGG forwards (Johnson / C3) and the StarGAN D step's no-grad fake generation: their GPU tests, then
# same-box A/Bs (VST_VGG_BATCHED, VST_SG_DIRECT).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05cc; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests -k "style or vgg or VGG or c3 or johnson or Johnson or perceptual or gram or stargan" > $O/t.log 2>&1 || { echo tests failed; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 1 2; do
  for arm in default VST_VGG_BATCHED=0; do
    if [ "$arm" = default ]; then envs=""; else envs="$arm"; fi
    env $envs timeout -k 10 300 python3 tools/vggbench.py > $O/v_${arm}_$r.log 2>&1 || { echo "vggbench $arm failed"; tail -5 $O/v_${arm}_$r.log; exit 1; }
    echo "$arm $(tail -1 $O/v_${arm}_$r.log)"
  done
done
TAG=r05cc/sg_new bash tools/gpu_sgtrace.sh > /dev/null || exit 1
true
head -1 $O/sg_new/sg_summary.txt
exit 0
