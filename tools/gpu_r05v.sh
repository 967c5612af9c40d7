#!/bin/bash
# VGG data gradients on the dgrad-as-forward kernel: style / VGG / C3 / Johnson GPU tests, then a same-box A/B
# (VST_VGG_DGRAD_FPROP) of the Johnson and C3 steps, 2 rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05v}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_style.py tests/test_gpu_c3.py tests/test_gpu_fullsize.py -k "style or vgg or VGG or c3 or johnson or Johnson or perceptual or gram" > $O/t.log 2>&1 || { echo tests failed; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 1 2; do
  for arm in default ${ARM2:-VST_VGG_DGRAD_FPROP=0}; do
    if [ "$arm" = default ]; then envs=""; else envs="$arm"; fi
    env $envs timeout -k 10 300 python3 tools/vggbench.py > $O/v_${arm}_$r.log 2>&1 || { echo "vggbench $arm failed"; tail -5 $O/v_${arm}_$r.log; exit 1; }
    tail -1 $O/v_${arm}_$r.log
  done
done
exit 0
