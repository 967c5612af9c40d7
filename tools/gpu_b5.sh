#!/bin/bash
# K-restricted border GEMM (REFL 5) check: parity tests, per-kernel times of the dgrad op under each
# border setting (rocprofv3 kernel stats of kbench.py dgrad), then the same-box step A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/b5
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "dgrad_refl_in_fused or dgrad_reflect_border or production_resnet" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/pytest.log | head -20; exit $rc; }
for arm in "VST_BORDER5=1" "VST_BORDER5=0" "VST_BORDER_KS=3" "VST_BORDER_KS=8" "VST_BORDER_KS=12"; do
  tag=$(echo $arm | tr '=' '_')
  export $arm
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- python3 tools/kbench.py dgrad 20 > $O/$tag.log 2>&1 || { echo "prof $arm failed"; tail -5 $O/$tag.log; exit 1; }
  unset VST_BORDER5 VST_BORDER_KS
  f=$(find $O/$tag -name "*kernel_stats.csv" | head -1)
  echo "== $arm"; grep -E "border|conv_fprop|reduce" "$f" | cut -d, -f1-4 | cut -c1-200
done
ARMS="default VST_BORDER5=0" TAG=b5 bash tools/ab_step.sh
