#!/bin/bash
# Border GEMM K-split sweep (kernel stats), dgrad PMC record, and the fused border+IN route A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/b5b
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "convT_phases or conv_transpose" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/pytest.log | head -20; exit $rc; }
for arm in "VST_BORDER5=1" "VST_BORDER5=0" "VST_BORDER_KS=2" "VST_BORDER_KS=3" "VST_BORDER_KS=8" "VST_BORDER_KS=12"; do
  tag=$(echo $arm | tr '=' '_')
  export $arm
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- python3 tools/kbench.py dgrad 20 > $O/$tag.log 2>&1 || { echo "prof $arm failed"; tail -5 $O/$tag.log; exit 1; }
  unset VST_BORDER5 VST_BORDER_KS
  f=$(find $O/$tag -name "*kernel_stats.csv" | head -1)
  echo "== $arm"; grep -E "border|conv_fprop|reduce" "$f" | cut -d, -f1-4 | cut -c1-220
done
OPS="dgrad" TAG=pmc_r03d bash tools/profile_counters.sh && python3 tools/pmc_resblock.py gpurun_out/pmc_r03d gpurun_out/pmc_r03d/r03d 5 || exit 1
ARMS="default VST_DGRAD_IN=1 VST_CONVT_GROUPED=0" TAG=b5b STEPS=20 bash tools/ab_step.sh
