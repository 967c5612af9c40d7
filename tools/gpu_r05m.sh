#!/bin/bash
# Round-5: inference A/B of the pre-split A operands (B=1 / B=16, tools/gpu_infab.sh), the 256x64 image-layer weight
# gradient tile (VST_WG_K256=1) on the per-layer table + its op tests, and the full-size parity logs (per-parameter
# HIP / own-fp32 deviation ratios, tools/parity_ratios.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05m}
mkdir -p $O
VST_APRE=1 TAG=${TAG:-r05m}/trace_apre bash tools/gpu_trace.sh > /dev/null || exit 1
head -24 $O/trace_apre/step_summary.txt | cut -c1-60,100-175
ARMS="default VST_APRE=1" TAG=${TAG:-r05m}/infab bash tools/gpu_infab.sh > /dev/null || exit 1
cat $O/infab/infab.jsonl | tr -d '\n' | sed 's/}/}\n/g' | grep -o '"arm": "[^"]*", "b[0-9]*": "[^"]*"' | sed 's/initialize network with normal//'
VST_WG_K256=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "wgrad or tap" > $O/t_k256.log 2>&1 || { echo k256 tests failed; tail -30 $O/t_k256.log; exit 1; }
tail -1 $O/t_k256.log
for arm in default VST_WG_K256=1; do
  if [ "$arm" = default ]; then envs=""; else envs="$arm"; fi
  env $envs timeout -k 10 240 python -u tools/layertable.py 3 2> $O/lt.err | grep '^{' > $O/lt_$arm.jsonl || { echo "layertable $arm failed"; tail -20 $O/lt.err; exit 1; }
  echo "$arm"; grep -E "7x7 s1 3->64|wgrad_swap" $O/lt_$arm.jsonl | cut -c1-140
done
VST_PARITY_LOG=$O/parity timeout -k 10 500 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullsize.py > $O/t_full.log 2>&1
rc=$?
tail -1 $O/t_full.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 1; fi
python3 tools/parity_ratios.py $O/parity 10
exit 0
