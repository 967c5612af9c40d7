cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/${TAG:-r1e}; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -30 $OUT/pytest.log | grep -E "passed|failed|FAILED|Error|assert" | head -30
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit 1; fi
for m in bf16x3 bf16x6; do
  LAYERS=res,d128,d256,D4 VST_CONV_MATH=$m timeout -k 10 200 python -u tools/convbench.py > $OUT/convbench_$m.log 2>&1 || { echo convbench failed; tail $OUT/convbench_$m.log; exit 1; }
done
echo done
