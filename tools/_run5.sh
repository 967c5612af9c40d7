cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/${TAG:-r1g}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_style.py} -k "${K:-}" -m gpu -v -x --timeout 180 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert|passed|failed" $OUT/pytest.log | tail -40
exit $rc
