# Parity tests, then the train-step bench without extras / CPU baseline -> gpurun_out/$TAG/
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/${TAG:-quick}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'],d['ms_per_step'])"
