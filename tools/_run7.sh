cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/${TAG:-r1j}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_models.py tests/test_gpu_style.py -m gpu -q -x --timeout 180 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $OUT/pytest.log | head -20; exit 1; fi
TILES=auto LAYERS=res,D4 VST_CONV_MATH=bf16x3 timeout -k 10 200 python -u tools/convbench.py > $OUT/convbench.log 2>&1 || { tail $OUT/convbench.log; exit 1; }
grep layer $OUT/convbench.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
