cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/${TAG:-r1d}; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -30 $OUT/pytest.log | grep -E "passed|failed|FAILED|Error|assert" | head -30
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit 1; fi
for m in bf16x3 bf16x6; do
  TILES=auto VST_CONV_MATH=$m timeout -k 10 200 python -u tools/convbench.py > $OUT/convbench_$m.log 2>&1 || { echo convbench failed; tail $OUT/convbench_$m.log; exit 1; }
  grep layer $OUT/convbench_$m.log
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
if [ -n "$PROF" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o prof -- python3 bench.py --steps 7 --warmup 3 --no-cpu-baseline --no-extras > $OUT/prof.log 2>&1 || { echo prof failed; tail -20 $OUT/prof.log; exit 1; }
fi
echo done
