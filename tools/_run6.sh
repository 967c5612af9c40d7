# PMC traffic of the dominant kernel, full GPU test suite, bench, kernel-trace profile of the bench.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/${TAG:-r1i}; mkdir -p $OUT
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_f -o p -- python3 tools/kbench.py fprop 5 > $OUT/pmc_f.log 2>&1 || { echo pmc fetch failed; tail -5 $OUT/pmc_f.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_w -o p -- python3 tools/kbench.py fprop 5 > $OUT/pmc_w.log 2>&1 || { echo pmc write failed; tail -5 $OUT/pmc_w.log; exit 1; }
python3 tools/pmc_conv.py $OUT/pmc_f $OUT/pmc_w $OUT/r01_conv_fprop_pmc.json || exit 1
mkdir -p profiles && cp $OUT/r01_conv_fprop_pmc.json profiles/
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -5 $OUT/pytest.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error" $OUT/pytest.log | head; exit 1; fi
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o prof -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > $OUT/prof.log 2>&1 || { echo prof failed; tail -20 $OUT/prof.log; exit 1; }
echo done
