#!/bin/bash
# Round-3 GPU check: the new parity tests first, then the whole GPU suite, the default bench line and
# the single-GPU runs of the DP workloads (c4 StarGAN, c5 MoGAN at 1024x436).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03a}
mkdir -p $OUT
PYT="python -u -m pytest -x -v --timeout 900 --timeout-method thread"
timeout -k 10 900 ${PYT/ -x/} -m gpu tests/test_gpu_abi.py tests/test_gpu_dp.py tests/test_library_ops.py tests/test_gpu_fullsize.py > $OUT/pytest_new.log 2>&1 || { echo "new tests failed"; tail -40 $OUT/pytest_new.log; exit 1; }
tail -3 $OUT/pytest_new.log
if [ -n "$FULL" ]; then
  timeout -k 10 900 $PYT -m gpu tests > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
  tail -3 $OUT/pytest.log
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
  timeout -k 10 200 python -u bench.py --workload c4 --steps 20 --warmup 5 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { echo c4 failed; tail -20 $OUT/bench_c4.err; exit 1; }
  cat $OUT/bench_c4.json
  timeout -k 10 300 python -u bench.py --workload c5 --steps 6 --warmup 2 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { echo c5 failed; tail -20 $OUT/bench_c5.err; exit 1; }
  cat $OUT/bench_c5.json
fi
echo done
