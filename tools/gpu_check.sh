#!/bin/bash
# Round GPU check: parity tests, bench, conv microbench, rocprofv3 kernel-trace of the train step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-run}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
if [ -n "$CONVBENCH" ]; then
  for m in bf16x3 fp32; do
    VST_CONV_MATH=$m timeout -k 10 200 python -u tools/convbench.py > $OUT/convbench_$m.log 2>&1 || { echo convbench failed; tail $OUT/convbench_$m.log; exit 1; }
  done
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o prof -- python3 bench.py --steps 7 --warmup 3 --no-cpu-baseline --no-extras > $OUT/prof.log 2>&1 || { echo prof failed; tail -20 $OUT/prof.log; exit 1; }
echo done
