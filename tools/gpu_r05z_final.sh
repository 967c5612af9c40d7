#!/bin/bash
# Round-5 final measurement set (one, after the last kernel change): the whole GPU suite, smoke(), the step and
# inference kernel traces, the bench line.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r05z
bash tools/gpu_call.sh \
  "timeout -k 10 700 python3 -u -m pytest -q --timeout 280 --timeout-method thread tests -m gpu -p no:cacheprovider > gpurun_out/r05z/t.log 2>&1; rc=\$?; tail -3 gpurun_out/r05z/t.log; exit \$rc" \
  "timeout -k 10 300 python3 -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "TAG=r05z_trace bash tools/gpu_trace.sh > /dev/null" \
  "TAG=r05z_inf bash tools/gpu_inftrace.sh > /dev/null" \
  "timeout -k 10 500 python3 bench.py > gpurun_out/r05z/bench.json 2> gpurun_out/r05z/bench.err; rc=\$?; tail -c 400 gpurun_out/r05z/bench.json; exit \$rc"
