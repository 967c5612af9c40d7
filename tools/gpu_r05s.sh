#!/bin/bash
# StarGAN: every stargan GPU test (golden, full-size iteration vs oracle, DP) + two C4 timings.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05s}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests -k "stargan or StarGAN" > $O/t_sg.log 2>&1 || { echo sg tests failed; tail -30 $O/t_sg.log; exit 1; }
tail -1 $O/t_sg.log
for r in 1 2; do
  timeout -k 10 200 python3 tools/sgbench.py > $O/sg$r.log 2>&1 || { echo sgbench failed; tail -5 $O/sg$r.log; exit 1; }
  tail -2 $O/sg$r.log | head -1
  tail -1 $O/sg$r.log | grep -o '"ms_per_d_iteration": [0-9.]*'
done
exit 0
