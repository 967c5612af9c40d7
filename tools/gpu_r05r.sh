#!/bin/bash
# StarGAN tests + C4 timing on the current sources, then the round-5 PMC passes (tools/gpu_r05z_pmc.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05r; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests -k "stargan" > $O/t_sg.log 2>&1 || { echo sg tests failed; tail -30 $O/t_sg.log; exit 1; }
tail -1 $O/t_sg.log
timeout -k 10 200 python3 tools/sgbench.py > $O/sg.log 2>&1 || { echo sgbench failed; tail -5 $O/sg.log; exit 1; }
tail -1 $O/sg.log | grep -o '"ms_per_d_iteration": [0-9.]*'
bash tools/gpu_r05z_pmc.sh || exit 1
exit 0
