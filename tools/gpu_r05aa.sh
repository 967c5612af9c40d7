#!/bin/bash
# RAFT SepConvGRU split-K: RAFT / MoGAN / Sintel GPU tests, then a same-box A/B (VST_FWD_HW_SPLITK), 2 rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05aa; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_raft.py tests/test_gpu_mogan.py tests/test_gpu_sintel.py tests/test_gpu_fullsize.py -k "raft or RAFT or mogan or sintel or corr" > $O/t.log 2>&1 || { echo tests failed; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 1 2; do
  for arm in default VST_FWD_HW_SPLITK=0 VST_RAFT_CS8=0; do
    if [ "$arm" = default ]; then envs=""; else envs="$arm"; fi
    env $envs timeout -k 10 300 python3 tools/raftbench.py > $O/r_${arm}_$r.log 2>&1 || { echo "raftbench $arm failed"; tail -5 $O/r_${arm}_$r.log; exit 1; }
    tail -1 $O/r_${arm}_$r.log
  done
done
exit 0
