#!/bin/bash
# Round-4 GPU check of the swapped last-layer weight gradient: its parity tests and the tap / generator /
# step tests around it, the two forms' kernel split (rocprofv3), then the same-box step A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04sw
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "tap or instnorm" > $O/t_ops.log 2>&1 || { echo ops tests failed; tail -30 $O/t_ops.log; exit 1; }
tail -2 $O/t_ops.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_train.py > $O/t_train.log 2>&1 || { echo train tests failed; tail -30 $O/t_train.log; exit 1; }
tail -2 $O/t_train.log
timeout -k 10 240 python3 -u tools/proto_wg_swap.py > $O/proto.log 2>&1 || { echo proto failed; tail -5 $O/proto.log; exit 1; }
cat $O/proto.log
KB_REPS=5 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/proto_wg_swap.py > $O/prof.log 2>&1 || { echo prof failed; tail -5 $O/prof.log; exit 1; }
ARMS="default VST_TAP_SWAP=0" TAG=r04sw/ab bash tools/ab_step.sh
