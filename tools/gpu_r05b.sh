#!/bin/bash
# Round-5: the PatchGAN head row kernels (patch.hip): their parity tests + the conv / model tests that
# reach the head, the per-layer table, then the same-box step A/B against VST_HEAD=0.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05b}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_patch.py tests/test_gpu_ops.py tests/test_gpu_models.py tests/test_gpu_train.py > $O/t.log 2>&1 || { echo tests failed; tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 240 python -u tools/layertable.py 3 2> $O/layertable.err | grep '^{' > $O/layertable.jsonl || { echo layertable failed; tail -20 $O/layertable.err; exit 1; }
tail -1 $O/layertable.jsonl
ARMS="${ARMS:-default VST_HEAD=0}" TAG=${TAG:-r05b}/ab bash tools/ab_step.sh
